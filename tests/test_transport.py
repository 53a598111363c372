"""The Peer.Handle boundary (rbe_get_outbox / rbe_push_messages) on the CPU
tier: W host builds of the device step (tests/soa_cpu), each stepping the
replicas it owns, exchange every cross-engine message through the raftpb-form
transport API; every owned replica must equal the oracle stepping all replicas
in one process.  test_gpu_transport.py runs the same loop on the HIP engine."""
import pytest

import oracle as O
from soa_cpu.soa import SoaCpu
from transport_util import run_transport

CASES = {
    # steady replication, 3 replicas over 2 engines
    "C2_w2": (dict(n_groups=12, n_replicas=3, wl_enabled=True, wl_start_round=30), 2, 120, {}),
    # quiesce + 9:1 reads, every replica of a group on its own engine
    "C4_w3": (dict(n_groups=12, n_replicas=3, quiesce=True, wl_enabled=True, wl_start_round=30,
                   wl_active_mod=2, wl_read_permille=900), 3, 300, {}),
    # 5 replicas, check-quorum, elections from scratch, quiesce and reads over 4 engines
    # (no isolation schedule: k_isolate reads the roles of every replica of a group,
    # which an engine stepping only some of them does not have)
    "N5_w4": (dict(n_groups=8, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
                   wl_start_round=25, wl_active_mod=2, wl_read_permille=500, seed=777), 4, 300,
              dict()),
    # the isolation schedule with every replica of a group on another engine
    "C3_iso_w3": (dict(n_groups=12, n_replicas=5, check_quorum=True, wl_enabled=True,
                       wl_start_round=40, iso_period=50, iso_len=30, iso_mod=3), 3, 250,
                  dict()),
}


@pytest.mark.parametrize("name", list(CASES))
def test_transport_parity_cpu(name):
    kw, world, rounds, extra = CASES[name]
    engs = [SoaCpu(trace=True, rep_world=world, rep_rank=r, **kw, **extra) for r in range(world)]
    ref = O.Harness(**kw)
    d, moved = run_transport(engs, ref, kw["n_replicas"], rounds)
    assert d is None, f"{name}: first divergence {d}"
    assert moved > rounds, "the transport carried (almost) nothing"
    for e in engs:
        assert e.faults()[0] == 0


def test_push_rejects_bad_batches():
    from dragonboat_amd.engine import RbeEntry, RbeMessage
    kw = dict(n_groups=4, n_replicas=3, wl_enabled=True, wl_start_round=5)
    e = SoaCpu(trace=True, rep_world=2, rep_rank=0, **kw)
    e.step()
    m = RbeMessage(type=16, to=1, from_=2, term=1)  # Heartbeat 2 -> 1 in group 0
    # group 0: replica 0 (node 1) is owned by rank 0, node 2 by rank 1: a valid hop
    e.push_messages([0], [m], [])
    with pytest.raises(RuntimeError):  # sender stepped by this engine (node 1 of group 0)
        e.push_messages([0], [RbeMessage(type=16, to=2, from_=1, term=1)], [])
    with pytest.raises(RuntimeError):  # group out of range
        e.push_messages([9], [m], [])
    with pytest.raises(RuntimeError):  # entry index does not follow LogIndex
        rep = RbeMessage(type=12, to=1, from_=2, term=1, log_index=3, n_entries=1)
        e.push_messages([0], [rep], [RbeEntry(index=9, term=1)])
    one = SoaCpu(trace=True, **kw)
    one.step()
    with pytest.raises(RuntimeError):  # rep_world 1: every sender is local
        one.push_messages([0], [m], [])


def test_push_filters_like_peer_handle():
    """Peer.Handle (peer.go:186-198): a local message type is refused (the
    reference panics), a response from a node outside the group is dropped,
    and the rest of the batch is delivered."""
    from dragonboat_amd.engine import RbeMessage
    kw = dict(n_groups=4, n_replicas=3, wl_enabled=True, wl_start_round=5)
    e = SoaCpu(trace=True, rep_world=2, rep_rank=0, **kw)
    e.step()
    for local in (1, 2, 8, 9, 10, 0, 11):  # Election ... BatchedReadIndex (entryutils.go:97-104)
        with pytest.raises(RuntimeError):
            e.push_messages([0], [RbeMessage(type=local, to=1, from_=2, term=1)], [])
    # a HeartbeatResp from node 7, not a member of a 3-node group: dropped
    e.push_messages([0], [RbeMessage(type=18, to=1, from_=7, term=1)], [])
    # a RequestVote from a non-member cannot be represented: refused
    with pytest.raises(RuntimeError):
        e.push_messages([0], [RbeMessage(type=14, to=1, from_=7, term=9)], [])
