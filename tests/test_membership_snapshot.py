"""Membership carried by snapshots (cfg.membership with cfg.snapshot_entries)
on the CPU tier: the device step compiled for the host (tests/soa_cpu) against
the oracle harness, round by round — every view field (each replica's voter
set included), the trace digest and the snapshot state, which now also holds
the snapshot's membership and the state machine's.

Covered (reference):
  * a node snapshot records the state machine's membership at its index
    (pb.Snapshot.Membership, raft.pb.go:733-739; rsm membership applied with
    each ConfigChange);
  * InstallSnapshot carries it (makeInstallSnapshotMessage, raft.go:684-697);
    the receiver restores the log (raft.go:439-470), its state machine
    recovers from the snapshot, and the node calls Peer.RestoreRemotes at the
    next step (rsm/statemachine.go:236, node.go:241-264, peer.go:159-165) →
    Handle(SnapshotReceived) → restoreRemotes (raft.go:472-517, 1566, the
    SnapshotReceived row of every role, 2049-2097): voters replaced, remotes
    reset, a leader the snapshot does not list steps down;
  * a node restarted over a LogDB with a snapshot reads its voters from it
    (logdb NodeState, raft.go:260-270);
  * the host's own Peer.RestoreRemotes (rbe_restore_remotes).
The remove / re-add schedule (cc_period) and isolations push removed and
isolated replicas behind the leaders' compaction markers, so they come back by
InstallSnapshot with a membership that differs from theirs."""
import random

import pytest

import oracle as O
from parity_util import C2, C3_HOT, MIXED, counters_match, view_diff
from soa_cpu.soa import SoaCpu
from test_membership import CATCHUP, MEMB

SNAP = dict(snapshot_entries=8, compaction_overhead=2)
CASES = {
    "C2": (dict(C2, n_groups=24, **MEMB, **SNAP), CATCHUP, 400),
    "C3_HOT": (dict(C3_HOT, n_groups=24, **MEMB, **SNAP), CATCHUP, 400),
    "MIXED": (dict(MIXED, **MEMB, snapshot_entries=10, compaction_overhead=0),
              dict(CATCHUP), 400),
    "C3_HOT_N7": (dict(C3_HOT, n_groups=16, n_replicas=7, **MEMB, **SNAP), CATCHUP, 400),
}


def run_memb_snap(eng, ref, rounds, skip=()):
    """Lockstep with the snapshot state compared every round.  Returns the
    number of restores of a snapshot whose membership differs from the
    restoring replica's voters, and of snapshots taken with a non-trivial
    membership."""
    restored_diff, snap_rem = 0, 0
    prev = ref.views()
    for rnd in range(rounds):
        eng.run(1)
        ref.run(1)
        ev, hv = eng.views(), ref.views()
        for i in range(len(hv)):
            d = view_diff(ev[i], hv[i], skip)
            assert d is None, f"round {rnd + 1} replica {i}: {d}"
        es = eng.snapshot_state()
        for i in range(len(hv)):
            os_ = ref.snapshot_state(i)
            assert tuple(es[i]) == os_, f"round {rnd + 1} replica {i}: {tuple(es[i])} != {os_}"
            if os_[6]:
                snap_rem += 1
            # a snapshot restored this round whose membership is not the view's
            if os_[2] > os_[4] and hv[i].processed == os_[2] and prev[i].processed < os_[2]:
                if os_[6] != (prev[i].removed & 0x1F):
                    restored_diff += 1
        prev = hv
    return restored_diff, snap_rem


@pytest.mark.parametrize("mode", ["pipeline", "full_table"])
@pytest.mark.parametrize("name", list(CASES))
def test_membership_snapshot_parity(name, mode):
    kw, extra, rounds = CASES[name]
    eng = SoaCpu(trace=True, full_only=mode == "full_table", **kw, **extra)
    ref = O.Harness(**kw)
    diff, snap_rem = run_memb_snap(eng, ref, rounds)
    n, bits = eng.faults()
    assert n == 0, f"faults {bits:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    assert snap_rem > 0, "no snapshot ever recorded a removed voter"
    assert diff > 0, "no replica restored a snapshot with a membership other than its own"


@pytest.mark.parametrize("name", ["C2", "C3_HOT", "MIXED", "C3_HOT_N7"])
def test_membership_snapshot_untraced(name):
    """The bench paths (untraced: lazy quiesced ticks, group sleep)."""
    kw, extra, rounds = CASES[name]
    eng = SoaCpu(trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, rounds, skip=("digest",))
    assert eng.faults()[0] == 0


def test_restart_over_snapshot_membership():
    """rbe_launch over a LogDB whose snapshot lists fewer voters: the restarted
    raft takes them (NodeState), the state machine too."""
    from launch_util import restart
    kw, extra, _ = CASES["C2"]
    eng = SoaCpu(trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, 150)
    picks = [i for i in range(eng.n_rep) if ref.snapshot_state(i)[6]]
    assert picks, "no snapshot with a removed voter to restart from"
    restart(eng, ref, picks[:12], None, snapshots=True)  # the whole LogDB above the marker
    run_memb_snap(eng, ref, 150)
    assert eng.faults()[0] == 0


def host_restore_schedule(eng, ref, rounds, seed=7):
    """Peer.RestoreRemotes from the host (rbe_restore_remotes / PUSH_RESTORE) on
    random replicas with random voter sets; both sides driven identically."""
    rng = random.Random(seed)
    n = ref.n_replicas
    calls = 0
    for rnd in range(rounds):
        if rnd >= 30:
            for r in range(eng.n_rep):
                if rng.random() < 0.02:
                    voters = sorted(rng.sample(range(1, n + 1), rng.randrange(1, n + 1)))
                    rem = sum(1 << (v - 1) for v in range(1, n + 1) if v not in voters)
                    eng.restore_remotes([r], [voters])
                    ref.push(O.PUSH_RESTORE, r, rem)
                    calls += 1
        eng.run(1)
        ref.run(1)
        ev, hv = eng.views(), ref.views()
        for i in range(len(hv)):
            d = view_diff(ev[i], hv[i])
            assert d is None, f"round {rnd + 1} replica {i}: {d}"
    return calls


def test_host_restore_remotes():
    kw = dict(C2, n_groups=8, ext_inputs=True, membership=True)
    eng = SoaCpu(trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    assert host_restore_schedule(eng, ref, 150) > 10
    assert eng.faults()[0] == 0


def test_restore_remotes_checks():
    from dragonboat_amd.engine import InputError, RBE_E_INVALID, RBE_E_STATE
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError) as ei:  # needs cfg.membership
        eng.restore_remotes([0], [[1, 2, 3]])
    assert ei.value.rc == RBE_E_STATE
    m = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True, membership=True)
    for bad in ([[1, 4]], [[2, 2]], [[0]]):  # node outside the group, repeated, NoNode
        with pytest.raises(InputError) as ei:
            m.restore_remotes([0], bad)
        assert ei.value.rc == RBE_E_INVALID
    m.restore_remotes([0], [[1, 3]])
    with pytest.raises(InputError) as ei:  # one per replica per step
        m.restore_remotes([0], [[1]])
    assert ei.value.rc == RBE_E_STATE
