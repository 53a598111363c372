"""Inbound frames straight into the inbox planes (rbe_wire_ingest) on the CPU
tier: W host builds of the device step (tests/soa_cpu) exchange every
cross-engine message only as encoded MessageBatch frames (rbe_wire_encode per
destination engine → bytes → rbe_wire_ingest), which the receiver decodes,
checks (Peer.Handle, peer.go:186-198) and scatters with the same functions the
device kernels run (dragonboat_amd/csrc/rbe_ingest.h).  Every owned replica
must equal the oracle stepping all replicas in one process, as over
rbe_push_messages (test_transport.py).  test_gpu_wire_ingest.py runs the same
on the HIP engine."""
import pytest

import oracle as O
import session_scenarios as S
from soa_cpu.soa import SoaCpu
from test_transport import CASES
from transport_util import deliver_wire, run_transport


@pytest.mark.parametrize("name", list(CASES))
def test_wire_transport_parity_cpu(name):
    kw, world, rounds, extra = CASES[name]
    engs = [SoaCpu(trace=True, rep_world=world, rep_rank=r, **kw, **extra) for r in range(world)]
    ref = O.Harness(**kw)
    d, moved = run_transport(engs, ref, kw["n_replicas"], rounds, wire=True)
    assert d is None, f"{name}: first divergence {d}"
    assert moved > rounds
    for e in engs:
        assert e.faults()[0] == 0


@pytest.mark.parametrize("world", [2, 3])
def test_wire_session_entries_cpu(world):
    """Forwarded Proposes and Replicates with session fields and KiB Cmds: the
    receiver writes the heap records itself."""
    S.session_over_transport(SoaCpu, world, wire=True)


def test_wire_ingest_checks_cpu():
    from dragonboat_amd.engine import RBE_E_CORRUPT, RBE_E_INVALID, RBE_E_STATE, InputError
    from parity_util import C2
    kw = dict(C2, n_groups=6)
    a = SoaCpu(trace=True, rep_world=2, rep_rank=0, **kw)
    b = SoaCpu(trace=True, rep_world=2, rep_rank=1, **kw)
    for _ in range(30):
        a.run(1)
        b.run(1)
        deliver_wire([a, b])
    data, _ = a.wire_encode(dst_rank=1)
    assert data
    # frames meant for rank 1 are refused by rank 0 (its own replicas' senders)
    with pytest.raises(InputError) as ei:
        a.wire_ingest(data)
    assert ei.value.rc == RBE_E_INVALID
    bad = bytearray(data)
    bad[-1] ^= 0xFF
    with pytest.raises(InputError) as ei:
        b.wire_ingest(bytes(bad))
    assert ei.value.rc == RBE_E_CORRUPT
    assert b.wire_ingest(b"")["messages"] == 0
    one = SoaCpu(trace=True, **kw)
    one.run(2)
    with pytest.raises(InputError) as ei:
        one.wire_ingest(data)
    assert ei.value.rc == RBE_E_STATE
