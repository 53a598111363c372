"""rbe_wire_ingest on the HIP engine: W engines in one process on cuda:0
(rep_world = W) exchange every cross-engine message only as MessageBatch
frames — rbe_wire_encode per destination engine on the sender's device, the
bytes, rbe_wire_ingest on the receiver's device (decode, Peer.Handle checks,
radix sort by inbox list, scatter into the inbox planes; rbe_ingest.h).  No
record crosses back to the host.  Every owned replica must equal the oracle
(CPU twin: test_wire_ingest.py)."""
import pytest

import oracle as O
import session_scenarios as S
from test_gpu_session_entries import _make
from test_transport import CASES
from transport_util import deliver, deliver_wire, run_transport

pytestmark = pytest.mark.gpu


def _engines(world, kw, extra):
    from dragonboat_amd.engine import Engine
    return [Engine(device=0, trace=True, rep_world=world, rep_rank=r, **kw, **extra)
            for r in range(world)]


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_wire_transport_parity(gpu_available, name):
    kw, world, rounds, extra = CASES[name]
    engs = _engines(world, kw, extra)
    ref = O.Harness(**kw)
    d, moved = run_transport(engs, ref, kw["n_replicas"], rounds, wire=True)
    assert d is None, f"{name}: first divergence {d}"
    assert moved > rounds
    for e in engs:
        assert e.fault_summary()[0] == 0
        e.close()


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_wire_session_entries(gpu_available, world):
    S.session_over_transport(_make, world, wire=True)


def test_gpu_wire_ingest_equals_push(gpu_available):
    """The same rounds through rbe_push_messages and through rbe_wire_ingest
    leave identical replica views on both engine pairs, round by round."""
    from parity_util import C4, view_diff
    kw = dict(C4, n_groups=300)
    a, b = _engines(2, kw, {}), _engines(2, kw, {})
    n, n_rep = kw["n_replicas"], kw["n_groups"] * kw["n_replicas"]
    total = 0
    for rnd in range(150):
        for e in a + b:
            e.step()
        deliver(a, n, n_rep)
        total += deliver_wire(b)[0]
        va, vb = [e.views() for e in a], [e.views() for e in b]
        for r in range(2):
            for i in range(n_rep):
                assert view_diff(va[r][i], vb[r][i]) is None, (rnd, r, i)
    assert total > 1000
    for e in a + b:
        e.close()
