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


def test_gpu_wire_ingest_one_readback_equals_exact(gpu_available):
    """The one-read-back ingest (counts kept on the device, capacities from the
    last call, the writing walk gated on the device) leaves the same replica
    views as the exact path (RBE_INGEST_EXACT: read-backs between stages),
    round by round, through traffic that grows past the capacities (retried)
    and with big frames walked by chunks (groups_per_batch 0)."""
    import os
    from parity_util import C2, view_diff
    kw = dict(C2, n_groups=400)
    os.environ["RBE_WIRE_BIG"] = "2048"  # pair a walks its frames by chunks
    try:
        a = _engines(2, kw, {})
    finally:
        del os.environ["RBE_WIRE_BIG"]
    b = _engines(2, kw, {})
    n_rep = kw["n_groups"] * kw["n_replicas"]
    for rnd in range(120):
        for e in a + b:
            e.step()
        deliver_wire(a)
        os.environ["RBE_INGEST_EXACT"] = "1"
        try:
            deliver_wire(b)
        finally:
            del os.environ["RBE_INGEST_EXACT"]
        if rnd % 10 == 0 or rnd > 110:
            va, vb = [e.views() for e in a], [e.views() for e in b]
            for r in range(2):
                for i in range(n_rep):
                    assert view_diff(va[r][i], vb[r][i]) is None, (rnd, r, i)
    for e in a + b:
        assert e.fault_summary()[0] == 0
        e.close()


def test_gpu_wire_ingest_checks(gpu_available):
    """rbe_wire_ingest's refusals on the HIP engine, once its capacities are
    measured (the one-read-back path): a refused stream writes nothing (the
    engine then steps exactly as its twin that never saw it)."""
    from dragonboat_amd.engine import RBE_E_CORRUPT, RBE_E_INVALID, RBE_E_STATE, InputError
    from parity_util import C2, view_diff
    from transport_util import encode_for
    kw = dict(C2, n_groups=6)
    a, b = _engines(2, kw, {})
    a2, b2 = _engines(2, kw, {})
    for _ in range(30):
        for e in (a, b, a2, b2):
            e.run(1)
        deliver_wire([a, b])
        deliver_wire([a2, b2])
    data = encode_for(a, 1)
    assert data
    with pytest.raises(InputError) as ei:  # frames for rank 1 refused by rank 0
        a.wire_ingest(data)
    assert ei.value.rc == RBE_E_INVALID
    bad = bytearray(data)
    bad[-1] ^= 0xFF
    with pytest.raises(InputError) as ei:
        b.wire_ingest(bytes(bad))
    assert ei.value.rc == RBE_E_CORRUPT
    assert b.wire_ingest(b"")["messages"] == 0
    for _ in range(20):
        for e in (a, b, a2, b2):
            e.run(1)
        deliver_wire([a, b])
        deliver_wire([a2, b2])
    for x, y in ((a, a2), (b, b2)):
        vx, vy = x.views(), y.views()
        for i in range(len(vx)):
            assert view_diff(vx[i], vy[i]) is None, i
    from dragonboat_amd.engine import Engine
    one = Engine(device=0, trace=True, **kw)
    one.run(2)
    with pytest.raises(InputError) as ei:
        one.wire_ingest(data)
    assert ei.value.rc == RBE_E_STATE
    for e in (a, b, a2, b2, one):
        e.close()
