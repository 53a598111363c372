"""The Peer.Handle boundary on the GPU: W HIP engines in one process on
cuda:0 (rep_world = W) exchange every cross-engine message through
rbe_get_outbox / rbe_push_messages; every owned replica must equal the oracle
(tests/transport_util.py, CPU twin: test_transport.py)."""
import pytest

import oracle as O
from test_transport import CASES
from transport_util import run_transport


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_transport_parity_gpu(name):
    from dragonboat_amd.engine import Engine
    kw, world, rounds, extra = CASES[name]
    engs = [Engine(device=0, trace=True, rep_world=world, rep_rank=r, **kw, **extra)
            for r in range(world)]
    ref = O.Harness(**kw)
    d, moved = run_transport(engs, ref, kw["n_replicas"], rounds)
    assert d is None, f"{name}: first divergence {d}"
    assert moved > rounds
    for e in engs:
        assert e.fault_summary()[0] == 0
