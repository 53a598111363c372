"""Every group size (N = 1..7) and spare slots on the HIP engine against the
oracle harness, round by round; the CPU-tier twin is tests/test_group_sizes.py."""
import pytest

import oracle as O
from parity_util import C3, counters_match, run_lockstep
from test_group_sizes import SIZES, shapes
from test_membership import CATCHUP, MEMB

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", ["C2", "C3", "C4"])
@pytest.mark.parametrize("n", SIZES)
def test_gpu_group_size_parity(gpu_available, n, shape):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = shapes(n)[shape]
    eng = Engine(device=0, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1)
    assert d is None, f"N={n} {shape}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    eng.close()


@pytest.mark.parametrize("n", [2, 4, 6, 7])
def test_gpu_group_size_untraced(gpu_available, n):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = shapes(n)["C4"]
    eng = Engine(device=0, trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, rounds, every=1, skip=("digest",)) is None
    eng.close()


@pytest.mark.parametrize("n,nv", [(5, 3), (4, 1), (6, 3), (7, 4)])
def test_gpu_spare_slots_join(gpu_available, n, nv):
    from dragonboat_amd.engine import Engine
    kw = dict(C3, n_groups=12, n_replicas=n, n_voters=nv, **MEMB)
    eng = Engine(device=0, trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    for _ in range(6):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"N={n} V={nv}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    eng.close()
