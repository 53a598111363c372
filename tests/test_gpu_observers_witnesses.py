"""Observers and witnesses on the HIP engine against the oracle harness, round
by round; the CPU-tier twin is tests/test_observers_witnesses.py."""
import pytest

import oracle as O
from parity_util import run_lockstep
from test_membership import CATCHUP
from test_observers_witnesses import OW_CASES, SIZES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(OW_CASES))
def test_gpu_observer_witness_schedule(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, rounds = OW_CASES[name]
    eng = Engine(device=0, trace=True, **kw, **SIZES.get(name, CATCHUP))
    ref = O.Harness(**kw)
    wit = 0
    for _ in range(rounds // 50):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"{name}: first divergence {d}"
        wit |= max(v.witnesses for v in ref.views())
    assert wit
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_observer_witness_untraced(gpu_available):
    from dragonboat_amd.engine import Engine
    kw, _ = OW_CASES["N6"]
    eng = Engine(device=0, trace=False, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, 300, every=1, skip=("digest",)) is None
    eng.close()


def test_gpu_observer_witness_snapshots(gpu_available):
    from dragonboat_amd.engine import Engine
    from test_membership_snapshot import run_memb_snap
    kw = dict(OW_CASES["N5"][0], snapshot_entries=8, compaction_overhead=2, iso_mod=2)
    eng = Engine(device=0, trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, 400)
    assert eng.fault_summary()[0] == 0
    eng.close()
