"""Membership carried by snapshots on the HIP engine (libdragonboat_amd.so)
against the oracle harness, round by round; the CPU-tier twin is
tests/test_membership_snapshot.py (its docstring lists the reference paths)."""
import pytest

import oracle as O
from parity_util import counters_match
from test_membership_snapshot import CASES, host_restore_schedule, run_memb_snap

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_membership_snapshot_parity(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = CASES[name]
    eng = Engine(device=0, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    diff, snap_rem = run_memb_snap(eng, ref, rounds)
    nf, fo = eng.fault_summary()
    assert nf == 0, f"{name}: {nf} faulted replicas, bits {fo:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    assert snap_rem > 0 and diff > 0, (snap_rem, diff)
    eng.close()


@pytest.mark.parametrize("name", ["C2", "C3_HOT", "MIXED", "C3_HOT_N7"])
def test_gpu_membership_snapshot_untraced(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = CASES[name]
    eng = Engine(device=0, trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, rounds, skip=("digest",))
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_restart_over_snapshot_membership(gpu_available):
    from dragonboat_amd.engine import Engine
    from launch_util import restart
    kw, extra, _ = CASES["C2"]
    eng = Engine(device=0, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, 150)
    picks = [i for i in range(eng.n_rep) if ref.snapshot_state(i)[6]]
    assert picks
    restart(eng, ref, picks[:12], None, snapshots=True)  # the whole LogDB above the marker
    run_memb_snap(eng, ref, 150)
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_host_restore_remotes(gpu_available):
    from dragonboat_amd.engine import Engine
    from parity_util import C2
    from test_membership import CATCHUP
    kw = dict(C2, n_groups=8, ext_inputs=True, membership=True)
    eng = Engine(device=0, trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    assert host_restore_schedule(eng, ref, 150) > 10
    assert eng.fault_summary()[0] == 0
    eng.close()
