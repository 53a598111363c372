"""GPU tier of tests/test_log_compaction.py: node snapshots, LogDB compaction
and InstallSnapshot through libdragonboat_amd.so (k_full_list takes every
step of a snapshot-enabled engine), diffed round by round against the oracle
harness, snapshot state (rbe_get_snapshot_state) included."""
import pytest

import oracle as O
from test_log_compaction import CASES, run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["C3_SNAP", "C3_NOCQ_SNAP", "C3_R64_ISO100", "MIXED_SNAP",
                                  "C4_SNAP", "N7_SNAP"])
def test_gpu_compaction_install_snapshot_parity(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = CASES[name]
    eng = Engine(device=0, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    restored = run_case(eng, ref, rounds)
    nf, fo = eng.fault_summary()
    assert nf == 0, f"{nf} faulted replicas, bits {fo:#x}"
    if name != "C4_SNAP":
        assert restored > 0
    eng.close()


def test_gpu_compaction_untraced(gpu_available):
    from dragonboat_amd.engine import Engine
    kw, extra, rounds = CASES["C3_SNAP"]
    eng = Engine(device=0, trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_case(eng, ref, rounds, skip=("digest",)) > 0
    assert eng.fault_summary()[0] == 0
    eng.close()


@pytest.mark.parametrize("name", ["C3_SNAP", "MIXED_SNAP"])
def test_gpu_restart_after_compaction(gpu_available, name):
    """rbe_launch over compacted LogDBs (marker, snapshot, entries above the
    marker) on the HIP engine; twin of test_log_compaction's host-build test."""
    from dragonboat_amd.engine import Engine
    from launch_util import restart
    from parity_util import counters_match
    kw, extra, _ = CASES[name]
    eng = Engine(device=0, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    run_case(eng, ref, 180)
    ring = extra.get("ring", 64)
    n = kw["n_replicas"]
    compacted = [i for i in range(eng.n_rep) if ref.snapshot_state(i)[0] > 0]
    assert len(compacted) > 5
    lead = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER and i in compacted]
    restart(eng, ref, sorted(set(compacted[:4] + lead[:3] + list(range(2 * n, 3 * n)))), ring,
            snapshots=True)
    run_case(eng, ref, 120)
    assert eng.fault_summary()[0] == 0
    assert not counters_match(eng.counters(), ref.counters())
    eng.close()
