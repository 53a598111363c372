"""Host-driven snapshots on the HIP engine (rbe_snapshot_saved / rbe_compact
with cfg.ext_apply) against the oracle harness driven the same way; the
CPU-tier twin is tests/test_host_snapshots.py."""
import pytest

import oracle as O
from test_host_snapshots import CASES, DRIVE, run_host_snapshots

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_host_driven_snapshots(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw = CASES[name]
    eng = Engine(device=0, trace=True, **kw, **DRIVE)
    ref = O.Harness(**kw)
    saved, compacted, restored = run_host_snapshots(eng, ref, 300)
    assert eng.fault_summary()[0] == 0
    assert saved > 20 and compacted > 10 and restored > 0, (saved, compacted, restored)
    eng.close()


def test_gpu_host_driven_snapshots_untraced(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = CASES["C3_HOT"]
    eng = Engine(device=0, trace=False, **kw, **DRIVE)
    ref = O.Harness(**kw)
    run_host_snapshots(eng, ref, 200, skip=("digest",))
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_host_driven_snapshots_apply_queue(gpu_available):
    """One step's input holds an applied index, apply-queue flags (twice for
    some replicas), a snapshot and a compaction for the same replica: the
    scatter writes each replica's Hot flags from one lane at a time."""
    from dragonboat_amd.engine import Engine
    kw = CASES["C3_HOT"]
    eng = Engine(device=0, trace=True, **kw, **DRIVE)
    ref = O.Harness(**kw)
    saved, compacted, _ = run_host_snapshots(eng, ref, 200, ready=0.5)
    assert eng.fault_summary()[0] == 0
    assert saved > 10 and compacted > 5, (saved, compacted)
    eng.close()
