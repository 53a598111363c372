"""GPU tier of tests/test_log_compaction.py: node snapshots, LogDB compaction
and InstallSnapshot through libdragonboat_amd.so (k_full_list takes every
step of a snapshot-enabled engine), diffed round by round against the oracle
harness, snapshot state (rbe_get_snapshot_state) included."""
import pytest

import oracle as O
from test_log_compaction import CASES, run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["C3_SNAP", "C3_NOCQ_SNAP", "C3_R64_ISO100", "MIXED_SNAP",
                                  "C4_SNAP"])
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
