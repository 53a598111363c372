"""Explicit Peer.Commit on the HIP engine (rbe_commit / rbe_get_update_commits
through the C ABI, cfg.ext_commit) against the oracle harness, round by round:
a host whose persistence lags and sometimes saves only a prefix of an Update
(tests/commit_util.py).  Every replica field and trace digest, and every
UpdateCommit the engine reports, equal the oracle's.  CPU-tier twin:
tests/test_ext_commit.py."""
import pytest

import oracle as O
from commit_util import run_commit_driven, run_commit_snapshots
from parity_util import C2, C3, C4
from test_ext_commit import SNAP_CASES, SNAP_COMMIT, SNAP_SIZES

pytestmark = pytest.mark.gpu

DRIVEN = dict()


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("C4", C4),
                                     ("C3_N7", dict(C3, n_replicas=7))])
def test_gpu_delayed_persist_parity(gpu_available, name, kw):
    from dragonboat_amd.engine import Engine
    base = dict(kw, n_groups=12, ext_inputs=True, ext_apply=True, ext_commit=True)
    sizes = dict(DRIVEN) if base["n_replicas"] > 5 else DRIVEN  # tests/test_ext_commit.py
    eng, ref = Engine(device=0, trace=True, **dict(base, **sizes)), O.Harness(**base)
    d, st = run_commit_driven(eng, ref, 160, seed=5)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    assert st["committed"] > 100 and st["partial"] > 5, st
    eng.close()


def test_gpu_commit_panic_faults(gpu_available):
    from dragonboat_amd.engine import Engine
    eng = Engine(device=0, trace=True, n_groups=1, n_replicas=3, ext_inputs=True,
                 ext_apply=True, ext_commit=True)
    for _ in range(3):
        eng.step()
    c = eng.views()[0].committed
    eng.commit([0], [(c + 5, 0, 0, 0, 0, 0)])  # processed above committed: commitUpdate panics
    eng.step()
    n, bits = eng.fault_summary()
    assert n == 1 and bits & 0x20
    eng.close()


@pytest.mark.parametrize("name", list(SNAP_CASES))
def test_gpu_snapshots_with_delayed_persist(gpu_available, name):
    """ext_commit with host-driven snapshots and InstallSnapshot: the Updates'
    snapshots, UpdateCommits (StableSnapshotTo), snapshot state, views and
    digests equal the oracle's every round (CPU twin in test_ext_commit.py)."""
    from dragonboat_amd.engine import Engine
    base = dict(SNAP_CASES[name], **SNAP_COMMIT)
    eng, ref = Engine(device=0, trace=True, **dict(base, **SNAP_SIZES)), O.Harness(**base)
    d, st = run_commit_snapshots(eng, ref, 300, seed=11)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    assert st["saved"] > 20 and st["compacted"] > 10 and st["restored"] > 0, st
    eng.close()
