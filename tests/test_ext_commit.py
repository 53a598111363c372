"""Explicit Peer.Commit (rbe_commit / rbe_get_update_commits, cfg.ext_commit)
on the CPU tier: the device step code compiled for the host (tests/soa_cpu)
against the oracle harness, whose node defers entryLog.commitUpdate
(logentry.go:335-355) to the host exactly as the engine does.  A host that
persists late or only partly gets the unsaved entries again in its next
Update (EntriesToSave from savedTo + 1, inmemory.go:117-123) and the
unprocessed committed entries again (entriesToApply from processed + 1)."""
import pytest

import oracle as O
from commit_util import run_commit_driven, run_commit_snapshots
from dragonboat_amd.engine import InputError, RBE_E_STATE
from parity_util import C2, C3, C3_HOT, C4
from soa_cpu.soa import SoaCpu

DRIVEN = dict()


def _pair(kw):
    base = dict(kw, ext_inputs=True, ext_apply=True, ext_commit=True)
    sizes = dict(DRIVEN)
    if kw.get("n_replicas", 3) > 5:
        sizes["ecap"] = 256  # a leader copies a range for each of its remotes in one round
    return SoaCpu(trace=True, **dict(base, **sizes)), O.Harness(**base)


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("C4", C4),
                                     ("C3_N7", dict(C3, n_groups=24, n_replicas=7))])
def test_delayed_persist_parity(name, kw):
    eng, ref = _pair(dict(kw, n_groups=12))
    d, st = run_commit_driven(eng, ref, 160, seed=5)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    assert st["committed"] > 100 and st["partial"] > 5 and st["checked"] > 100, st


def test_no_commit_returns_entries_again():
    """Without a commit savedTo stays: every Update returns the same unsaved
    entries (and more), processed stays, committed entries come back."""
    eng, ref = _pair(dict(n_groups=1, n_replicas=3))
    for _ in range(25):
        eng.step()
        ref.step()
    v = ref.views()
    assert all(x.saved_to == 0 and x.processed == 0 for x in v)
    assert [x.saved_to for x in eng.views()] == [0, 0, 0]
    ucs = eng.update_commits()
    assert all(u[2] == v[i].last_index and u[0] == v[i].committed for i, u in enumerate(ucs))
    assert ucs == [ref.update_commit(i) for i in range(3)]


def test_commit_calls_refused():
    eng = SoaCpu(trace=True, n_groups=2, n_replicas=3, ext_inputs=True, ext_apply=True,
                 ext_commit=True)
    eng.step()
    with pytest.raises(InputError) as ei:  # the same replica twice in one batch
        eng.commit([1, 1], [(0, 0, 3, 1, 0, 0)] * 2)
    assert ei.value.rc == RBE_E_STATE
    eng.commit([1], [(0, 0, 3, 1, 0, 0)])
    with pytest.raises(InputError) as ei:  # a second commit before the next step
        eng.commit([1], [(0, 0, 3, 1, 0, 0)])
    assert ei.value.rc == RBE_E_STATE
    eng.step()
    assert eng.views()[1].saved_to == 3
    plain = SoaCpu(trace=True, n_groups=1, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError) as ei:
        plain.commit([0], [(0, 0, 0, 0, 0, 0)])
    assert ei.value.rc == RBE_E_STATE


def test_commit_panics_fault_the_replica():
    """commitUpdate panics (logentry.go:335-355) set RBE_FAULT_PANIC instead."""
    eng, ref = _pair(dict(n_groups=1, n_replicas=3))
    for _ in range(3):
        eng.step()
        ref.step()
    # processed beyond committed
    eng.commit([0], [(ref.views()[0].committed + 5, 0, 0, 0, 0, 0)])
    with pytest.raises(RuntimeError):
        ref.commit(0, (ref.views()[0].committed + 5, 0, 0, 0, 0, 0))
    eng.step()
    n, bits = eng.faults()
    assert n == 1 and bits & 0x20


# ext_commit with snapshots: host-driven snapshots (rbe_snapshot_saved /
# rbe_compact) and InstallSnapshot for the isolated replicas; the Update of a
# restoring step carries the snapshot until a commit names it
SNAP_COMMIT = dict(ext_inputs=True, ext_apply=True, ext_commit=True, snapshot_entries=1)
SNAP_CASES = {"C3_HOT": dict(C3_HOT, n_groups=16), "C3_N7": dict(C3, n_groups=12, n_replicas=7)}
SNAP_SIZES = dict()


@pytest.mark.parametrize("name", list(SNAP_CASES))
def test_snapshots_with_delayed_persist(name):
    base = dict(SNAP_CASES[name], **SNAP_COMMIT)
    eng, ref = SoaCpu(trace=True, **dict(base, **SNAP_SIZES)), O.Harness(**base)
    d, st = run_commit_snapshots(eng, ref, 300, seed=11)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    assert st["saved"] > 20 and st["compacted"] > 10, st
    assert st["restored"] > 0 and st["carried"] > st["restored"] and st["snap_commits"] > 0, st

