"""Group-range snapshots (rbe_export_groups / rbe_import_groups, rbe_snap.h) on the
host build of the step: checkpoint/resume must continue bit-exact with the oracle,
a partial import must overwrite exactly its groups, and bad snapshots are refused
with the C-ABI error codes.  The GPU tier runs the same through the HIP engine and
imports a host-build snapshot into it (tests/test_gpu_snapshot.py).

Reference behaviour restated: a dragonboat node restarted on an existing log
resumes the same protocol state (peer.go:64-87 Launch, raft.go:283-330
loadState); the reference's own restart tests check that the state after a
restart is the state before (raft_test.go TestRaftNodeRestart*-style) — here the
oracle harness plays the uninterrupted node."""
import pytest

import oracle as O
from parity_util import C2, C3, C4, ENGINE_EXTRA, MIXED, run_lockstep, view_diff
from soa_cpu.soa import SnapshotError, SoaCpu, lib

RBE_E_INVALID, RBE_E_NOMEM, RBE_E_STATE = -1, -3, -5
CASES = {"C2": (C2, 77), "C3": (C3, 141), "C4": (C4, 233), "MIXED": (MIXED, 118)}


@pytest.mark.parametrize("name", list(CASES))
def test_resume_matches_uninterrupted_oracle(name):
    kw, at = CASES[name]
    extra = ENGINE_EXTRA.get(name, {})
    a = SoaCpu(trace=True, **kw, **extra)
    a.run(at)
    snap = a.export_groups()
    b = SoaCpu(trace=True, **kw, **extra)
    b.import_groups(snap, resume=True)
    ref = O.Harness(**kw)
    ref.run(at)
    ev, rv = b.views(), ref.views()
    for i in range(len(rv)):
        assert view_diff(ev[i], rv[i]) is None, (i, view_diff(ev[i], rv[i]))
    d = run_lockstep(b, ref, 120, every=1)
    assert d is None, f"{name}: first divergence after resume {d}"
    assert b.faults()[0] == 0


def test_partial_import_overwrites_only_its_groups():
    """Two engines of one configuration diverge (B gets extra host-pushed
    proposals); importing A's groups [5, 17) into B makes exactly those groups
    equal A's, and leaves B's others alone."""
    kw = dict(C3, ext_inputs=True)
    a = SoaCpu(trace=True, **kw)
    b = SoaCpu(trace=True, **kw)
    a.run(89)
    b.run(88)
    # B diverges through host-pushed proposals at every replica of every group
    b.push_proposals(list(range(b.n_rep)), [[b"div-%d" % i] for i in range(b.n_rep)])
    b.run(1)
    before = [tuple(getattr(v, "digest") for v in [x]) for x in b.views()]
    b.import_groups(a.export_groups(5, 12))
    n = kw["n_replicas"]
    av, bv = a.views(), b.views()
    for i in range(len(bv)):
        g = i // n
        if 5 <= g < 17:
            assert view_diff(bv[i], av[i]) is None, (i, view_diff(bv[i], av[i]))
        else:
            assert (bv[i].digest,) == before[i], i
    # the snapshot's planes are the group range only: their size adds up per
    # group; the log section after them (the cold logs below the ring) comes on top
    f1, f12 = lib().soa_snapshot_bytes(a.h, 1), lib().soa_snapshot_bytes(a.h, 12)
    assert (f12 - f1) % 11 == 0 and f12 > f1
    assert len(a.export_groups(0, 12)) >= f12


def test_import_rejects_other_behaviour():
    """A snapshot resumes bit-exact only under the configuration that wrote it:
    a different seed (or timeout, quorum check, workload ...) is refused."""
    a = SoaCpu(trace=True, **C4)
    b = SoaCpu(trace=True, **dict(C4, seed=0xBADC0DE))
    a.run(3)
    b.run(3)
    with pytest.raises(SnapshotError) as ei:
        b.import_groups(a.export_groups(0, 2))
    assert ei.value.rc == RBE_E_INVALID
    c = SoaCpu(trace=True, **dict(C4, election_rtt=12))
    c.run(3)
    with pytest.raises(SnapshotError):
        c.import_groups(a.export_groups(0, 2))


def test_export_import_roundtrip_is_identity():
    a = SoaCpu(trace=True, **C4)
    a.run(61)
    snap = a.export_groups()
    a.import_groups(snap)
    assert a.export_groups() == snap


def test_snapshot_errors():
    a = SoaCpu(trace=True, **C2)
    a.run(10)
    snap = a.export_groups(3, 4)
    # short export buffer
    with pytest.raises(SnapshotError) as ei:
        a.export_groups(0, 2, cap=64)
    assert ei.value.rc == RBE_E_NOMEM
    # empty / out-of-range ranges
    for first, count in ((0, 0), (64, 1), (60, 5)):
        with pytest.raises(SnapshotError) as ei:
            a.export_groups(first, count)
        assert ei.value.rc == RBE_E_INVALID
    # a snapshot from another round is refused without RESUME
    a.run(1)
    with pytest.raises(SnapshotError) as ei:
        a.import_groups(snap)
    assert ei.value.rc == RBE_E_STATE
    # RESUME needs the whole engine
    with pytest.raises(SnapshotError) as ei:
        a.import_groups(snap, resume=True)
    assert ei.value.rc == RBE_E_INVALID
    # geometry mismatch (ring), truncation, corrupted magic
    b = SoaCpu(trace=True, **C2, ring=128)  # (another geometry)
    b.run(10)
    for bad in (snap, snap[:-1], b"\0" * 8 + snap[8:]):
        with pytest.raises(SnapshotError) as ei:
            (b if bad is snap else a).import_groups(bad)
        assert ei.value.rc in (RBE_E_INVALID, RBE_E_STATE)
