"""Node snapshots, LogDB compaction and InstallSnapshot (config.SnapshotEntries /
CompactionOverhead) through the device step logic (host build, tests/soa_cpu),
diffed round by round against the oracle harness, whose node snapshots every
SnapshotEntries applied entries and compacts its LogDB to index -
CompactionOverhead at the next step (oracle/harness.cpp, node.go:585-692,
849-866).  A replica isolated long enough falls behind the leader's compaction
marker and is brought back by InstallSnapshot (raft.go:684-697, 758-792;
restore raft.go:439-470), the transport reporting the outcome at the sender's
next step (SnapshotStatus, raft.go:1758-1771).

Bar: every view field (digest included: it folds each message, an
InstallSnapshot's snapshot index/term in place of LogIndex/LogTerm) and the
snapshot state (marker, snapshot index/term, reqSnapshotIndex, compactLogTo)
equal the oracle's every round."""
import pytest

import oracle as O
from parity_util import C3, C4, MIXED, counters_match, view_diff
from soa_cpu.soa import SoaCpu

SNAP = dict(snapshot_entries=20, compaction_overhead=5)
CASES = {
    # isolation epochs of 30 rounds leave the cut-off replica > 25 entries behind
    "C3_SNAP": (dict(C3, **SNAP), dict(), 400),
    "C3_HOT_SNAP": (dict(C3, iso_mod=2, snapshot_entries=8, compaction_overhead=2),
                    dict(), 400),
    # no check-quorum: an isolated remote stays active, so the leader streams it
    # snapshots the transport fails (SnapshotStatus reject, clearPendingSnapshot)
    "C3_NOCQ_SNAP": (dict(C3, check_quorum=False, **SNAP), dict(), 400),
    # a 64-entry window and 100-round partitions, fault-free
    "C3_R64_ISO100": (dict(C3, iso_period=150, iso_len=100, **SNAP), dict(), 600),
    "MIXED_SNAP": (dict(MIXED, snapshot_entries=10, compaction_overhead=0),
                   dict(), 500),
    "C4_SNAP": (dict(C4, **SNAP), {}, 400),
    # groups of 7 (slot 6's outbox word in the sender's own place), leaders isolated
    "N7_SNAP": (dict(C3, n_groups=24, n_replicas=7, iso_mod=2, **SNAP), dict(), 400),
}


def run_case(eng, ref, rounds, skip=()):
    """Lockstep with the snapshot state compared too; returns the number of
    rounds in which some replica held a snapshot it received (snapshot index
    ahead of its own snapshot requests)."""
    restored = 0
    for rnd in range(rounds):
        eng.run(1)
        ref.run(1)
        ev, hv = eng.views(), ref.views()
        for i in range(len(hv)):
            d = view_diff(ev[i], hv[i], skip)
            assert d is None, f"round {rnd + 1} replica {i}: {d}"
        es = eng.snapshot_state()
        seen = False
        for i in range(len(hv)):
            os_ = ref.snapshot_state(i)
            assert tuple(es[i]) == os_, f"round {rnd + 1} replica {i}: {tuple(es[i])} != {os_}"
            if os_[2] > os_[4]:
                seen = True
        restored += seen
    return restored


@pytest.mark.parametrize("name", list(CASES))
def test_compaction_install_snapshot_parity(name):
    kw, extra, rounds = CASES[name]
    eng = SoaCpu(trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    restored = run_case(eng, ref, rounds)
    n, bits = eng.faults()
    assert n == 0, f"faults {bits:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"
    assert any(ref.snapshot_state(i)[0] > 0 for i in range(eng.n_rep)), "no compaction"
    if "C3" in name or "MIXED" in name:
        assert restored > 0, "no replica was brought back by InstallSnapshot"


def test_compaction_untraced_parity():
    kw, extra, rounds = CASES["C3_SNAP"]
    eng = SoaCpu(trace=False, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_case(eng, ref, rounds, skip=("digest",)) > 0
    assert eng.faults()[0] == 0


def test_compaction_full_table_only():
    """The same rounds through the full handler table alone (k_full_list)."""
    kw, extra, rounds = CASES["C3_SNAP"]
    eng = SoaCpu(full_only=True, trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_case(eng, ref, 200) >= 0
    assert eng.faults()[0] == 0


def test_compaction_state_survives_group_export():
    """rbe_export_groups / rbe_import_groups carry the snapshot planes: an
    engine resumed from a mid-run export (past compactions and InstallSnapshots)
    keeps stepping in lockstep with the oracle."""
    kw, extra, _ = CASES["C3_NOCQ_SNAP"]
    a = SoaCpu(trace=True, **kw, **extra)
    a.run(170)
    b = SoaCpu(trace=True, **kw, **extra)
    b.import_groups(a.export_groups(), resume=True)
    ref = O.Harness(**kw)
    ref.run(170)
    assert run_case(b, ref, 200) > 0
    assert b.faults()[0] == 0


def test_compaction_launch_checks():
    """rbe_launch over a compacted LogDB: the batch is refused whole when the
    commit lies below the marker (loadState panics, raft.go:429-437), when
    entries reach down to the marker, or when there is no snapshot plane."""
    from dragonboat_amd.engine import RBE_E_INVALID, InputError
    eng = SoaCpu(trace=True, **dict(C3, **SNAP))
    eng.run(5)
    ents = [[(i, 2, 0, b"") for i in range(11, 21)]]
    with pytest.raises(InputError) as ei:  # commit below the marker
        eng.launch([0], [(2, 0, 9, 20, 10, 2, 10, 2)], ents)
    assert ei.value.rc == RBE_E_INVALID
    with pytest.raises(InputError):  # an entry at the marker
        eng.launch([0], [(2, 0, 12, 20, 10, 2, 10, 2)], [[(i, 2, 0, b"") for i in range(10, 21)]])
    with pytest.raises(InputError):  # a marker without its term
        eng.launch([0], [(2, 0, 12, 20, 10, 0, 10, 2)], ents)
    plain = SoaCpu(trace=True, **C3)
    with pytest.raises(InputError):  # no snapshots configured
        plain.launch([0], [(2, 0, 12, 20, 10, 2, 10, 2)], ents)
    eng.launch([0], [(2, 0, 12, 20, 10, 2, 10, 2)], ents)


@pytest.mark.parametrize("name", ["C3_SNAP", "C3_NOCQ_SNAP", "MIXED_SNAP"])
def test_restart_after_compaction(name):
    """Restarts over compacted LogDBs (Peer.Launch over an existing log,
    peer.go:64-86; entryLog from GetRange: processed = marker,
    logentry.go:86-96; Term(marker) from the LogDB): replicas restarted with
    their LogDB's marker, snapshot and entries above the marker continue
    bit-exact with the oracle's restarted nodes, which recover their state
    machine from that snapshot."""
    from launch_util import restart
    kw, extra, rounds = CASES[name]
    eng = SoaCpu(trace=True, **kw, **extra)
    ref = O.Harness(**kw)
    run_case(eng, ref, 180)
    ring = extra.get("ring", 64)
    n = kw["n_replicas"]
    compacted = [i for i in range(eng.n_rep) if ref.snapshot_state(i)[0] > 0]
    assert len(compacted) > 5
    lead = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER and i in compacted]
    picks = sorted(set(compacted[:4] + lead[:3] + list(range(2 * n, 3 * n))))
    restart(eng, ref, picks, ring, snapshots=True)
    run_case(eng, ref, 120)
    restart(eng, ref, compacted[-3:], ring, snapshots=True)
    run_case(eng, ref, 80)
    assert eng.faults()[0] == 0
    assert not counters_match(eng.counters(), ref.counters())


def test_compaction_fast_step_aux():
    """The fast steps' summary-word variant (as k_fast_both runs them) with
    node snapshots taken inside the fast epilogue."""
    kw, extra, rounds = CASES["C3_SNAP"]
    eng = SoaCpu(trace=True, staged=4, **kw, **extra)
    ref = O.Harness(**kw)
    assert run_case(eng, ref, rounds) > 0
    assert eng.faults()[0] == 0


def test_compaction_keeps_fast_paths():
    """Snapshots are taken inside the fast steps; only the step after one (the
    compaction) and InstallSnapshot traffic take the full handler table."""
    from parity_util import C2
    kw = dict(C2, snapshot_entries=20, compaction_overhead=5)
    eng = SoaCpu(trace=True, **kw)
    ref = O.Harness(**kw)
    run_case(eng, ref, 200)
    assert eng.slow_total() < 0.25 * eng.counters()["steps"]
