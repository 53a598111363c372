"""The spill tiers on the CPU tier (the device step compiled for the host,
tests/soa_cpu): inputs the reference handles without limits, which overflow
every fixed capacity of the engine's planes, run bit-exact with the oracle
and fault-free with the default capacities (ring 64, ecap 32, rq_cap 8, maxm
12, rtr_cap / dri_cap 8).  dragonboat_amd/csrc/rbe_spill.h:

  * the cold log: entryLog below the in-memory ring (logentry.go:144-161 term,
    186-246 getEntriesFromLogDB) — a follower isolated for 150 rounds, or a
    node relaunched hundreds of entries behind, is caught up from it, and a
    stale leader's long uncommitted tail is cut back (inMemory.merge,
    inmemory.go:201-234) with the window restored from it;
  * the round spill heap: catch-up Replicates sized by MaxEntrySize
    (raft.go:709-740, limitSize entryutils.go:50-64) past the sender's ecap
    arena, message lists past maxm, ReadyToReads past rtr_cap;
  * the readIndex queue past rq_cap (readindex.go:43-116 is unbounded).

The GPU twins are in test_gpu_spill.py."""
import pytest

import oracle as O
from launch_util import restart
from parity_util import counters_match, run_lockstep
from soa_cpu.soa import SoaCpu

# C3-shaped: 5 replicas, proposals every round at whoever leads, every other
# group's leader isolated for 150 of every 200 rounds; snapshots off (the
# reference default SnapshotEntries = 0: the LogDB keeps every entry)
LONG_ISO = dict(n_groups=16, n_replicas=5, wl_enabled=True, wl_start_round=30, iso_period=200,
                iso_len=150, iso_mod=2)


def _check(eng, ref, rounds, skip=(), counters=True):
    d = run_lockstep(eng, ref, rounds, every=1, skip=skip)
    assert d is None, f"first divergence {d}"
    n, bits = eng.faults()
    assert n == 0, f"faults {bits:#x}"
    if counters:  # (an engine resumed from a snapshot counts from there)
        bad = counters_match(eng.counters(), ref.counters())
        assert not bad, f"counters differ {bad}"


@pytest.mark.parametrize("check_quorum", [True, False])
@pytest.mark.parametrize("mode", ["pipeline", "full_table", "untraced"])
def test_long_isolation_cold_log(check_quorum, mode):
    """Without CheckQuorum the isolated leader keeps its role and appends 150
    uncommitted entries (more than the ring): on its return the new leader's
    entries replace that tail from below the window.  With it, the isolated
    replica steps down and falls 150 entries behind: its catch-up Replicate
    carries them from the leader's cold log, past the 32-entry arena."""
    kw = dict(LONG_ISO, check_quorum=check_quorum)
    trace = mode != "untraced"
    eng = SoaCpu(full_only=mode == "full_table", trace=trace, **kw)
    ref = O.Harness(trace=trace, **kw)
    _check(eng, ref, 620, skip=() if trace else ("digest",))
    st = eng.spill_stats()
    assert st["oom"] == 0
    assert st["pool_pages_used"] > 0, "the cold log was never used"
    assert st["spill_peak_bytes"] > 0, "no message or entry went to the spill heap"


def test_relaunch_far_behind():
    """Every group's leader is isolated at round 600 for 540 rounds: under
    CheckQuorum it steps down and falls 500+ entries behind while the others
    go on.  When the isolation ends it is relaunched through rbe_launch with
    its whole LogDB (~600 entries: the ring takes the last 64, the cold log
    the rest) and rejoins: the new leader backtracks over its short
    uncommitted tail and sends the 500+ missing entries from its cold log in
    one Replicate (limitSize, far past the 32-entry arena)."""
    kw = dict(n_groups=6, n_replicas=3, check_quorum=True, wl_enabled=True, wl_start_round=20,
              iso_period=600, iso_len=540, iso_mod=1)
    eng, ref = SoaCpu(trace=True, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 600, every=20) is None
    isolated = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    assert len(isolated) == kw["n_groups"]
    assert run_lockstep(eng, ref, 540, every=20) is None
    views = ref.views()
    behind = min(max(views[g * 3 + k].last_index for k in range(3)) - views[r].last_index
                 for g, r in enumerate(isolated))
    assert behind > 500, behind
    restart(eng, ref, isolated, None)  # the whole LogDB
    _check(eng, ref, 59)  # (the next epoch at 1200 isolates again)
    views = ref.views()
    # caught up (within the round in flight) where the backtracking over the
    # stale tail (one index per round trip, remote.go:155-171) has finished
    caught = [r for g, r in enumerate(isolated)
              if views[r].last_index + 1 >= max(views[g * 3 + k].last_index for k in range(3))]
    assert caught, "no relaunched replica caught up" 
    st = eng.spill_stats()
    assert st["pool_pages_used"] > 0 and st["spill_peak_bytes"] > 0 and st["oom"] == 0


def test_readindex_queue_past_rq_cap():
    """A leader short of quorum under CheckQuorum receives one ReadIndex per
    round for 12 rounds with rq_cap = 8: readIndex.addRequest queues them all
    (readindex.go:43-67) until the check-quorum boundary steps it down and
    reset clears the queue; bit-exact and fault-free."""
    kw = dict(n_groups=4, n_replicas=3, check_quorum=True, wl_enabled=True,
              wl_start_round=20, wl_read_permille=0, wl_active_mod=4, iso_period=60,
              iso_len=30, iso_mod=1, ext_inputs=True)
    eng, ref = SoaCpu(trace=True, rq_cap=8, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 60, every=1) is None
    leaders = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    assert leaders
    longest = 0
    for rnd in range(12):
        for r in leaders:
            ctx = ((60 + rnd + 1) << 32 | (r + 1), 77 + rnd)
            eng.push_read_index([r], [ctx])
            ref.push(O.PUSH_READ, r, ctx[0], ctx[1])
        assert run_lockstep(eng, ref, 1, every=1) is None
        longest = max([longest] + [v.rq_count for v in ref.views()])
    assert longest > 8, f"the queue never passed rq_cap ({longest})"
    _check(eng, ref, 40)


TINY = {  # the fast steps stay on (their own limits hold) / every capacity minimal
    "fast": dict(maxm=2, ecap=2, rq_cap=4, ring=8),
    "tiny": dict(maxm=1, rtr_cap=1, dri_cap=1, ecap=1, rq_cap=1, ring=8),
}


@pytest.mark.parametrize("caps", list(TINY))
@pytest.mark.parametrize("full_only", [False, True])
def test_lists_and_queues_past_capacity(caps, full_only):
    """Small plane capacities under the MIXED-shaped workload (5 replicas,
    CheckQuorum, Quiesce, reads and proposals, isolations): every message
    list, arena, output list and queue spills, including the fast steps'
    outbox stash, and the engine still equals the oracle round by round."""
    kw = dict(n_groups=12, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
              wl_start_round=25, wl_active_mod=2, wl_read_permille=500, iso_period=37,
              iso_len=20, iso_mod=2, seed=12345)
    eng = SoaCpu(trace=True, full_only=full_only, **TINY[caps], **kw)
    ref = O.Harness(**kw)
    _check(eng, ref, 300)
    st = eng.spill_stats()
    assert st["spill_peak_bytes"] > 0 and st["pool_pages_used"] > 0 and st["oom"] == 0


def test_snapshot_carries_cold_log_and_queue():
    """A group-range snapshot carries the spill tiers that live across rounds
    (rbe_snap.h log section): taken mid-isolation, when the isolated leaders
    hold 100+ uncommitted entries below their ring and the others' logs are
    mostly cold, resumed in a fresh engine it continues bit-exact with the
    oracle — the returning leaders' tails are cut back and the isolated
    followers caught up from the imported cold logs."""
    kw = dict(LONG_ISO, check_quorum=False)
    a, ref = SoaCpu(trace=True, **kw), O.Harness(trace=True, **kw)
    assert run_lockstep(a, ref, 340, every=20) is None
    assert a.spill_stats()["pool_pages_used"] > 0
    snap = a.export_groups()
    b = SoaCpu(trace=True, **kw)
    b.import_groups(snap, resume=True)
    _check(b, ref, 200, counters=False)
    # an import over live groups gives their old pages back to the pool first:
    # afterwards the engine holds exactly the snapshot's pages
    pages = a.spill_stats()["pool_pages_used"]
    b2 = SoaCpu(trace=True, **kw)
    b2.run(340)
    b2.import_groups(snap)
    assert b2.spill_stats()["pool_pages_used"] == pages


def test_snapshot_readindex_queue_in_pages():
    """A leader's readIndex queue past rq_cap (in pool pages) travels in the
    snapshot and resumes bit-exact."""
    kw = dict(n_groups=4, n_replicas=3, check_quorum=True, wl_enabled=True,
              wl_start_round=20, wl_read_permille=0, wl_active_mod=4, iso_period=60,
              iso_len=30, iso_mod=1, ext_inputs=True)
    a, ref = SoaCpu(trace=True, rq_cap=8, **kw), O.Harness(trace=True, **kw)
    assert run_lockstep(a, ref, 60, every=1) is None
    leaders = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    for rnd in range(10):
        for r in leaders:
            ctx = ((60 + rnd + 1) << 32 | (r + 1), 77 + rnd)
            a.push_read_index([r], [ctx])
            ref.push(O.PUSH_READ, r, ctx[0], ctx[1])
        assert run_lockstep(a, ref, 1, every=1) is None
    assert max(v.rq_count for v in a.views()) > 8
    b = SoaCpu(trace=True, rq_cap=8, **kw)
    b.import_groups(a.export_groups(), resume=True)
    assert [v.rq_count for v in b.views()] == [v.rq_count for v in a.views()]
    _check(b, ref, 40, counters=False)


def test_snapshot_refuses_round_spill():
    """Messages the next round reads from the round spill heap are not carried:
    the export is refused with RBE_E_STATE, and succeeds a round later once
    nothing spilled is in flight (rbe_export_groups contract)."""
    from soa_cpu.soa import SnapshotError
    kw = dict(n_groups=12, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
              wl_start_round=25, wl_active_mod=2, wl_read_permille=500, iso_period=37,
              iso_len=20, iso_mod=2, seed=12345)
    a = SoaCpu(trace=True, **TINY["tiny"], **kw)
    refused = ok_after = 0
    for _ in range(120):
        a.run(1)
        try:
            a.export_groups()
            if refused:
                ok_after += 1
        except SnapshotError as e:
            assert e.rc == -5
            refused += 1
    assert refused and ok_after
