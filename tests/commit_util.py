"""Host-driven persistence (cfg.ext_commit): the node calls Peer.Commit with
the UpdateCommit of an Update only after SaveRaftState has persisted it
(node.go:975-994, peer.go:282-293, 410-427).  This driver plays a host whose
persistence lags: each round it reads the UpdateCommit of every replica's last
step from the engine (rbe_get_update_commits) and from the oracle harness,
requires them equal, and commits a replica's pending Update only some rounds
later, sometimes only a saved prefix of it (stable_log_to below the Update's
last entry, with that entry's term).  Both sides get the same commits, so
every replica field and trace digest must stay equal (input_util.run_driven
compares them round by round)."""
from __future__ import annotations

import random

from input_util import run_driven


def commit_hook(eng, ref, seed, p_commit=0.55, p_partial=0.25, tweak=None):
    """`tweak(replica, uc)`, if given, may change each UpdateCommit before
    both sides get it."""
    rng = random.Random(seed ^ 0xC0FFEE)
    n = eng.cfg.n_replicas
    pend = {}
    state = {"checked": 0, "committed": 0, "partial": 0}

    def before_round(rnd):
        if rnd == 0:
            return
        euc = eng.update_commits()
        for r in range(eng.n_rep):
            ouc = ref.update_commit(r)
            assert tuple(euc[r]) == tuple(ouc), (rnd, r, "UpdateCommit", euc[r], ouc)
            state["checked"] += any(ouc)
            if any(ouc):
                pend[r] = ouc  # the latest Update holds everything still unsaved
        reps, ucs = [], []
        for r in sorted(pend):
            if rng.random() >= p_commit:
                continue  # persistence lags: commit in a later round (or never)
            uc = list(pend.pop(r))
            v = ref.views()[r]
            if uc[2] and rng.random() < p_partial and uc[2] > v.saved_to + 1:
                # only a prefix of EntriesToSave is durable yet
                to = rng.randrange(v.saved_to + 1, uc[2])
                uc[2], uc[3] = to, ref.log_term(r // n, r % n, to)
                state["partial"] += 1
            if tweak is not None:
                uc = list(tweak(r, tuple(uc)))
            reps.append(r)
            ucs.append(tuple(uc))
        if reps:
            eng.commit(reps, ucs)
            for r, uc in zip(reps, ucs):
                ref.commit(r, uc)
            state["committed"] += len(reps)

    return before_round, state


def run_commit_driven(eng, ref, rounds, seed, **kw):
    hook, state = commit_hook(eng, ref, seed)
    d = run_driven(eng, ref, rounds, seed=seed, ext_apply=True, before_round=hook, **kw)
    return d, state


def run_commit_snapshots(eng, ref, rounds, seed, every=12, overhead=3, **kw):
    """ext_commit with host-driven snapshots (cfg.snapshot_entries with
    ext_apply): commit_hook's lagging persistence plus the node's snapshot
    worker (rbe_snapshot_saved / rbe_compact, as tests/test_host_snapshots.py).
    An Update that carries a restored snapshot keeps carrying it until a
    commit names it (StableSnapshotTo, peer.go:410-427; inmemory.go:168-176;
    a commit without it would leave a later Update's Processed at the
    snapshot index, below raft's, which commitUpdate panics on, logentry.go:
    337-342).  Every round the Updates' snapshots and the
    node snapshot state must equal the oracle's too.  The host here is a
    node's: its LastApplied never passes what it has persisted (the node
    saves an Update before it applies it, node.go:975-994), so the LogDB it
    compacts holds every entry up to the raft log's last (rbe.h, rbe_commit)."""
    rng = random.Random(seed ^ 0x5A5A)
    counts = {"snap_commits": 0}  # commits naming a carried snapshot

    def tweak(r, uc):
        saved = max(ref.views()[r].saved_to, uc[2])
        if uc[1] > saved:
            uc = (uc[0], saved) + uc[2:]
        counts["snap_commits"] += uc[4] != 0
        return uc

    hook, state = commit_hook(eng, ref, seed, tweak=tweak)
    n = eng.cfg.n_replicas
    n_rep = eng.n_rep
    applied = [0] * n_rep
    last_ss = [0] * n_rep
    pend = {}
    state.update(carried=0, saved=0, compacted=0, restored=0)

    def before_round(rnd):
        hook(rnd)
        if rnd == 0:
            return
        eus = eng.update_snapshots()
        es = eng.snapshot_state()
        for r in range(n_rep):
            ous = ref.update_snapshot(r)
            assert tuple(eus[r]) == ous, (rnd, r, "Update.Snapshot", eus[r], ous)
            state["carried"] += ous[0] != 0
            oss = ref.snapshot_state(r)
            assert tuple(int(x) for x in es[r]) == tuple(oss), (rnd, r, "snapshot state",
                                                                  tuple(es[r]), oss)
            if oss[2] > last_ss[r]:  # a snapshot the host did not save: restored
                state["restored"] += 1
                last_ss[r] = oss[2]
        if rnd < 30:
            return
        for r in range(n_rep):
            if r in pend and rng.random() < 0.4:
                to = pend.pop(r)
                eng.compact([r], [to])
                ref.compact(r, to)
                state["compacted"] += 1
            elif applied[r] > last_ss[r] + every and rng.random() < 0.5:
                idx = applied[r]
                term = ref.log_term(r // n, r % n, idx)
                if term == 0:
                    continue
                eng.snapshot_saved([r], [idx], [term])
                ref.snapshot_saved(r, idx, term)
                last_ss[r] = idx
                if idx > overhead:
                    pend[r] = idx - overhead
                state["saved"] += 1

    def on_ops(ops):
        for kind, r, a in ops:
            if kind == "applied":
                applied[r] = a

    d = run_driven(eng, ref, rounds, seed=seed, ext_apply=True, before_round=before_round,
                   on_ops=on_ops, **kw)
    state.update(counts)
    return d, state
