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


def commit_hook(eng, ref, seed, p_commit=0.55, p_partial=0.25):
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
