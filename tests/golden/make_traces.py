"""Generate tests/golden/traces.json: per-configuration round-trace checkpoints
of the oracle harness (a checksum of every replica's running trace digest
every CHECK rounds, plus the final protocol state of every replica).

The oracle is the C++ restatement of internal/raft (oracle/); the reference
itself (Go) cannot run in this image, so these vectors pin the restatement
against drift and give the GPU tests a committed target.  The C1 entry also
carries the reference-semantics known answer committed = 3 bootstrap config
changes (peer.go:396-404) + 1 leader no-op (raft.go:985) + 10,000 proposals.

    python tests/golden/make_traces.py     # rewrites traces.json
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))

import oracle as O  # noqa: E402
from parity_util import C2, C3, C3_HOT, C4, C4_DENSE, MIXED, SINGLE  # noqa: E402

CHECK = 50
C1_FULL = dict(n_groups=1, n_replicas=3, wl_enabled=True, wl_start_round=30,
               wl_stop_round=10030)
CONFIGS = {"C1_10k": (C1_FULL, 10050), "C2": (C2, 300), "C3": (C3, 400), "C3_HOT": (C3_HOT, 400),
           "C4": (C4, 500), "C4_DENSE": (C4_DENSE, 400), "SINGLE": (SINGLE, 150),
           "MIXED": (MIXED, 600)}


def digest_checksum(views):
    h = hashlib.sha256()
    for v in views:
        h.update(int(v.digest).to_bytes(8, "little"))
    return h.hexdigest()[:16]


def final_state(views):
    return [[v.term, v.leader_id, v.committed, v.last_index, v.role] for v in views]


def trace(kw, rounds, views_fn, run_fn):
    points = []
    done = 0
    while done < rounds:
        k = min(CHECK, rounds - done)
        run_fn(k)
        done += k
        points.append([done, digest_checksum(views_fn())])
    return points


def main():
    out = {"_about": __doc__.strip().splitlines()[0], "check_every": CHECK, "configs": {}}
    for name, (kw, rounds) in CONFIGS.items():
        h = O.Harness(**kw)
        pts = trace(kw, rounds, h.views, h.run)
        out["configs"][name] = {"kw": kw, "rounds": rounds, "checkpoints": pts,
                                "final": final_state(h.views()), "counters": h.counters()}
    json.dump(out, open(os.path.join(HERE, "traces.json"), "w"), indent=0)


if __name__ == "__main__":
    main()
