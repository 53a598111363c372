"""Diagnostic: what the general step (k_full_list) does per item on a workload
(default C3): the full-list slot's event counters over R rounds after the
settle, per round and per step — inbound / outbound messages, entries, ring
accesses, remote touches — beside the fast kernels'."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd.engine import Engine, make_config  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c3"
R = int(sys.argv[2]) if len(sys.argv) > 2 else 50
kw, settle, _ = bench.WORKLOADS[w]
eng = Engine(make_config(trace=False, **dict(kw)))
eng.run(settle)
eng.sync()
eng.reset_counters()
eng.run(R)
eng.sync()
out = {"workload": w, "rounds": R, "kernels": {}}
for i, name in enumerate(eng.kernel_names()):
    if not name:
        continue
    c = eng.kernel_counters(i)
    st = max(1, c["steps"])
    out["kernels"][name] = {"per_round": {k: v / R for k, v in c.items() if v},
                            "per_step": {k: round(v / st, 3) for k, v in c.items() if v}}
print(json.dumps(out, indent=1))
