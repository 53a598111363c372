"""Diagnostic: k_triage's time against its load on C4 shapes — the default
(1M groups, 10% active), no client input at all (every group asleep after the
settle: the awake lists are empty), and 100k / 300k groups at the default
density — per-kernel µs from rbe_profile_rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd.engine import Engine, make_config  # noqa: E402

kw0, settle, _ = bench.WORKLOADS["c4"]
shapes = [("c4", {}), ("c4 no input", {"wl_enabled": False}),
          ("c4 100k", {"n_groups": 100_000}), ("c4 300k", {"n_groups": 300_000})]
for name, over in shapes:
    eng = Engine(make_config(trace=False, **dict(kw0, **over)))
    eng.run(settle)
    eng.sync()
    ms = eng.profile_rounds(20)
    names = eng.kernel_names()
    print(json.dumps({"shape": name, "us": {n: round(v * 1e3 / 20, 1) for n, v in zip(names, ms) if n}}),
          flush=True)
    eng.close()
