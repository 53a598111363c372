"""Copy a GPU pass's evidence from gpurun_out/ into profiles/<name>/ with a
summary of the timed window (the last STEPS dispatches of each kernel in the
rocprofv3 kernel trace, which are the bench's timed rounds)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
src = os.path.join(ROOT, "gpurun_out")
dst = os.path.join(ROOT, "profiles", name)
os.makedirs(dst, exist_ok=True)
for f in ["bench.json", "gpu_tests.log", "smoke.log", "traffic_c4.json", "traffic_c2m.json"]:
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
for f in ["run_kernel_stats.csv"]:
    p = os.path.join(src, "prof", f)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, "rocprof_kernel_stats.csv"))
lines = [f"# {name}: rocprofv3 --kernel-trace --stats of `python3 bench.py --no-cpu-baseline`", ""]
tr = os.path.join(src, "prof", "run_kernel_trace.csv")
if os.path.exists(tr):
    by = defaultdict(list)
    for r in csv.DictReader(open(tr)):
        by[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines += ["Timed window (last %d dispatches of each round kernel; the bench times the same rounds "
              "with HIP events):" % steps, "", "| kernel | dispatches | avg µs (window) | avg µs (all) |",
              "|---|---|---|---|"]
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1][-steps:])):
        w = v[-steps:]
        lines.append(f"| `{k[:60]}` | {len(v)} | {sum(w) / len(w) / 1e3:.1f} | {sum(v) / len(v) / 1e3:.1f} |")
b = os.path.join(src, "bench.json")
if os.path.exists(b):
    d = json.loads(open(b).read().strip().splitlines()[-1])
    lines += ["", "Bench line (`python3 bench.py`):", "", "```json", json.dumps(d, indent=1), "```"]
open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:20]))
