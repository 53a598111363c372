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
# optional workload: take gpurun_out/bench_<w>.json and gpurun_out/prof_<w>/
# (scripts/gpu_workloads.sh) instead of bench.json and prof/
wl = sys.argv[3] if len(sys.argv) > 3 else None
bench_name = f"bench_{wl}.json" if wl else "bench.json"
prof_dir = f"prof_{wl}" if wl else "prof"
cmd = f"python3 bench.py --workload {wl} --steps {steps} --no-cpu-baseline" if wl else \
    "python3 bench.py --no-cpu-baseline"
src = os.path.join(ROOT, "gpurun_out")
dst = os.path.join(ROOT, "profiles", name)
os.makedirs(dst, exist_ok=True)
for f in [bench_name, "gpu_tests.log", "smoke.log", "traffic_c4.json", "traffic_c2m.json"]:
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, "bench.json" if f == bench_name else f))
for f in ["run_kernel_stats.csv"]:
    p = os.path.join(src, prof_dir, f)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, "rocprof_kernel_stats.csv"))
lines = [f"# {name}: rocprofv3 --kernel-trace --stats of `{cmd}`", ""]
tr = os.path.join(src, prof_dir, "run_kernel_trace.csv")
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
b = os.path.join(src, bench_name)
if os.path.exists(b):
    d = json.loads(open(b).read().strip().splitlines()[-1])
    lines += ["", f"Bench line (`{cmd.replace(' --no-cpu-baseline', '')}`):", "", "```json",
              json.dumps(d, indent=1), "```"]
open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:20]))
