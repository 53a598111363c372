"""Fold one GPU pass of `scripts/gpu_run.sh OUT ... prof` into profiles/<name>/:
the bench line, the rocprofv3 stats, the round kernels' dispatch trace (only
k_triage / k_fast_both / k_full_list, a few hundred KB) and summary.md, which
averages the LAST `window` dispatches of each round kernel — the bench's timed
and profiled rounds, not its settle and warmup — next to the bench's own
HIP-event split of the same rounds, with the ratio of the two.

    python3 scripts/round_evidence.py gpurun_out/r06x profiles/r06_final [window]

window defaults to the bench's steps + prof_rounds (read from its JSON line)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
ROUND = ("k_triage", "k_fast_both", "k_full_list")


def last_json(p):
    for line in reversed(open(p).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {p}")


bench_p = os.path.join(src, "bench_prof.json")
b = last_json(bench_p)
shutil.copy(bench_p, os.path.join(dst, "bench.json"))
window = int(sys.argv[3]) if len(sys.argv) > 3 else \
    int(b["steps"]) + int(b["roofline"].get("profiled_rounds", 0))
prof = os.path.join(src, "prof")
stats = os.path.join(prof, "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(dst, "rocprof_kernel_stats.csv"))
elif os.path.exists(os.path.join(prof, "run_results.db")):  # (kept whole: 1 MB)
    shutil.copy(os.path.join(prof, "run_results.db"), os.path.join(dst, "rocprof_results.db"))
by = defaultdict(list)
rows = []


def dispatches():
    """(start ns, kernel name, duration ns) in dispatch order: the CSV kernel
    trace, or rocprofv3's rocpd database (its default output format)"""
    tr = os.path.join(prof, "run_kernel_trace.csv")
    if os.path.exists(tr):
        with open(tr) as f:
            for r in csv.DictReader(f):
                yield (int(r["Start_Timestamp"]), r["Kernel_Name"],
                       int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        return
    import sqlite3
    db = sqlite3.connect(os.path.join(prof, "run_results.db"))
    yield from db.execute("select start, name, end - start from kernels order by start")


for st, k, d in dispatches():
    base = next((x for x in ROUND if x in k), None)
    if base is None:
        continue
    by[base].append(d)
    rows.append((st, base, d))
with open(os.path.join(dst, "round_kernel_trace.csv"), "w") as f:
    f.write("start_ns,kernel,duration_ns\n")
    for s, k, d in rows:
        f.write(f"{s},{k},{d}\n")
hip = {k["kernel"]: k["avg_us"] for k in b["round"]["kernels"]}
# the same command without the profiler (gpu_run.sh bench: bench_default.json),
# whose kernel split the profiler does not inflate
plain_p = os.path.join(src, "bench_default.json")
plain = last_json(plain_p) if os.path.exists(plain_p) else None
hip0 = {k["kernel"]: k["avg_us"] for k in plain["round"]["kernels"]} if plain else {}
if plain:
    shutil.copy(plain_p, os.path.join(dst, "bench_default.json"))
lines = [f"# {os.path.basename(dst)}: steady-state round kernels", "",
         f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --also \"\"` "
         f"(C4, {b['steps']} timed + {b['roofline'].get('profiled_rounds', 0)} profiled rounds; "
         f"library {b.get('library', {}).get('sha256_16', '?')}).", "",
         f"rocprofv3 averages over the LAST {window} dispatches of each round kernel (the timed and "
         "profiled rounds; the earlier ones are the 260 settle rounds with every group active and "
         "the warmup), against the bench's HIP-event split of its profiled rounds:", "",
         "| kernel | dispatches | rocprof avg µs (last window) | rocprof avg µs (all) | "
         "bench µs, same run (under the profiler) | bench µs, run without the profiler | "
         "rocprof / bench without |",
         "|---|---|---|---|---|---|---|"]
for k in ROUND:
    v = by.get(k, [])
    if not v:
        continue
    w = v[-window:]
    a = sum(w) / len(w) / 1e3
    h, h0 = hip.get(k), hip0.get(k)
    fmt = lambda x: f"{x:.1f}" if x else "-"
    ratio = f"{a / h0:.3f}" if h0 else "-"
    lines.append(f"| `{k}` | {len(v)} | {a:.1f} | {sum(v) / len(v) / 1e3:.1f} | {fmt(h)} | "
                 f"{fmt(h0)} | {ratio} |")
rf = (plain or b)["roofline"]
lines += ["", "The bench's split times each kernel by a start / stop event pair its own dispatch "
          "stamps (hipExtLaunchKernel, rbe_profile_rounds); under rocprofv3 every dispatch is "
          "slower, so the run without the profiler is the one the roofline below uses.",
          "", "A kernel whose rounds carry no item (C4's `k_full_list`: the full list is empty "
          "in the steady state) is one dispatch of a few µs; its ratio measures the profiler's "
          "per-dispatch cost (~1 µs), not work."]
lines += ["", f"Roofline (dominant kernel `{rf['kernel']}`): {rf['alg_bytes_per_launch']:.0f} B "
          f"algorithmic per launch / {rf['avg_launch_us']:.2f} µs = {rf['achieved']:.0f} GB/s, "
          f"frac {rf['frac']:.4f} of {rf['peak']:.0f} GB/s; ms_per_step {(plain or b)['ms_per_step']:.4f}.",
          "", "Bench line:", "", "```json", json.dumps(b, indent=1), "```"]
open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:16]))
