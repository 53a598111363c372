#!/bin/bash
# Kernel-trace stats plus the SQ-side PMC passes of one workload (default c4).
# Each GPU step has its own time limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 50 --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/prof_$w.log
echo "rocprof ok"
WORKLOAD=$w bash scripts/pmc_sq.sh > gpurun_out/pmc_sq_$w.txt 2>&1
cat gpurun_out/pmc_sq_$w.txt
