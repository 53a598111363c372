#!/bin/bash
# One GPU-box pass for the round's evidence: smoke, GPU parity tests, the
# default bench line (with the CPU baseline), a rocprofv3 kernel-trace summary
# of the same bench command, and the PMC traffic passes.  Each GPU step has
# its own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke ok $(( $(date +%s) - S ))s"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "rocprof ok $(( $(date +%s) - S ))s"
WORKLOADS="c4" bash scripts/pmc_traffic.sh
echo "pmc ok $(( $(date +%s) - S ))s"
