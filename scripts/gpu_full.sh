#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, default bench (with CPU baseline),
# rocprofv3 kernel-trace summary of the bench.  Each GPU step has its own limit
# and the steps are chained so the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke ok $(( $(date +%s) - S ))s"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests ok $(( $(date +%s) - S ))s"
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "rocprof ok $(( $(date +%s) - S ))s"
