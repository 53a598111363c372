#!/bin/bash
# Round 4, first call: the group-layout microbenchmark, the rate-limiter GPU
# tests, the default bench line.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 120 ./scripts/microbench/group_shape > gpurun_out/group_shape.log 2>&1
echo "microbench ok $(( $(date +%s) - S ))s"; cat gpurun_out/group_shape.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rate_limit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_rl.log 2>&1
echo "rl tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests_rl.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench ok $(( $(date +%s) - S ))s"; cut -c1-600 gpurun_out/bench.json
