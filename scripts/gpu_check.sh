#!/bin/bash
# GPU parity tests (the whole -m gpu tier) then the default bench line.  Each
# GPU step has its own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests FAILED $(( $(date +%s) - S ))s"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  echo "bench ok $(( $(date +%s) - S ))s"
fi
