#!/bin/bash
# The whole -m gpu suite and smoke() on the library in the tree.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok $(( $(date +%s) - S ))s"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests.log
