#!/bin/bash
# Round 5: the whole GPU suite on the new library, the dense-vs-random
# microbenchmark, the default bench line and the C3 line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 120 ./scripts/microbench/group_shape > gpurun_out/r05c_group_shape.txt 2>&1
echo "microbench ok $(( $(date +%s) - S ))s"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c_gpu_tests.log 2>&1
echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05c_gpu_tests.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err
echo "bench ok $(( $(date +%s) - S ))s"
