#!/bin/bash
# Round 4: microbenchmark + the GPU tests touched this round.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 200 ./scripts/microbench/group_shape > gpurun_out/group_shape.log 2>&1
echo "microbench ok $(( $(date +%s) - S ))s"; cat gpurun_out/group_shape.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_observers_witnesses.py tests/test_gpu_node_ids.py tests/test_gpu_group_sizes.py tests/test_gpu_membership_snapshot.py tests/test_gpu_host_snapshots.py tests/test_gpu_membership.py tests/test_gpu_log_compaction.py tests/test_gpu_launch.py tests/test_gpu_rate_limit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests_b.log
