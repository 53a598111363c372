#!/bin/bash
# Round 5: ext_commit x snapshots, runtime node ids, two-set refusal, the
# scatter phases, multi-ConfigChange handoff, on the GPU; then the suites that
# share those paths.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 900 python -u -m pytest tests/test_gpu_ext_commit.py tests/test_gpu_host_snapshots.py tests/test_gpu_node_ids.py tests/test_gpu_observers_witnesses.py tests/test_gpu_membership.py tests/test_gpu_membership_snapshot.py tests/test_gpu_group_sizes.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05b_tests.log
