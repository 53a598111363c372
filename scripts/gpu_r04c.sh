#!/bin/bash
# Round 4: microbenchmark, the GPU tests touched this round, then A/B of the
# fast kernel's LDS counters (default library) against build/ctr0.so.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 200 ./scripts/microbench/group_shape > gpurun_out/group_shape.log 2>&1
echo "microbench ok $(( $(date +%s) - S ))s"; cat gpurun_out/group_shape.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_observers_witnesses.py tests/test_gpu_node_ids.py tests/test_gpu_group_sizes.py tests/test_gpu_membership_snapshot.py tests/test_gpu_host_snapshots.py tests/test_gpu_membership.py tests/test_gpu_log_compaction.py tests/test_gpu_launch.py tests/test_gpu_rate_limit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || { tail -40 gpurun_out/gpu_tests_b.log; exit 1; }
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests_b.log
for i in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/ctr0.so; do
    for w in c4 c2m; do
      RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -1
    done
  done
done
echo "all ok $(( $(date +%s) - S ))s"
