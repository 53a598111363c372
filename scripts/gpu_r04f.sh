#!/bin/bash
# Round 4: the general step's remote slots in LDS — GPU parity of the paths
# that take k_full_list, then C3 / C4 / c3s A/B against build/lrem0.so and
# build/lrem_defer.so.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_membership.py tests/test_gpu_observers_witnesses.py tests/test_gpu_log_compaction.py tests/test_gpu_group_sizes.py tests/test_gpu_node_inputs.py tests/test_gpu_outputs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_lrem.log 2>&1 || { tail -40 gpurun_out/gpu_lrem.log; exit 1; }
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_lrem.log
for i in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/lrem0.so build/lrem_defer.so; do
    for w in c3 c4; do
      RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -5
    done
  done
done
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err || { tail -20 gpurun_out/bench_c4h.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4h.json').read().strip().splitlines()[-1]);print('c4h', d['ms_per_step'], d['boundary'])"
echo "all ok $(( $(date +%s) - S ))s"
