#!/bin/bash
# Round 4: k_full_list grid 64 vs 256 (C4 empty launches, C3 work), and the
# c4h line with the push split.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -m pytest tests/test_gpu_outputs.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_outputs.log 2>&1 || { tail -30 gpurun_out/gpu_outputs.log; exit 1; }
tail -1 gpurun_out/gpu_outputs.log
for i in 1; do
  for lib in dragonboat_amd/libdragonboat_amd.so; do
    for w in c4 c3; do
      RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -5
    done
  done
done
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err || { tail -20 gpurun_out/bench_c4h.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4h.json').read().strip().splitlines()[-1]);print('c4h', d['ms_per_step'], d['boundary'])"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_c4h -o run -- python3 bench.py --workload c4h --steps 30 --warmup 5 > gpurun_out/prof_c4h.log 2>&1 || { tail -20 gpurun_out/prof_c4h.log; exit 1; }
echo "all ok $(( $(date +%s) - S ))s"
