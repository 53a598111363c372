#!/bin/bash
# Round 4: groups of 4..6 on the fast kernel at one wave per SIMD with the
# leader inbox in LDS (build/wide1.so): parity on the GPU, then C3 A/B.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
RBE_LIB=$PWD/build/wide1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group_sizes.py tests/test_gpu_observers_witnesses.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_wide1.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_wide1.log | head; tail -30 gpurun_out/gpu_wide1.log; exit 1; }
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_wide1.log
for i in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/wide1.so; do
    for w in c3 c3s; do
      RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -5
    done
  done
done
echo "all ok $(( $(date +%s) - S ))s"
