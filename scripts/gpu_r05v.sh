#!/bin/bash
# Round 5 A/B: follower chunks first in k_fast_both (build/libdragonboat_amd_ff.so)
# at effective grids 0.7 and 1.0; parity on the ff build.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
RBE_LIB=$PWD/build/libdragonboat_amd_ff.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05v_tests.log 2>&1
echo "tests ff: $(tail -1 gpurun_out/r05v_tests.log)"
for rep in 1 2; do
for lib in dragonboat_amd/libdragonboat_amd.so build/libdragonboat_amd_ff.so; do
  for vg in 700 1000; do
    for w in c4 c3; do
      RBE_FAST_VGRID=$vg RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) vg$vg $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
done
