#!/bin/bash
# Round 5 A/B: k_fast_both steps each role's back segments (a leader's
# proposal rounds, a follower's Replicate rounds) first (build/lib_bf.so)
# against the default; parity on it.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
RBE_LIB=$PWD/build/lib_bf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ad_tests.log 2>&1
echo "tests bf: $(tail -1 gpurun_out/r05ad_tests.log)"
for rep in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/lib_bf.so; do
    for w in c4 c3 c2; do
      RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
