#!/bin/bash
# Round 5 A/B: k_full_list in blocks of 256 / 128 / 64 threads (same waves):
# C3 (general steps of catch-up leaders), C3s, C4; parity on the 64 build.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
RBE_LIB=$PWD/build/libdragonboat_amd_fb64.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1
echo "tests fb64: $(tail -1 gpurun_out/r05s_tests.log)"
for rep in 1 2; do
for lib in dragonboat_amd/libdragonboat_amd.so build/libdragonboat_amd_fb128.so build/libdragonboat_amd_fb64.so; do
  for w in c3 c3s c4; do
    RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
