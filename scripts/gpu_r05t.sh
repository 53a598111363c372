#!/bin/bash
# Round 5 A/B: double-buffered ring <-> arena copies (current library) against
# the single-buffered build with 64-thread full-list blocks; parity tests first.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_membership.py tests/test_gpu_snapshot.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t_tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/r05t_tests.log)"
for rep in 1 2; do
for lib in build/libdragonboat_amd_fb64.so dragonboat_amd/libdragonboat_amd.so; do
  for w in c3 c3s c2s; do
    RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
