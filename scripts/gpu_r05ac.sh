#!/bin/bash
# Round 5 A/B: k_triage loads its awake-list region without waiting for the
# region's count (build/lib_spec.so) against the default; C4 parity on it.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
RBE_LIB=$PWD/build/lib_spec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ac_tests.log 2>&1
echo "tests spec: $(tail -1 gpurun_out/r05ac_tests.log)"
for rep in 1 2 3; do
for lib in dragonboat_amd/libdragonboat_amd.so build/lib_spec.so; do
  RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
  python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) c4" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
done
done
