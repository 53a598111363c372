#!/bin/bash
# GPU parity tests against a candidate library, then an A/B of bench lines
# (default library and each in $LIBS) on the C4 workload.  Every GPU step has
# its own time limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TEST_LIB" ]; then
  RBE_LIB=$PWD/$TEST_LIB timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ab.log 2>&1 || { tail -30 gpurun_out/gpu_tests_ab.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_ab.log
fi
for lib in dragonboat_amd/libdragonboat_amd.so ${LIBS}; do
  for w in ${WORKLOADS:-c4}; do
    RBE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w"
  done
done
