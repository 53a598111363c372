#!/bin/bash
# GPU tests on the default library, then back-to-back bench lines of the
# default library and each in $LIBS (A/B, alternating twice).  Every GPU step
# has its own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests FAILED $(( $(date +%s) - S ))s"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  echo "gpu tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/gpu_tests.log
fi
for rep in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so ${LIBS}; do
    for w in ${WORKLOADS:-c4}; do
      RBE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab_$rep_$(basename $lib)_$w.json 2>gpurun_out/ab.err
      python3 scripts/summarize_bench.py gpurun_out/ab_$rep_$(basename $lib)_$w.json "$(basename $lib) $w"
    done
  done
done
