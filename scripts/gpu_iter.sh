#!/bin/bash
# Iteration pass: GPU parity tests, then the bench workloads without the CPU leg.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for w in ${WORKLOADS:-c4 c2m c2 c3}; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  python3 scripts/summarize_bench.py gpurun_out/bench_$w.json $w
done
