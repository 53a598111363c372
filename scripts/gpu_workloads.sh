#!/bin/bash
# Bench lines + rocprofv3 kernel-trace summaries for the BASELINE configs
# other than the default C4 (C2 = 10k x 3 steady replication, C3 = 100k x 5
# with leader isolation), each with its CPU baseline.  Each GPU step has its
# own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
for W in ${WORKLOADS:-c2 c3}; do
  timeout -k 10 400 python -u bench.py --workload $W --steps ${STEPS:-50} > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err
  echo "bench $W ok $(( $(date +%s) - S ))s"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$W -o run --output-format csv -- python3 bench.py --workload $W --steps ${STEPS:-50} --no-cpu-baseline > gpurun_out/prof_$W.log 2>&1
  echo "rocprof $W ok $(( $(date +%s) - S ))s"
done
