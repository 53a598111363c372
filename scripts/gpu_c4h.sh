#!/bin/bash
# The host-driven C4 line (bench.py --workload c4h) and the PMC traffic passes
# of the default C4 line on the same library.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 400 python -u bench.py --workload c4h --steps ${STEPS:-50} --warmup 5 > gpurun_out/bench_c4h.json 2> gpurun_out/bench_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"
if [ -z "$NO_PMC" ]; then
  WORKLOADS="c4" bash scripts/pmc_traffic.sh
  echo "pmc ok $(( $(date +%s) - S ))s"
fi
