#!/bin/bash
# Size sweep of one workload: per-kernel time vs groups (latency- vs throughput-bound).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
w=${WORKLOAD:-c4}
for g in ${SIZES:-125000 250000 500000 1000000 2000000 4000000}; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --workload $w --groups $g --no-cpu-baseline > gpurun_out/scale_${w}_$g.json 2> gpurun_out/scale_${w}_$g.err
  python3 scripts/summarize_bench.py gpurun_out/scale_${w}_$g.json ${w}_$g
done
