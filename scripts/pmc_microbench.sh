#!/bin/bash
# Calibration of the PMC traffic counters on the group_shape microbenchmark,
# whose per-launch bytes and store counts are known by construction: one
# rocprofv3 pass per counter group, each under a hard limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ctr in "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum" FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmc_mb_$tag -o run --output-format csv -- ./scripts/microbench/group_shape > gpurun_out/pmc_mb_$tag.log 2>&1
done
