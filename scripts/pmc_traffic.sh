#!/bin/bash
# HBM traffic per pipeline kernel from PMC counters: one rocprofv3 pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), each
# under its own hard time limit, then scripts/pmc_traffic.py folds them into
# profiles/traffic_<workload>.json.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-c4 c2m}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${w}_$ctr -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmc_${w}_$ctr.log 2>&1
  done
  # request counts (the store audit): TCP->TCC write / read requests
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_${w}_REQ -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmc_${w}_REQ.log 2>&1
  python3 scripts/pmc_traffic.py $w gpurun_out/pmc_${w}_FETCH_SIZE gpurun_out/pmc_${w}_WRITE_SIZE gpurun_out/pmc_${w}_REQ
done
