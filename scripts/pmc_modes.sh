#!/bin/bash
# TLB and L2-request PMC passes of one workload under each RBE_GROUP_LIST
# setting in $MODES (A/B of the triage modes).  Each pass has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
for m in ${MODES:-0 1}; do
  export RBE_GROUP_LIST=$m
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d gpurun_out/pmctlb_${w}_$m -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline > gpurun_out/pmctlb_${w}_$m.log 2>&1
  echo "== mode $m TLB"; python3 scripts/pmc_summary.py gpurun_out/pmctlb_${w}_$m
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d gpurun_out/pmcreq_${w}_$m -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline > gpurun_out/pmcreq_${w}_$m.log 2>&1
  echo "== mode $m requests"; python3 scripts/pmc_summary.py gpurun_out/pmcreq_${w}_$m
done
