#!/bin/bash
# Instruction-cache and address-translation PMC passes for one workload.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/pmcic_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmcic_$w.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmcic_$w
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d gpurun_out/pmctlb_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmctlb_$w.log 2>&1 || true
python3 scripts/pmc_summary.py gpurun_out/pmctlb_$w || true
