#!/bin/bash
# TA (texture address) busy cycles against GPU-active cycles per kernel: is a
# round kernel bound by the per-CU address/issue path of its scattered
# accesses?  One pass, its own time limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES -d gpurun_out/pmcta_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline > gpurun_out/pmcta_$w.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmcta_$w
