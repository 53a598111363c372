#!/bin/bash
# SQ-side PMC passes (instruction mix, wait cycles) for one workload.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmcsq_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmcsq_$w.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmcsq_$w
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/pmcsq2_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmcsq2_$w.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmcsq2_$w
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d gpurun_out/pmcsq3_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline --also "" > gpurun_out/pmcsq3_$w.log 2>&1 || true
python3 scripts/pmc_summary.py gpurun_out/pmcsq3_$w || true
