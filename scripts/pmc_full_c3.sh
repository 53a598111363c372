#!/bin/bash
# What bounds k_full_list on C3: SQ wait / issue / instruction-mix counters over
# 60 profiled rounds (isolation epochs included), two passes.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmcfull1 -o run --output-format csv -- python3 bench.py --workload c3 --steps 60 --warmup 2 --prof-rounds 60 --no-cpu-baseline > gpurun_out/pmcfull1.log 2>&1
echo pass1 ok
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/pmcfull2 -o run --output-format csv -- python3 bench.py --workload c3 --steps 60 --warmup 2 --prof-rounds 60 --no-cpu-baseline > gpurun_out/pmcfull2.log 2>&1
echo pass2 ok
