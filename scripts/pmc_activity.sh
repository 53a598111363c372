#!/bin/bash
# Where a fast-step wave's cycles go: SQ activity/wait counters, two passes,
# at the workload's size and at 1/8 of it (lone waves).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
w=${WORKLOAD:-c4}
for g in ${SIZES:-125000 1000000}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM -d gpurun_out/pmcact1_${w}_$g -o run --output-format csv -- python3 bench.py --workload $w --groups $g --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline > gpurun_out/pmcact1_${w}_$g.log 2>&1
  echo "== $g pass 1"; python3 scripts/pmc_summary.py gpurun_out/pmcact1_${w}_$g
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES -d gpurun_out/pmcact2_${w}_$g -o run --output-format csv -- python3 bench.py --workload $w --groups $g --steps 10 --warmup 2 --prof-rounds 10 --no-cpu-baseline > gpurun_out/pmcact2_${w}_$g.log 2>&1
  echo "== $g pass 2"; python3 scripts/pmc_summary.py gpurun_out/pmcact2_${w}_$g
done
