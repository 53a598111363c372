#!/bin/bash
# Round 5: single-copy ingest + register header parse in the chunked walk.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire.py tests/test_gpu_wire_ingest.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05k_tests.log
for g in 512 100000; do
  timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb $g > gpurun_out/r05k_ingest_$g.json 2> gpurun_out/r05k_ingest_$g.err
  echo "ingest gpb=$g"; cat gpurun_out/r05k_ingest_$g.json
done
timeout -k 10 200 python -u scripts/wire_big_bench.py > gpurun_out/r05k_big.json 2> gpurun_out/r05k_big.err
echo "big"; cat gpurun_out/r05k_big.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05k_prof_big -o big -- python3 $GRAFT_REPO_ROOT/scripts/wire_big_bench.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05k_prof_big.log 2>&1
echo "prof big ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05k_prof_ing -o ing -- python3 $GRAFT_REPO_ROOT/scripts/wire_ingest_bench.py --gpb 512 > $GRAFT_REPO_ROOT/gpurun_out/r05k_prof_ing.log 2>&1
echo "prof ingest ok $(( $(date +%s) - S ))s"
timeout -k 10 200 python -u scripts/phase_timing.py c4 > gpurun_out/r05k_phase_c4.log 2>&1
echo "phase"; cat gpurun_out/r05k_phase_c4.log
