#!/bin/bash
# Round 5: ingest workload with one walk launch, per-frame walk vs chunked walk
# thresholds; the host-driven line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire_ingest.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05j_tests.log
for big in 262144 16384 8192; do
  RBE_WIRE_BIG=$big timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb 512 > gpurun_out/r05j_ingest_$big.json 2> gpurun_out/r05j_ingest_$big.err
  echo "ingest big=$big"; cat gpurun_out/r05j_ingest_$big.json
done
timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb 100000 > gpurun_out/r05j_ingest_all.json 2> gpurun_out/r05j_ingest_all.err
echo "ingest gpb all"; cat gpurun_out/r05j_ingest_all.json
cd /tmp && RBE_WIRE_BIG=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05j_prof_ing -o ing -- python3 $GRAFT_REPO_ROOT/scripts/wire_ingest_bench.py --gpb 512 > $GRAFT_REPO_ROOT/gpurun_out/r05j_prof_ing.log 2>&1
cd $GRAFT_REPO_ROOT
echo "prof ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/r05j_c4h.json 2> gpurun_out/r05j_c4h.err
echo "c4h ok"; cat gpurun_out/r05j_c4h.json
