#!/bin/bash
# Round 5: parallel crc for big frames, 2-D compact, piecewise overlapped
# upload: wire tests, ingest workload (and chunked walk on its 18 KB frames),
# 7 MB decode, kernel split.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire.py tests/test_gpu_wire_ingest.py tests/test_gpu_replica.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -2 gpurun_out/r05i_tests.log
for g in 512 100000; do
  timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb $g > gpurun_out/r05i_ingest_$g.json 2> gpurun_out/r05i_ingest_$g.err
  echo "ingest $g ok"; cat gpurun_out/r05i_ingest_$g.json
done
RBE_WIRE_BIG=16384 timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb 512 > gpurun_out/r05i_ingest_512_chunked.json 2> gpurun_out/r05i_ingest_c.err
echo "chunked 512 ok"; cat gpurun_out/r05i_ingest_512_chunked.json
timeout -k 10 200 python -u scripts/wire_big_bench.py > gpurun_out/r05i_big.json 2> gpurun_out/r05i_big.err
echo "big ok $(( $(date +%s) - S ))s"; cat gpurun_out/r05i_big.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05i_prof_big -o big -- python3 $GRAFT_REPO_ROOT/scripts/wire_big_bench.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05i_prof_big.log 2>&1
echo "prof big ok $(( $(date +%s) - S ))s"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05i_prof_ing -o ing -- python3 $GRAFT_REPO_ROOT/scripts/wire_ingest_bench.py --gpb 512 > $GRAFT_REPO_ROOT/gpurun_out/r05i_prof_ing.log 2>&1
echo "prof ingest ok $(( $(date +%s) - S ))s"
