#!/bin/bash
# Round 5: segmented batch scan + segmented crc on encode for big frames —
# the wire suites, then the ingest bench with one frame per slot pair.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire.py tests/test_gpu_wire_ingest.py tests/test_gpu_replica.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05af_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s: $(tail -1 gpurun_out/r05af_tests.log)"
for g in 100000 512; do
  timeout -k 10 300 python -u scripts/wire_ingest_bench.py --gpb $g > gpurun_out/r05af_ingest_$g.json 2> gpurun_out/r05af_ingest_$g.err
  echo "gpb=$g $(cat gpurun_out/r05af_ingest_$g.json)"
done
