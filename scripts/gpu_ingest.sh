#!/bin/bash
# Wire ingest on the GPU: the parity tests, then the at-scale hop timed and
# under rocprofv3 --stats.  Each GPU step has its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire_ingest.py tests/test_gpu_wire.py \
  tests/test_gpu_transport.py tests/test_gpu_session_entries.py -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/ingest_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python -u scripts/wire_ingest_bench.py --groups ${GROUPS_:-100000} \
  > gpurun_out/ingest_bench.json 2> gpurun_out/ingest_bench.err
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ingest -o run -- \
  python3 scripts/wire_ingest_bench.py --groups ${GROUPS_:-100000} --rounds 10 --warmup 30 \
  > gpurun_out/prof_ingest.log 2>&1
echo "prof ok"
