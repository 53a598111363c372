#!/bin/bash
# Round 5: big frames walked by chunks (parity tests + the 7 MB decode time),
# the C2 full-size test, and the host-driven line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_big.py tests/test_gpu_wire.py tests/test_gpu_wire_ingest.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -3 gpurun_out/r05f_tests.log
timeout -k 10 200 python -u scripts/wire_big_bench.py > gpurun_out/r05f_big.json 2> gpurun_out/r05f_big.err
echo "big ok $(( $(date +%s) - S ))s"; cat gpurun_out/r05f_big.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05f_prof -o big -- python3 $GRAFT_REPO_ROOT/scripts/wire_big_bench.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05f_prof.log 2>&1
cd $GRAFT_REPO_ROOT
echo "prof ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/r05f_c4h.json 2> gpurun_out/r05f_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"; cat gpurun_out/r05f_c4h.json
