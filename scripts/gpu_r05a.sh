#!/bin/bash
# Round 5, first box: the graph tests, then the driver's exact bench command
# twice (event round vs kernel sum), then the default 200-step line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "graph" > gpurun_out/r05a_tests.log 2>&1
echo "graph tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05a_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05a_bench20.json 2> gpurun_out/r05a_bench20.err
echo "bench20 ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --also "" > gpurun_out/r05a_bench20b.json 2> gpurun_out/r05a_bench20b.err
echo "bench20b ok $(( $(date +%s) - S ))s"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --also "" > gpurun_out/r05a_bench200.json 2> gpurun_out/r05a_bench200.err
echo "bench200 ok $(( $(date +%s) - S ))s"
