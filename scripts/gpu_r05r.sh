#!/bin/bash
# Round 5: full GPU suite on the effective-grid library, then the driver's
# bench command and a 200-step line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05r_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05r_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05r_bench20.json 2> gpurun_out/r05r_bench20.err
python3 scripts/summarize_bench.py gpurun_out/r05r_bench20.json "driver20" | head -4
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r05r_bench200.json 2> gpurun_out/r05r_bench200.err
python3 scripts/summarize_bench.py gpurun_out/r05r_bench200.json "200" | head -4
echo "bench ok $(( $(date +%s) - S ))s"
