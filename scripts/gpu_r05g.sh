#!/bin/bash
# Round 5: the 7 MB decode time and its kernel split.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 200 python -u scripts/wire_big_bench.py > gpurun_out/r05g_big.json 2> gpurun_out/r05g_big.err
echo "big ok $(( $(date +%s) - S ))s"; cat gpurun_out/r05g_big.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05g_prof -o big -- python3 $GRAFT_REPO_ROOT/scripts/wire_big_bench.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05g_prof.log 2>&1
echo "prof ok $(( $(date +%s) - S ))s"
