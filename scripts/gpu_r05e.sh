#!/bin/bash
# Round 5: the host-driven c4h line with one-pass input staging.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/r05e_c4h.json 2> gpurun_out/r05e_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"; cat gpurun_out/r05e_c4h.json
