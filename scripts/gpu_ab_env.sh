#!/bin/bash
# A/B of bench lines on one box: each entry of $RUNS is "label|env assignments|library"
# (empty library = the in-tree one).  Every GPU step has its own time limit; the
# first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra runs <<< "$RUNS"
for spec in "${runs[@]}"; do
  IFS='|' read -r label envs lib <<< "$spec"
  lib=${lib:-dragonboat_amd/libdragonboat_amd.so}
  env $envs RBE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload ${WORKLOAD:-c4} --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab_$label.json 2> gpurun_out/ab_$label.err
  python3 scripts/summarize_bench.py gpurun_out/ab_$label.json "$label"
done
