#!/bin/bash
# Round 5 A/B: the fused pipeline (RBE_MODE=fused: k_round triages and steps
# its own chunk, then k_full_list) against the default on engines without
# group sleep (C2, C3, C2m) and on C4.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for mode in default fused; do
  for w in c2 c3 c2m c4; do
    if [ $mode = fused ]; then export RBE_MODE=fused; else unset RBE_MODE; fi
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$mode $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
