#!/bin/bash
# Round 5 A/B: surplus blocks of k_fast_both's worst-case grid (RBE_FAST_GRID)
# at the 0.7 effective grid: 2048 (default) vs 1024 vs 832 on C4, C3, C2.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for g in 2048 1024 832; do
  for w in c4 c3 c2; do
    RBE_FAST_GRID=$g timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "grid $g $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
