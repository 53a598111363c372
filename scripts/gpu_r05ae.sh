#!/bin/bash
# Round 5: effective-grid re-sweep after the back-first order (C4, C3).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for vg in 600 650 700 750; do
  for w in c4 c3; do
    RBE_FAST_VGRID=$vg timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "vg $vg $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
