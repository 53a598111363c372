#!/bin/bash
# Round 5: C2m / C2s spread on one box (default, one block per chunk).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for vg in 700 1000; do
    for w in c2m c2s; do
      RBE_FAST_VGRID=$vg timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
      python3 scripts/summarize_bench.py gpurun_out/ab.json "vg$vg $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
