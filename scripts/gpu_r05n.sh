#!/bin/bash
# Round 5 A/B: the fast launches' grid cap (RBE_FAST_GRID), finer sweep, C4 and C2.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for g in 2048 640 704 768 832 896 1536; do
  for w in c4 c2; do
    RBE_FAST_GRID=$g timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "grid $g $w" | head -3 | tr '\n' ' ' | sed 's/  */ /g'; echo
  done
done
done
