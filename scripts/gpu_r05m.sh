#!/bin/bash
# Round 5 A/B: the fast launches' grid cap on C4, C2, C3 (RBE_FAST_GRID).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 2048 1024 768 2048 1024 512; do
  for w in c4 c3; do
    RBE_FAST_GRID=$g timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "grid $g $w" | head -4
  done
done
