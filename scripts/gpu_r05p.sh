#!/bin/bash
# Round 5 A/B: does the best fast grid scale with the chunk count? C4 at 500k
# and 2M groups, and C4-shaped variants (c4h, c2m, c2s) at 768 vs 2048.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # grid workload groups
  RBE_FAST_GRID=$1 timeout -k 10 300 python -u bench.py --workload $2 ${3:+--groups $3} --no-cpu-baseline --also "" --steps 60 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
  python3 scripts/summarize_bench.py gpurun_out/ab.json "grid $1 $2 ${3}" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
}
for g in 2048 384 448 512 2048; do run $g c4 500000; done
for g in 2048 1408 1536 1664 2048; do run $g c4 2000000; done
for g in 2048 768 2048 768; do run $g c2m; done
