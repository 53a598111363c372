#!/bin/bash
# Round 5 A/B: k_fast_both's effective grid (0.7 x chunks in list mode) vs one
# block per chunk (RBE_FAST_VGRID=1000); C3 with 700 forced.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label env workload
  env $2 timeout -k 10 300 python -u bench.py --workload $3 --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
  python3 scripts/summarize_bench.py gpurun_out/ab.json "$1 $3" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
}
for rep in 1 2; do
  run default X=1 c4
  run vg1000 RBE_FAST_VGRID=1000 c4
  run default X=1 c3
  run vg700 RBE_FAST_VGRID=700 c3
  run default X=1 c2
  run vg700 RBE_FAST_VGRID=700 c2
done
