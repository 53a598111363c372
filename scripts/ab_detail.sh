#!/bin/bash
# A/B with the per-kernel split printed (diagnostic builds under build/).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in dragonboat_amd/libdragonboat_amd.so ${LIBS}; do
  for w in ${WORKLOADS:-c4}; do
    RBE_LIB=$PWD/$lib RBE_MODE=${MODE:-split} timeout 200 python bench.py --workload $w --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $w"
  done
done
