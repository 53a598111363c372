#!/bin/bash
# A/B: the default library against build/ variants, split and fused pipelines.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in dragonboat_amd/libdragonboat_amd.so ${LIBS}; do
  for mode in ${MODES:-split fused}; do
    for w in ${WORKLOADS:-c4 c2m}; do
      RBE_LIB=$PWD/$lib RBE_MODE=$mode timeout 200 python bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
      python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) $mode $w" | head -1
    done
  done
done
