#!/bin/bash
# k_triage replicas per block on C4 (group sleep, list mode): 2048 (default) vs 1024 vs 512.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/tri1024.so build/tri512.so; do
    RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --also "" \
      --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) c4 #$rep" | grep -E "ms/step|k_triage"
  done
done
