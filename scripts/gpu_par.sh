#!/bin/bash
# The round's parity as a launch argument (RBE_PAR_ARG=1: k_triage loads its
# awake list with the round clock): C4 A/B pairs, then the GPU suite on it.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in dragonboat_amd/libdragonboat_amd.so build/par.so; do
    RBE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --also "" \
      --steps 100 --warmup 10 > gpurun_out/ab.json 2>gpurun_out/ab.err
    python3 scripts/summarize_bench.py gpurun_out/ab.json "$(basename $lib) c4 #$rep" | grep -E "ms/step|k_triage"
  done
done
RBE_LIB=$PWD/build/par.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/par_tests.log 2>&1
echo "par gpu tests ok"; tail -1 gpurun_out/par_tests.log
