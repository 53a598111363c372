#!/bin/bash
# Diagnostic microbenchmarks only (scripts/microbench, built beforehand).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in ${MICRO:-group_shape}; do
  timeout -k 10 300 ./scripts/microbench/$b > gpurun_out/$b.log 2>&1
  echo "== $b"; cat gpurun_out/$b.log
done
