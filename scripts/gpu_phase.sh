#!/bin/bash
# Diagnostic: per-phase wave cycles of k_triage and the fast steps (RBE_PHASE_TIMING build).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in c4 c2 c3; do
  timeout -k 10 200 python -u scripts/phase_timing.py $w > gpurun_out/phase_$w.log 2>&1 || { tail -20 gpurun_out/phase_$w.log; exit 1; }
  cat gpurun_out/phase_$w.log
done
