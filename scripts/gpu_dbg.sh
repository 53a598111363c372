#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/debug_memb.py MIXED > gpurun_out/dbg_memb.log 2>&1 || true
RBE_MODE=full timeout -k 10 300 python -u scripts/debug_memb.py MIXED > gpurun_out/dbg_memb_full.log 2>&1 || true
head -c 20000 gpurun_out/dbg_memb.log | head -120
echo ======= full
head -5 gpurun_out/dbg_memb_full.log
