#!/bin/bash
# Round 5: the GPU suite on the pruned library, an A/B of the message-list and
# arena capacities on C4 (footprint and TLB reach of the fast kernel), and the
# host-driven line with the pinned uploads and RBE_COLLECT_SKIP_LOCAL.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
rm -f gpurun_out/r05d_ab.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1
echo "tests ok $(( $(date +%s) - S ))s"; tail -1 gpurun_out/r05d_tests.log
for c in "" "maxm=6" "maxm=4" "maxm=4,ecap=8" "" "maxm=4,ecap=8"; do
  timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --also "" ${c:+--cfg $c} >> gpurun_out/r05d_ab.jsonl 2>> gpurun_out/r05d_ab.err
  echo "ab [$c] ok $(( $(date +%s) - S ))s"
done
timeout -k 10 300 python -u bench.py --workload c4h --steps 50 --warmup 5 > gpurun_out/r05d_c4h.json 2> gpurun_out/r05d_c4h.err
echo "c4h ok $(( $(date +%s) - S ))s"
