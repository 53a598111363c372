#!/bin/bash
# Round 5 close: SQ-side PMC passes (wave cycles, wait share, instruction mix)
# for the C4 and C2 pipelines on the tree's library, for the next round's plan.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_sq
mkdir -p $O
for w in c4 c2; do
  WORKLOAD=$w bash scripts/pmc_sq.sh > $O/sq_$w.txt 2>&1
  echo "== $w"; cat $O/sq_$w.txt
done
