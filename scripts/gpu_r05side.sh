#!/bin/bash
# Round 5: the general step over triage's list on a second stream beside
# k_fast_both (default) against one stream (RBE_FULL_SIDE=0), C4 / C3 / C2,
# two runs each, then the -m gpu suite on the default.  Each GPU step has its
# own limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_side
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for w in c4 c3 c2; do
    for sd in 1 0; do
      RBE_FULL_SIDE=$sd timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > $O/ab_${w}_side${sd}_$rep.json 2> $O/ab_${w}_side${sd}_$rep.err
      python3 scripts/summarize_bench.py $O/ab_${w}_side${sd}_$rep.json "side$sd $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
