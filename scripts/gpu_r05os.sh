#!/bin/bash
# Round 5: k_fast_both waits on instruction fetch (SQ_WAIT_INST_ANY 37% of its
# wave cycles on C4, its N=3 code is 122 KB): the library built -O3 (default)
# against -Os and -O2 builds (scripts/build_variant.sh) and the split pipeline
# (RBE_MODE=split: one kernel per role), C4 twice, C3 and C2
# once each, then the I-cache pass on the default.  Each GPU step has its own
# limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_os
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in default v_os v_o2 split; do
    lib=dragonboat_amd/libdragonboat_amd.so
    mode=both
    [ "$v" = v_os ] || [ "$v" = v_o2 ] && lib=build/$v.so
    [ "$v" = split ] && mode=split
    for w in c4 $([ $rep = 1 ] && echo c3 c2); do
      RBE_MODE=$mode RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > $O/ab_${w}_${v}_$rep.json 2> $O/ab_${w}_${v}_$rep.err
      python3 scripts/summarize_bench.py $O/ab_${w}_${v}_$rep.json "$v $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
WORKLOAD=c4 bash scripts/pmc_icache.sh > $O/icache_c4.txt 2>&1
cat $O/icache_c4.txt
