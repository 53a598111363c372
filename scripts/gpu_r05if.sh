#!/bin/bash
# Round 5: the library built with the AMDGPU backend's early if-conversion
# (-mllvm -amdgpu-early-ifcvt=1, build/v_ifcvt.so) against the default, C4
# three times each alternating, C3 and C2 once.  Each GPU step has its own
# limit; the first failure ends the call.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_if
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in default v_ifcvt; do
    lib=dragonboat_amd/libdragonboat_amd.so
    [ "$v" = v_ifcvt ] && lib=build/v_ifcvt.so
    for w in c4 $([ $rep = 1 ] && echo c3 c2); do
      RBE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --also "" --steps 100 --warmup 10 > $O/ab_${w}_${v}_$rep.json 2> $O/ab_${w}_${v}_$rep.err
      python3 scripts/summarize_bench.py $O/ab_${w}_${v}_$rep.json "$v $w" | head -4 | tr '\n' ' ' | sed 's/  */ /g'; echo
    done
  done
done
