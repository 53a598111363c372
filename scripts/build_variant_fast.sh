#!/bin/bash
# A/B variant of the engine library that recompiles only the untraced round
# translation units of the given group sizes with extra flags and links them
# with the tree's other objects (build/obj, from __graft_entry__.build()):
#   scripts/build_variant_fast.sh build/name.so "3 5" -DRBE_X=1 ...
set -e
cd "$(dirname "$0")/.."
out=$1; ns=$2; shift 2
obj=build/var_$(basename "$out" .so)
rm -rf "$obj"; mkdir -p "$obj"
cp build/obj/*.o "$obj"/
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-parameter $*"
for n in $ns; do
  /opt/rocm/bin/hipcc $F -DRBE_ROUND_N=$n -DRBE_ROUND_TRACE=0 -c -o $obj/rbe_round_${n}_0.o \
    dragonboat_amd/csrc/rbe_round.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out" $obj/*.o
echo built "$out"
