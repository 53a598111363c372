#!/bin/bash
# Build an A/B variant of the engine library with extra compiler flags:
#   scripts/build_variant.sh build/name.so -DRBE_FAST_WAVES=1 ...
# (same translation units as __graft_entry__.build(), objects under build/var_<name>)
set -e
cd "$(dirname "$0")/.."
out=$1; shift
obj=build/var_$(basename "$out" .so)
mkdir -p "$obj"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-parameter $*"
/opt/rocm/bin/hipcc $F -c -o $obj/e.o dragonboat_amd/csrc/rbe_engine.hip &
/opt/rocm/bin/hipcc $F -c -o $obj/s.o dragonboat_amd/csrc/rbe_sort.hip &
for n in 1 2 3 4 5 6 7; do for t in 0 1; do
  /opt/rocm/bin/hipcc $F -DRBE_ROUND_N=$n -DRBE_ROUND_TRACE=$t -c -o $obj/r_${n}_$t.o dragonboat_amd/csrc/rbe_round.hip &
done; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out" $obj/*.o
echo built "$out"
