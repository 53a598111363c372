// One translation unit per group size N and trace mode (-DRBE_ROUND_N=1..7,
// -DRBE_ROUND_TRACE=0 or 1): the round pipeline's kernels for them and
// launch_round<N, TRACE> (rbe_kernels.h), linked into libdragonboat_amd.so
// with rbe_engine.hip.
#include "rbe_kernels.h"

#if !defined(RBE_ROUND_N) || !defined(RBE_ROUND_TRACE)
#error "build with -DRBE_ROUND_N=1..7 and -DRBE_ROUND_TRACE=0 or 1"
#endif

namespace rbe {
template int launch_round<RBE_ROUND_N, RBE_ROUND_TRACE != 0>(const Planes&, const Params&,
                                                             const Lists&, hipStream_t, int,
                                                             RoundArg, hipEvent_t*);
}  // namespace rbe
