// Stable device radix sort of (u64 key, u32 value) pairs, its own translation
// unit so the rocPRIM/hipCUB instantiation is compiled once.  rbe_wire_ingest
// sorts decoded messages by inbox list with it; a radix sort keeps the stream
// order of equal keys, which is the order a list's messages are handled in.
#include <hipcub/hipcub.hpp>
#include <cstddef>
#include <cstdint>

namespace rbe {
int dev_sort_pairs(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout,
                   const uint32_t* vin, uint32_t* vout, uint64_t n, int end_bit,
                   hipStream_t stream) {
  if (n > 0x7FFFFFFFull) return -1;
  const hipError_t rc = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kin, kout, vin, vout,
                                                           (int)n, 0, end_bit, stream);
  return rc == hipSuccess ? 0 : -1;
}
}  // namespace rbe
