// dq_sort.hip -- the bucket sort of the frequency group-by's sorted-bucket path (dq_freq.hip):
// rocPRIM's device radix sort of (slice id, 16-B record) pairs on the low `bits` key bits.
// Kept in its own translation unit: rocPRIM's templates dominate its compile time.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dq_internal.h"

namespace dq {

hipError_t sort_freq_records(void* d_tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                             const FreqRec* recs_in, FreqRec* recs_out, uint64_t n, int bits, hipStream_t stream) {
  return rocprim::radix_sort_pairs(d_tmp, tmp_bytes, keys_in, keys_out, recs_in, recs_out, (size_t)n, 0u,
                                   (unsigned)bits, stream);
}

}  // namespace dq
