// dq_sort.hip -- rocPRIM primitives of the frequency group-by's sorted-bucket path (dq_freq.hip):
// the radix sort of (slice id, 16-B record) pairs on the id's `bits` bits,
// and the exclusive scan that numbers the aggregation work items.  Kept in its own translation
// unit: rocPRIM's templates dominate its compile time.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dq_internal.h"

namespace dq {

hipError_t sort_freq_records(void* d_tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                             const FreqRec* recs_in, FreqRec* recs_out, uint64_t n, int bits, hipStream_t stream) {
  return rocprim::radix_sort_pairs(d_tmp, tmp_bytes, keys_in, keys_out, recs_in, recs_out, (size_t)n,
                                   0u, (unsigned)bits, stream);
}

hipError_t scan_freq_pieces(void* d_tmp, size_t& tmp_bytes, const uint32_t* pieces, uint32_t* piece_start,
                            uint64_t n, hipStream_t stream) {
  return rocprim::exclusive_scan(d_tmp, tmp_bytes, pieces, piece_start, 0u, (size_t)n, rocprim::plus<uint32_t>(),
                                 stream);
}

}  // namespace dq
