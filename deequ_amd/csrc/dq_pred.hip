// dq_pred.hip -- generic predicate evaluation into row masks.
//
// Spark parses every Compliance predicate and `where` filter with `expr(String)`
// (Compliance.scala:49, Analyzer.scala:413-432) and evaluates it per row with SQL
// three-valued logic.  The fused scan kernel evaluates the common single-comparison forms
// inline; every other predicate of a plan is run here first, once per batch, by a small
// postfix interpreter (the plan's validated dq_pred_insn program).  Each wave evaluates 64
// consecutive rows and writes two 64-bit ballot words: TRUE bits and NOT-NULL bits.  The scan
// kernel then reads those masks (2 bits per row instead of the referenced columns' bytes).
// The interpreter itself (types, three-valued logic, Spark 2.2's casts) is dq_predeval.h, shared
// with the host build the CPU tests check against the oracle.
#include "dq_predeval.h"

namespace dq {

template <bool CAST>
__global__ __launch_bounds__(kBlock) void dq_pred_kernel(const PredProgram* __restrict__ progs,
                                                         const PredInsn* __restrict__ insns,
                                                         const uint8_t* __restrict__ pool,
                                                         const DevColumn* __restrict__ cols,
                                                         int64_t n_rows, uint64_t* out,
                                                         int64_t words_per_mask) {
  const PredProgram prog = progs[blockIdx.y];
  const PredInsn* code = insns + prog.first;
  const int lane = threadIdx.x & 63;
  const int64_t n_words = (n_rows + 63) >> 6;
  uint64_t* out_t = out + (int64_t)(2 * blockIdx.y) * words_per_mask;
  uint64_t* out_n = out_t + words_per_mask;
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < n_words;
       w += (int64_t)gridDim.x * (kBlock / 64)) {
    const int64_t row = (w << 6) + lane;
    bool t = false, nn = false;
    if (row < n_rows) pred::eval_program<CAST>(code, prog.n, pool, cols, row, t, nn);
    const uint64_t bt = __ballot(t);
    const uint64_t bn = __ballot(nn);
    if (lane == 0) {
      out_t[w] = bt;
      out_n[w] = bn;
    }
  }
}

// dst bit i = src bit (bit_offset + i): realigns a sliced Arrow bitmap so that bit 0 of
// byte 0 is row 0 of the batch.
__global__ void dq_realign_kernel(const uint8_t* __restrict__ src, int64_t bit_offset,
                                  int64_t n_bits, uint8_t* __restrict__ dst) {
  const int64_t n_bytes = (n_bits + 7) >> 3;
  const int64_t src_bytes = (bit_offset + n_bits + 7) >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_bytes;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bit = bit_offset + (i << 3);
    const int64_t b = bit >> 3;
    const uint32_t sh = (uint32_t)(bit & 7);
    uint32_t v = src[b] >> sh;
    if (sh && b + 1 < src_bytes) v |= (uint32_t)src[b + 1] << (8 - sh);
    dst[i] = (uint8_t)v;
  }
}

hipError_t launch_predicates(const PredProgram* d_progs, int n_progs, const PredInsn* d_insns,
                             const uint8_t* d_pool, const DevColumn* d_cols, int64_t n_rows,
                             uint64_t* d_mask_words, int64_t words_per_mask, bool with_cast, hipStream_t stream) {
  if (n_progs <= 0 || n_rows <= 0) return hipSuccess;
  const int64_t n_words = (n_rows + 63) >> 6;
  int64_t blocks = (n_words + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  if (with_cast)
    hipLaunchKernelGGL(dq_pred_kernel<true>, dim3((unsigned)blocks, n_progs), dim3(kBlock), 0, stream,
                       d_progs, d_insns, d_pool, d_cols, n_rows, d_mask_words, words_per_mask);
  else
    hipLaunchKernelGGL(dq_pred_kernel<false>, dim3((unsigned)blocks, n_progs), dim3(kBlock), 0, stream,
                       d_progs, d_insns, d_pool, d_cols, n_rows, d_mask_words, words_per_mask);
  return hipGetLastError();
}

// offs[i] -= first: utf8 offsets of a host batch copied verbatim, rebased to its first byte
__global__ void dq_rebase_offsets_kernel(int32_t* __restrict__ offs, int64_t n, int32_t first) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    offs[i] -= first;
}

hipError_t launch_rebase_offsets(int32_t* d_offs, int64_t n, int32_t first, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 1023) / 1024;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_rebase_offsets_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_offs, n, first);
  return hipGetLastError();
}

hipError_t launch_realign_bitmap(const uint8_t* src, int64_t bit_offset, int64_t n_bits,
                                 uint8_t* dst, hipStream_t stream) {
  const int64_t n_bytes = (n_bits + 7) >> 3;
  if (n_bytes <= 0) return hipSuccess;
  int64_t blocks = (n_bytes + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_realign_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src,
                     bit_offset, n_bits, dst);
  return hipGetLastError();
}

}  // namespace dq
