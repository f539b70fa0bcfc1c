// dq_hll.hip -- HLL++ register update for ApproxCountDistinct, bit-exact with deequ.
//
// Reproduces StatefulHyperloglogPlus.update (catalyst/StatefulHyperloglogPlus.scala:89-115):
//   x   = XxHash64Function.hash(v, type, 42)        (Spark 2.2.2 type dispatch)
//   idx = x >>> 55                                   (top p = 9 bits)
//   pw  = numberOfLeadingZeros((x << 9) | 0x100) + 1
//   M[idx] = max(M[idx], pw)
// and the merge (:121-139) = per-register max.  Because max is order-independent the result
// is bitwise identical whatever the block/wave schedule.
//
// Strings and booleans only: numeric columns are hashed inside their value scan (dq_scan.hip).
// Layout: blockIdx.y = HLL task (column, where), blockIdx.x = contiguous row chunk.  Each
// workgroup keeps its 512 registers as u32 in LDS (2 KiB) and updates them with ds_max_u32.  At the end every
// non-zero register is folded into the task's global registers with one atomicMax.  The host
// packs the 512 registers into the 52 Long words of ApproxCountDistinctState.
#include "dq_strhash.h"

namespace dq {

namespace {

__device__ inline void hll_update(uint32_t* regs, uint64_t x) { hll_update_lds(regs, x); }

// A boolean column hashes to one of two values (hashInt(1) / hashInt(0)), so its registers are
// those two updates, made when the workgroup's rows hold a selected true / a selected false:
// 32 rows per lane per step from the value, validity and `where` bitmaps, no per-row hash or
// LDS atomic.  (row_begin is a multiple of kScanRowAlign, so rows map to whole 32-bit words.)
__device__ inline uint32_t bitmap_word(const uint8_t* bm, int64_t row0, int64_t left) {
  const uint8_t* p = bm + (row0 >> 3);
  if (left >= 32) return *reinterpret_cast<const uint32_t*>(p);
  uint32_t v = 0u;  // tail: byte loads, never past ceil(n_rows / 8)
  for (int b = 0; b < (int)((left + 7) >> 3); ++b) v |= (uint32_t)p[b] << (8 * b);
  return v;
}

__device__ void hll_bool(uint32_t* regs, const DevColumn& col, const uint8_t* wt_bm,
                         int64_t row_begin, int64_t row_end) {
  const uint8_t* bits = static_cast<const uint8_t*>(col.values);
  uint32_t any_true = 0u, any_false = 0u;
  for (int64_t row0 = row_begin + (int64_t)threadIdx.x * 32; row0 < row_end; row0 += (int64_t)kBlock * 32) {
    const int64_t left = row_end - row0;
    const uint32_t in = left >= 32 ? 0xffffffffu : ((1u << (uint32_t)left) - 1u);
    uint32_t sel = in;
    if (col.validity) sel &= bitmap_word(col.validity, row0, left);
    if (wt_bm) sel &= bitmap_word(wt_bm, row0, left);
    const uint32_t v = bitmap_word(bits, row0, left);
    any_true |= sel & v;
    any_false |= sel & ~v;
  }
  const bool t = __syncthreads_or(any_true != 0u);
  const bool f = __syncthreads_or(any_false != 0u);
  if (threadIdx.x == 0) {
    if (t) hll_update(regs, xxh64_u32(1u, 42));
    if (f) hll_update(regs, xxh64_u32(0u, 42));
  }
}

// One row per lane: every row is hashed (NULL rows too: their offsets are valid, Arrow), so
// the only divergence is the string length; the register update is the scan kernel's
// unconditional ds_max with rank 0 for a row that is not selected.  (Batching 4 rows per lane
// to put more offset -> bytes loads in flight measured slower: 44.9 vs 40.6 ms on C3-utf8.)
__device__ void hll_utf8(uint32_t* regs, const DevColumn& col, const uint8_t* wt_bm,
                         int64_t row_begin, int64_t row_end) {
  const uint8_t* chars = static_cast<const uint8_t*>(col.values);
  const int32_t* offs = col.offsets;
  for (int64_t row = row_begin + threadIdx.x; row < row_end; row += kBlock) {
    uint32_t sel = col.validity ? (col.validity[row >> 3] >> (row & 7)) & 1u : 1u;
    if (wt_bm) sel &= (wt_bm[row >> 3] >> (row & 7)) & 1u;
    const int32_t b = offs[row];
    const uint32_t len = (uint32_t)(offs[row + 1] - b);
    W64 h;
    if (len < 32) {
      const uint64_t q[2] = {len >= 8 ? ld64(chars + b) : 0ull, len >= 16 ? ld64(chars + b + 8) : 0ull};
      h = xxh64_short_dev(chars + b, len, q);
    } else {
      const uint64_t x = xxh64_bytes(chars + b, (int64_t)len, 42);
      h = {(uint32_t)x ^ (uint32_t)(x >> 32), (uint32_t)(x >> 32)};  // back to the pre-final form
    }
    uint32_t idx, nlz, r;
    hll_slot(h, idx, nlz);
    asm("v_mad_u32_u24 %0, %1, %2, %2" : "=v"(r) : "v"(nlz), "v"(sel));
    __hip_atomic_fetch_max(&regs[idx], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

}  // namespace

__global__ __launch_bounds__(kBlock) void dq_hll_kernel(const HllTask* __restrict__ tasks,
                                                        const DevColumn* __restrict__ cols,
                                                        const DevMask* __restrict__ masks,
                                                        int64_t n_rows, uint32_t* registers) {
  __shared__ uint32_t regs[kHllM];
  const HllTask task = tasks[blockIdx.y];
  for (int r = threadIdx.x; r < kHllM; r += kBlock) regs[r] = 0u;
  __syncthreads();

  const int64_t n_chunks = (n_rows + kScanRowAlign - 1) / kScanRowAlign;
  const int64_t per_block = (n_chunks + gridDim.x - 1) / gridDim.x;
  const int64_t row_begin = min((int64_t)blockIdx.x * per_block * kScanRowAlign, n_rows);
  const int64_t row_end = min(row_begin + per_block * kScanRowAlign, n_rows);
  const DevColumn& col = cols[task.column];
  const uint8_t* wt_bm =
      task.where_mask >= 0 ? reinterpret_cast<const uint8_t*>(masks[task.where_mask].t) : nullptr;

  switch (task.ctype) {
    case DQ_T_BOOL: hll_bool(regs, col, wt_bm, row_begin, row_end); break;
    // (numeric columns are hashed inside their value scan: dq_scan_values_kernel, TF_HLL)
    case DQ_T_UTF8: hll_utf8(regs, col, wt_bm, row_begin, row_end); break;
    default: break;
  }
  __syncthreads();
  uint32_t* out = registers + (int64_t)task.reg_set * kHllM;
  for (int r = threadIdx.x; r < kHllM; r += kBlock) {
    const uint32_t v = regs[r];
    if (v) atomicMax(&out[r], v);
  }
}

hipError_t launch_hll(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols,
                      const DevMask* d_masks, int64_t n_rows, int blocks_per_task,
                      uint32_t* d_registers, hipStream_t stream) {
  if (n_tasks <= 0 || n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_hll_kernel, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream,
                     d_tasks, d_cols, d_masks, n_rows, d_registers);
  return hipGetLastError();
}

}  // namespace dq
