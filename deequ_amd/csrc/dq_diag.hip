// dq_diag.hip -- the VALU ceiling of the HLL hot loop, measured on the card it runs on.
//
// ApproxCountDistinct costs, per row, one Spark XXH64 of the value (StatefulHyperloglogPlus
// .scala:93): five 64x64-bit multiplies, each one v_mad_u64_u32 + two v_mul_lo_u32 on gfx950,
// all quarter-rate VALU ops, plus ~25 full-rate shifts / xors / adds, then the register index,
// rank and LDS max (:96-113).  Once the hash is in the same pass as the HBM stream, the pass
// is bounded by that VALU work, not by the bytes.  This kernel runs exactly that per-row
// work with no memory traffic (each lane feeds its hash back as the next value, 4 independent
// chains per lane) so bench.py can price the HLL kernels against the hash rate the card
// actually sustains, next to the 8 TB/s HBM roofline.
#include "dq_internal.h"

namespace dq {

template <bool WITH_HLL>
__global__ __launch_bounds__(kBlock) void dq_diag_hash_kernel(int iters, uint64_t* sink) {
  __shared__ uint32_t lregs[kHllM];
  if (WITH_HLL) {
    for (int r = threadIdx.x; r < kHllM; r += kBlock) lregs[r] = 0u;
    __syncthreads();
  }
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint64_t x[4] = {t * 4 + 1, t * 4 + 2, t * 4 + 3, t * 4 + 4};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // the scan kernel's per-row hash + register update
      const W64 h = spark_hash_dev<int64_t>((int64_t)x[c]);
      const W64 f = xxh64_final(h);
      x[c] = ((uint64_t)f.hi << 32) | f.lo;
      if (WITH_HLL) {
        uint32_t idx, nlz;
        hll_slot(h, idx, nlz);
        __hip_atomic_fetch_max(&lregs[idx], nlz + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  uint64_t acc = x[0] ^ x[1] ^ x[2] ^ x[3];
  if (WITH_HLL) {
    __syncthreads();
    acc += lregs[threadIdx.x];
  }
  if (acc == 0x5a5a5a5a5a5a5a5aull) sink[0] = acc;  // keeps the chains live; never true in practice
}

hipError_t launch_diag_hash(int blocks, int iters, bool with_hll, uint64_t* sink, hipStream_t s) {
  if (with_hll)
    hipLaunchKernelGGL((dq_diag_hash_kernel<true>), dim3(blocks), dim3(kBlock), 0, s, iters, sink);
  else
    hipLaunchKernelGGL((dq_diag_hash_kernel<false>), dim3(blocks), dim3(kBlock), 0, s, iters, sink);
  return hipGetLastError();
}

}  // namespace dq
