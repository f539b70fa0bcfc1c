// valu_rates.hip -- per-SIMD issue cost of the VALU / LDS instructions the fused scan + HLL hash
// are built from, measured on the card (gfx950).  Each kernel runs 8 independent dependency
// chains of ONE instruction per lane, 8 waves per SIMD (8 blocks of 256 threads per CU), so
// latency is hidden and the number is the SIMD's throughput: cycles per wave-instruction per
// SIMD = elapsed shader cycles / (instructions per wave * waves per SIMD).
// Build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kIters = 2048;
constexpr int kUnroll = 4;  // x 8 chains = 32 instructions per loop iteration

struct Stamp { unsigned long long t0, t1, r0, r1; };

__device__ inline void stamp_begin(Stamp* st, unsigned long long& t0, unsigned long long& r0) {
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  r0 = __builtin_amdgcn_s_memrealtime();
}
__device__ inline void stamp_end(Stamp* st, unsigned long long t0, unsigned long long r0) {
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) st[blockIdx.x] = {t0, t1, r0, r1};
}

// 32-bit chains: a_k = OP(a_k, b)
#define K32(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint32_t b = seed * 3u + 0x9e3779b9u, c = seed + 0x12345u;                                \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                        \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
    if (r == 0x5a5a5a5au) sink[0] = r;                                                        \
  }

// 64-bit chains: a_k = OP(a_k, b)   (b, c 64-bit VGPR pairs)
#define K64(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint64_t b = seed * 3ull + 0x9e3779b97f4a7c15ull, c = seed + 0x123456789ull;              \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                        \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
    if (r == 0x5a5a5a5aull) sink[0] = (uint32_t)r;                                            \
  }

// 64-bit results of 32-bit sources (converts)
#define K64S(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint32_t b = seed * 3u + 0x9e3779b9u, c = seed + 0x12345u;              \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                        \
        asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                        \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
    if (r == 0x5a5a5a5aull) sink[0] = (uint32_t)r;                                            \
  }

// v_mad_u64_u32 writes a 64-bit VGPR pair plus an SGPR-pair carry: its own form.
#define KMAD(NAME, OPC)                                                                     \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint64_t a[8];                                                                            \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) a[k] = threadIdx.x ^ (seed + k);            \
    uint32_t b = seed * 3u + 0x9e3779b9u;                                                     \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        _Pragma("unroll") for (int k = 0; k < 8; ++k) {                                       \
          uint64_t cc;                                                                        \
          asm volatile(OPC " %0, %1, %2, %3, %0" : "+v"(a[k]), "=s"(cc) : "v"((uint32_t)a[k]), "v"(b)); \
        }                                                                                     \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    uint64_t r = 0;                                                                           \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) r ^= a[k];                                  \
    if (r == 0x5a5a5a5aull) sink[0] = (uint32_t)r;                                            \
  }

// VOPC compares write an SGPR pair (no VALU result): chains through a dummy dependency.
#define KCMP(NAME, ASM)                                                                     \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    double a0 = threadIdx.x + seed, b = seed * 0.5;                                           \
    uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;                  \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "=s"(m0) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m1) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m2) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m3) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m4) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m5) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m6) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m7) : "v"(a0), "v"(b));                                       \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint64_t r = m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7;                                 \
    if (r == 0x5a5a5a5aull) sink[0] = (uint32_t)r;                                            \
  }

#define KCMP32(NAME, ASM)                                                                     \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint32_t a0 = threadIdx.x + seed, b = seed * 5u;                                           \
    uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;                  \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "=s"(m0) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m1) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m2) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m3) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m4) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m5) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m6) : "v"(a0), "v"(b));                                       \
        asm volatile(ASM : "=s"(m7) : "v"(a0), "v"(b));                                       \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint64_t r = m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7;                                 \
    if (r == 0x5a5a5a5aull) sink[0] = (uint32_t)r;                                            \
  }


// v_cndmask with VCC / an SGPR-pair mask
#define KSEL(NAME, ASM)                                                                     \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint32_t b = seed * 3u + 0x9e3779b9u;                                                     \
    uint64_t m = __ballot(threadIdx.x & 1);                                                   \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASM : "+v"(a0) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a1) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a2) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a3) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a4) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a5) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a6) : "v"(b), "s"(m));                                        \
        asm volatile(ASM : "+v"(a7) : "v"(b), "s"(m));                                        \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
    if (r == 0x5a5a5a5au) sink[0] = r;                                                        \
  }

// two instructions on separate chains, interleaved A B A B: additive costs mean one pipe
#define KMIX(NAME, ASMA, ASMB)                                                              \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    uint64_t d0 = a0, d1 = a1, d2 = a2, d3 = a3;                                              \
    uint32_t b = seed * 3u + 0x9e3779b9u, c = seed + 0x12345u;                                \
    uint64_t bb = b, cc = c;                                                                  \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll; ++u) {                                   \
        asm volatile(ASMA : "+v"(a0), "+v"(d0) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMB : "+v"(a4), "+v"(d0) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMA : "+v"(a1), "+v"(d1) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMB : "+v"(a5), "+v"(d1) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMA : "+v"(a2), "+v"(d2) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMB : "+v"(a6), "+v"(d2) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMA : "+v"(a3), "+v"(d3) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
        asm volatile(ASMB : "+v"(a7), "+v"(d3) : "v"(b), "v"(c), "v"(bb), "v"(cc));           \
      }                                                                                       \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(d0 ^ d1 ^ d2 ^ d3); \
    if (r == 0x5a5a5a5au) sink[0] = r;                                                        \
  }
// LDS max, no return value, lane-scattered addresses in a 2 KiB register bank (the HLL update)
__global__ __launch_bounds__(256) void k_ds_max_u32(Stamp* st, uint32_t* sink, uint32_t seed) {
  __shared__ uint32_t regs[512];
  for (int r = threadIdx.x; r < 512; r += 256) regs[r] = 0;
  uint32_t x = (threadIdx.x * 2654435761u) ^ seed;
  uint32_t addr[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { x = x * 1664525u + 1013904223u; addr[k] = ((x >> 10) & 511u) * 4u; }
  const uint32_t v = threadIdx.x & 31;
  unsigned long long t0, r0;
  stamp_begin(st, t0, r0);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("ds_max_u32 %0, %1" :: "v"(addr[k]), "v"(v) : "memory");
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  stamp_end(st, t0, r0);
  if (regs[threadIdx.x] == 0x5a5a5a5au) sink[0] = 1;
}

K32(v_add_u32, "v_add_u32 %0, %0, %1")
K32(v_xor_b32, "v_xor_b32 %0, %0, %1")
K32(v_alignbit_b32, "v_alignbit_b32 %0, %0, %1, 7")
K32(v_lshrrev_b32, "v_lshrrev_b32 %0, 3, %0")
K32(v_and_or_b32, "v_and_or_b32 %0, %0, %1, %2")
K32(v_xad_u32, "v_xad_u32 %0, %0, %1, %2")
K32(v_add3_u32, "v_add3_u32 %0, %0, %1, %2")
K32(v_lshl_add_u32, "v_lshl_add_u32 %0, %0, 3, %1")
K32(v_perm_b32, "v_perm_b32 %0, %0, %1, %2")
K32(v_bfe_u32, "v_bfe_u32 %0, %0, 3, 9")
K32(v_ffbh_u32, "v_ffbh_u32 %0, %0")
K32(v_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(v_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K32(v_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
K32(v_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(v_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(v_fma_f32, "v_fma_f32 %0, %0, %1, %2")
K32(v_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
K32(v_dot2_u32_u16, "v_dot2_u32_u16 %0, %0, %1, %2")
K32(v_dot4_u32_u8, "v_dot4_u32_u8 %0, %0, %1, %2")
K32(v_mul_lo_u16, "v_mul_lo_u16 %0, %0, %1")
K32(v_pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %0, %1")
K32(v_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %2")
K32(v_mov_b32_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K64(v_add_f64, "v_add_f64 %0, %0, %1")
K64(v_fma_f64, "v_fma_f64 %0, %0, %1, %2")
K64(v_mul_f64, "v_mul_f64 %0, %0, %1")
K64(v_min_f64, "v_min_f64 %0, %0, %1")
K64(v_lshlrev_b64, "v_lshlrev_b64 %0, 3, %0")
K64(v_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(v_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %2")
K64(v_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
K64(v_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
K64(v_pk_mov_b32, "v_pk_mov_b32 %0, %1, %0 op_sel:[0,1]")
K64S(v_cvt_f64_u32, "v_cvt_f64_u32 %0, %1")
KMAD(v_mad_u64_u32, "v_mad_u64_u32")
KCMP(v_cmp_lt_f64, "v_cmp_lt_f64 %0, %1, %2")
KCMP32(v_cmp_lt_u32, "v_cmp_lt_u32 %0, %1, %2")


K32(v_and_b32, "v_and_b32 %0, %0, %1")
K32(v_or_b32, "v_or_b32 %0, %0, %1")
K32(v_sub_u32, "v_sub_u32 %0, %0, %1")
K32(v_lshlrev_b32, "v_lshlrev_b32 %0, 3, %0")
K32(v_mov_b32, "v_mov_b32 %0, %1")
K32(v_max_u32, "v_max_u32 %0, %0, %1")
K32(v_bcnt_u32_b32, "v_bcnt_u32_b32 %0, %1, %0")
K32(v_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x36")
K32(v_or3_b32, "v_or3_b32 %0, %0, %1, %2")
K32(v_lshl_or_b32, "v_lshl_or_b32 %0, %0, 3, %1")
K32(v_add_f32, "v_add_f32 %0, %0, %1")
K32(v_mul_f32, "v_mul_f32 %0, %0, %1")
K32(v_max_f32, "v_max_f32 %0, %0, %1")
K32(v_xor_lit, "v_xor_b32 %0, 0x12345678, %0")
K32(v_alignbyte_b32, "v_alignbyte_b32 %0, %0, %1, 1")
K32(v_mul_i32_i24, "v_mul_i32_i24 %0, %0, %1")
K32(v_max3_u32, "v_max3_u32 %0, %0, %1, %2")
K32(v_add_u32_e64, "v_add_u32_e64 %0, %0, %1")
K32(v_mix_add_mul, "v_add_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1")
K32(v_mix_add_xor, "v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %2")
K32(v_mix_fma_alignbit, "v_fma_f32 %0, %0, %1, %2\n v_alignbit_b32 %0, %0, %1, 7")
K64S(v_cvt_f64_i32x, "v_cvt_f64_i32 %0, %1")
K64(v_fmac_f64, "v_fmac_f64 %0, %1, %2")
K64(v_max_f64, "v_max_f64 %0, %0, %1")
K64(v_ldexp_f64, "v_ldexp_f64 %0, %0, 3")
KSEL(v_cndmask_vcc, "s_mov_b64 vcc, %2\n v_cndmask_b32 %0, %0, %1, vcc")
KSEL(v_cndmask_e64, "v_cndmask_b32_e64 %0, %0, %1, %2")
KSEL(v_add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
KSEL(v_addc_co_u32, "s_mov_b64 vcc, %2\n v_addc_co_u32 %0, vcc, %0, %1, vcc")
KCMP(v_cmp_class_f64, "v_cmp_class_f64 %0, %1, 3")
KCMP32(v_cmp_ne_u32_e32, "v_cmp_ne_u32 vcc, %1, %2\n s_mov_b64 %0, vcc")
KCMP32(v_cmp_gt_u32_e64, "v_cmp_gt_u32_e64 %0, %1, %2")

KMIX(mx_add_alignbit, "v_add_u32 %0, %0, %2", "v_alignbit_b32 %0, %0, %2, 7")
KMIX(mx_xor_mullo, "v_xor_b32 %0, %0, %2", "v_mul_lo_u32 %0, %0, %2")
KMIX(mx_fma32_alignbit, "v_fma_f32 %0, %0, %2, %3", "v_alignbit_b32 %0, %0, %2, 7")
KMIX(mx_fma32_fma64, "v_fma_f32 %0, %0, %2, %3", "v_fma_f64 %1, %1, %4, %5")
KMIX(mx_add_madu64, "v_add_u32 %0, %0, %2", "v_mad_u64_u32 %1, vcc, %0, %2, %1")
KMIX(mx_alignbit_mullo, "v_alignbit_b32 %0, %0, %2, 7", "v_mul_lo_u32 %0, %0, %2")
KMIX(mx_xor_and, "v_xor_b32 %0, %0, %2", "v_and_b32 %0, %0, %2")
KMIX(mx_bitop3_add64, "v_bitop3_b32 %0, %0, %2, %3 bitop3:0x36", "v_add_f64 %1, %1, %4")
KMIX(mx_add_ffbh, "v_add_u32 %0, %0, %2", "v_ffbh_u32 %0, %0")

__global__ __launch_bounds__(256) void k_mx_ds_alignbit(Stamp* st, uint32_t* sink, uint32_t seed) {
  __shared__ uint32_t regs[512];
  for (int r = threadIdx.x; r < 512; r += 256) regs[r] = 0;
  uint32_t x = (threadIdx.x * 2654435761u) ^ seed;
  uint32_t a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { x = x * 1664525u + 1013904223u; a[k] = x; }
  const uint32_t v = threadIdx.x & 31, b = seed;
  unsigned long long t0, r0;
  stamp_begin(st, t0, r0);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[k]) : "v"(b));
      asm volatile("ds_max_u32 %0, %1" :: "v"((a[u] >> 10) & 2044u), "v"(v) : "memory");
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  stamp_end(st, t0, r0);
  uint32_t r = 0;
  for (int k = 0; k < 8; ++k) r ^= a[k];
  if (regs[threadIdx.x] + r == 0x5a5a5a5au) sink[0] = 1;
}

// Dependent-issue latency: ONE chain per wave (each instruction waits for the previous one), run
// with one wave per SIMD (see main: "lat" rows) -- cycles per instruction = the latency seen by a
// dependent instruction of the same wave.
#define L64(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint64_t a0 = threadIdx.x ^ seed;                                                         \
    uint64_t b = seed * 3ull + 0x9e3779b97f4a7c15ull, c = seed + 0x123456789ull;              \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll * 8; ++u)                                 \
        asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                        \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    if (a0 == 0x5a5a5a5aull) sink[0] = (uint32_t)a0;                                          \
  }
#define L32(NAME, ASM)                                                                      \
  __global__ __launch_bounds__(256) void k_##NAME(Stamp* st, uint32_t* sink, uint32_t seed) { \
    uint32_t a0 = threadIdx.x ^ seed;                                                         \
    uint32_t b = seed * 3u + 0x9e3779b9u, c = seed + 0x12345u;                                \
    unsigned long long t0, r0;                                                                \
    stamp_begin(st, t0, r0);                                                                  \
    for (int i = 0; i < kIters; ++i) {                                                        \
      _Pragma("unroll") for (int u = 0; u < kUnroll * 8; ++u)                                 \
        asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                        \
    }                                                                                         \
    stamp_end(st, t0, r0);                                                                    \
    if (a0 == 0x5a5a5a5au) sink[0] = a0;                                                      \
  }
L64(lat_add_f64, "v_add_f64 %0, %0, %1")
L64(lat_fma_f64, "v_fma_f64 %0, %0, %1, %2")
L64(lat_min_f64, "v_min_f64 %0, %0, %1")
L64(lat_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
L32(lat_add_u32, "v_add_u32 %0, %0, %1")
L32(lat_xor_b32, "v_xor_b32 %0, %0, %1")
L32(lat_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
L32(lat_alignbit_b32, "v_alignbit_b32 %0, %0, %1, 7")
L32(lat_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x36")

typedef void (*KFn)(Stamp*, uint32_t*, uint32_t);
struct Entry { const char* name; KFn fn; };
#define E(n) {#n, k_##n}
static const Entry kEntries[] = {
  E(v_add_u32), E(v_xor_b32), E(v_alignbit_b32), E(v_lshrrev_b32), E(v_and_or_b32), E(v_xad_u32),
  E(v_add3_u32), E(v_lshl_add_u32), E(v_perm_b32), E(v_bfe_u32), E(v_ffbh_u32), E(v_mul_lo_u32),
  E(v_mul_hi_u32), E(v_mul_u32_u24), E(v_mul_hi_u32_u24), E(v_mad_u32_u24), E(v_fma_f32),
  E(v_cvt_f32_u32), E(v_dot2_u32_u16), E(v_dot4_u32_u8), E(v_mul_lo_u16), E(v_pk_mul_lo_u16),
  E(v_pk_mad_u16), E(v_mov_b32_dpp), E(v_add_f64), E(v_fma_f64), E(v_mul_f64), E(v_min_f64),
  E(v_lshlrev_b64), E(v_lshl_add_u64), E(v_pk_fma_f32), E(v_pk_add_f32), E(v_pk_mul_f32),
  E(v_pk_mov_b32), E(v_cvt_f64_u32), E(v_mad_u64_u32), E(v_cmp_lt_f64), E(v_cmp_lt_u32),
  E(ds_max_u32),
  E(mx_add_alignbit),
  E(mx_xor_mullo),
  E(mx_fma32_alignbit),
  E(mx_fma32_fma64),
  E(mx_add_madu64),
  E(mx_alignbit_mullo),
  E(mx_xor_and),
  E(mx_bitop3_add64),
  E(mx_add_ffbh),
  E(mx_ds_alignbit),
  E(v_and_b32),
  E(v_or_b32),
  E(v_sub_u32),
  E(v_lshlrev_b32),
  E(v_mov_b32),
  E(v_max_u32),
  E(v_bcnt_u32_b32),
  E(v_bitop3_b32),
  E(v_or3_b32),
  E(v_lshl_or_b32),
  E(v_add_f32),
  E(v_mul_f32),
  E(v_max_f32),
  E(v_xor_lit),
  E(v_alignbyte_b32),
  E(v_mul_i32_i24),
  E(v_max3_u32),
  E(v_add_u32_e64),
  E(v_mix_add_mul),
  E(v_mix_add_xor),
  E(v_mix_fma_alignbit),
  E(v_cvt_f64_i32x),
  E(v_fmac_f64),
  E(v_max_f64),
  E(v_ldexp_f64),
  E(v_cndmask_vcc),
  E(v_cndmask_e64),
  E(v_add_co_u32),
  E(v_addc_co_u32),
  E(v_cmp_class_f64),
  E(v_cmp_ne_u32_e32),
  E(v_cmp_gt_u32_e64),
};

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
  Stamp* d_st;
  uint32_t* d_sink;
  CHK(hipMalloc(&d_st, sizeof(Stamp) * blocks));
  CHK(hipMalloc(&d_sink, 64));
  std::vector<Stamp> st(blocks);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double insts_per_wave = (double)kIters * kUnroll * 8;
  printf("{\"cus\": %d, \"blocks\": %d, \"waves_per_simd\": 8, \"insts_per_wave\": %.0f, \"rows\": [\n", cus, blocks,
         insts_per_wave);
  bool first = true;
  for (const Entry& en : kEntries) {
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms the clock up
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(en.fn, dim3(blocks), dim3(256), 0, 0, d_st, d_sink, 7u + rep);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
    }
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(st.data(), d_st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost));
    std::vector<double> cyc(blocks), clk(blocks);
    for (int b = 0; b < blocks; ++b) {
      cyc[b] = (double)(st[b].t1 - st[b].t0);
      clk[b] = cyc[b] / ((double)(st[b].r1 - st[b].r0) / 100e6) / 1e9;  // GHz
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(clk.begin(), clk.end());
    const double med_cyc = cyc[blocks / 2];
    // per SIMD: 8 waves each ran insts_per_wave instructions inside med_cyc cycles
    const double cpi = med_cyc / (insts_per_wave * 8.0);
    // chip-wide from wall time: wave-instructions / (SIMDs * seconds * clock)
    const double wave_insts = insts_per_wave * blocks * 4.0;
    const double cpi_wall = (ms * 1e-3) * clk[blocks / 2] * 1e9 * (cus * 4.0) / wave_insts;
    printf("%s  {\"insn\": \"%s\", \"cyc_per_wave_insn_per_simd\": %.3f, \"wall_based\": %.3f, \"ghz\": %.3f, \"ms\": %.3f}",
           first ? "" : ",\n", en.name, cpi, cpi_wall, clk[blocks / 2], ms);
    first = false;
  }
  printf("\n], \"latency\": [\n");
  // one wave per SIMD (64-thread blocks, 4 per CU), one dependency chain per wave
  static const Entry kLat[] = {E(lat_add_f64), E(lat_fma_f64), E(lat_min_f64), E(lat_lshl_add_u64), E(lat_add_u32),
                               E(lat_xor_b32), E(lat_mul_lo_u32), E(lat_alignbit_b32), E(lat_bitop3_b32)};
  const int lblocks = cus * 4;
  first = true;
  for (const Entry& en : kLat) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(en.fn, dim3(lblocks), dim3(64), 0, 0, d_st, d_sink, 7u + rep);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(st.data(), d_st, sizeof(Stamp) * lblocks, hipMemcpyDeviceToHost));
    std::vector<double> cyc(lblocks);
    for (int b = 0; b < lblocks; ++b) cyc[b] = (double)(st[b].t1 - st[b].t0);
    std::sort(cyc.begin(), cyc.end());
    printf("%s  {\"insn\": \"%s\", \"dependent_cycles\": %.3f}", first ? "" : ",\n", en.name,
           cyc[lblocks / 2] / insts_per_wave);
    first = false;
  }
  printf("\n]}\n");
  return 0;
}
