// dq_scan_fast.hip -- the fused value scan specialised for the common task shape: one 8-byte
// column (LongType / DoubleType), no `where` filter, at most one inline `column CMP literal`
// Compliance predicate, any of Size / Completeness / Sum / Mean / StandardDeviation / Minimum /
// Maximum and ApproxCountDistinct of that column.  Same semantics and the same ScanAcc partials
// as dq_scan_values_kernel (dq_scan.hip, which stays the general path); the reference job it
// replaces is AnalysisRunner.runScanningAnalyzers' single data.agg (AnalysisRunner.scala:306-313)
// plus StatefulHyperloglogPlus.update (StatefulHyperloglogPlus.scala:89-115).
//
// Why a second kernel.  With ApproxCountDistinct fused in, the pass is bound by VALU issue, not
// by HBM.  Measured on gfx950 (tools/ubench/valu_rates.hip, 8 waves per SIMD), a wave64 VALU
// instruction costs the SIMD ~2.3 cycles for add/sub/and/or/xor/lshr/bitop3/fma_f32 and ~4.2
// for nearly everything else (64-bit ops, multiplies, alignbit, compares, conversions,
// cndmask).  So this kernel is written for the fewest *weighted* issue cycles per row:
//   * NULL rows are neutralised once, not per statistic: a row that is not selected takes the
//     wave's shift value c (the first valid value the wave saw) through ONE bitop3 per 32-bit
//     word, `xm = valid ? x : c`.  c is itself a selected value of the column, so
//       - Min / Max and the HLL registers are unchanged by extra copies of c (min, max and the
//         register max are idempotent), no masking needed;
//       - d = xm - c is exactly 0 for those rows, so Σd, Σd² (StdDev moments) need no masking;
//       - the wrapping int64 sum and the predicate count are corrected once per wave:
//         Σ_sel x = Σ xm - n_unsel·c,  Σ_sel pred(x) = Σ pred(xm) - n_unsel·pred(c).
//     A wave that finds no valid value to use as c (a NULL-heavy chunk) runs the masked form of
//     the same loop (NaN for min/max, rank 0 for HLL) instead.
//   * the predicate is one v_cmp per row whose mask is counted on the scalar unit (s_bcnt1); the
//     host rewrites every operator to `x < lit` or `x == lit`, optionally negated:
//     x <= l  ==  x < l+1 (int) / x < nextafter(l, +inf) (fp);  x > l  ==  !(x <= l);
//     x >= l  ==  !(x < l);  x != l  ==  !(x == l)  -- a NaN x lands above every literal, as in
//     Spark's NaN-safe order;
//   * the HLL rank is ffbh of the top word of (x << 9), ONE alignbit away from the hash halves:
//     the only row it cannot rank (that top word all zero, 1 hash in 2^32) is stored as the
//     marker 0xFFFFFFFF (saturating +1), and a workgroup whose registers hold the marker
//     re-ranks those registers exactly over its own rows before folding them (no per-row cost).
#include "dq_scan_common.h"

namespace dq {

namespace {

enum FastPK : int { PK_NONE = 0, PK_LT_I = 1, PK_EQ_I = 2, PK_LT_F = 3, PK_EQ_F = 4 };

constexpr uint32_t kRankMarker = 0xFFFFFFFFu;  // a row whose rank is >= 33 (see hll_rank_fast)

// (x & m) | (c & ~m): one v_bitop3_b32 (the compiler picks the half-rate v_bfi_b32 for it).
// bitop3's table is indexed like vpternlog: S0 = 0xF0, S1 = 0xCC, S2 = 0xAA -> 0xE2.
__device__ inline uint32_t sel32(uint32_t x, uint32_t m, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe2" : "=v"(r) : "v"(x), "v"(m), "v"(c));
  return r;
}

// int64 -> double, correctly rounded: cvt(hi) * 2^32 + cvt(lo) as one fma
__device__ inline double i64_to_f64(uint32_t lo, uint32_t hi) {
  return fma((double)(int32_t)hi, 0x1p32, (double)lo);
}

__device__ inline double uniform_f64(double v) {  // a wave-uniform double into SGPRs
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The register update in min form: a register's rank is nlz(w) + 1 of its
// smallest w = (x << 9) | W_PADDING, so the workgroup keeps, per register, the MINIMUM of
// s = bits 54..24 of x (in bits 30..0; one alignbit and one and from the hash halves) with
// ds_min_u32, and turns it into a rank once, when folding: rank = nlz32(s) for s != 0 (s = 0:
// rank >= 32, the exact re-rank below).  No per-row v_ffbh and +1 (the max form measured
// 12.94 vs 12.93 ms on C2: kept for the shorter instruction stream).
// An untouched register keeps 0xFFFFFFFF, which no s reaches (bit 31 is clear).
__device__ inline void hll_key_min(W64 h, uint32_t& byte_off, uint32_t& s) {
  byte_off = (h.hi >> 21) & 0x7fcu;
  const uint32_t xlo = h.lo ^ h.hi;
  s = __builtin_amdgcn_alignbit(h.hi, xlo, 24) & 0x7fffffffu;
}
__device__ inline uint32_t hll_min_to_rank(uint32_t s) {
  if (s == 0xFFFFFFFFu) return 0u;
  return s ? (uint32_t)__builtin_clz(s) : kRankMarker;
}

// The exact rank of the same row (64-bit leading-zero count), for the marker re-rank.
__device__ inline uint32_t hll_rank_exact(W64 h) {
  const W64 x = xxh64_final(h);
  const uint64_t w = ((((uint64_t)x.hi << 32) | x.lo) << 9) | kHllWPadding;
  return (uint32_t)__clzll((long long)w) + 1u;
}

// x != x for the rare NaN paths: volatile, so the compiler cannot hoist the compare out of the
// wave-uniform branch that guards it into the hot loop.
__device__ inline bool is_nan_rare(double x) {
  uint32_t r;
  asm volatile("v_cmp_u_f64 vcc, %1, %1\n\tv_cndmask_b32 %0, 0, 1, vcc" : "=v"(r) : "v"(x) : "vcc");
  return r != 0u;
}

__device__ inline void lds_min(uint32_t* regs, uint32_t byte_off, uint32_t v) {
  __hip_atomic_fetch_min(reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(regs) + byte_off), v,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a * C + A (mod 2^64) on 32-bit halves with the cross terms as mul_lo -> mad_u64 (the mad adds
// the first cross term as its 64-bit addend, whose low half is a scratch register) -> add, i.e.
// v_mad_u64_u32 + v_mul_lo_u32 + v_mad_u64_u32 + v_add_u32 instead of the compiler's
// v_mad_u64_u32 + 2 v_mul_lo_u32 + v_add3_u32 (one full-rate add in place of a half-rate add3).
template <uint64_t C, uint64_t A = 0>
__device__ inline W64 w64_mul_fast(W64 a) {
  const uint64_t p = (uint64_t)a.lo * (uint32_t)C + A;
  uint32_t hi;
  asm("v_mul_lo_u32 v2, %1, %2\n\t"
      "v_mad_u64_u32 v[2:3], vcc, %3, %4, v[2:3]\n\t"
      "v_add_u32 %0, v2, %5"
      : "=v"(hi)
      : "v"(a.lo), "s"((uint32_t)(C >> 32)), "v"(a.hi), "s"((uint32_t)C), "v"((uint32_t)(p >> 32))
      : "v2", "v3", "vcc");
  return {(uint32_t)p, hi};
}

// xxh64_8_dev (dq_internal.h) with the multiplies above: Spark XXH64.hashLong, seed 42, the hash
// before its final h ^= h >> 32.
__device__ inline W64 xxh64_8_fast(uint32_t lo, uint32_t hi) {
  constexpr uint64_t RS = rotl64_c(42ull + kP5 + 8, 27);
  W64 k = w64_mul_fast<kP2>({lo, hi});
  k = w64_mul_fast<kP1>(w64_rotl<31>(k));
  W64 h = w64_rotl<27>(k);
  h.lo ^= (uint32_t)RS;
  h.hi ^= (uint32_t)(RS >> 32);
  h = w64_mul_fast<kP1, kP4>(h);
  h.lo ^= h.hi >> 1;                                   // h ^= h >> 33
  h = w64_mul_fast<kP2>(h);
  h.lo ^= __builtin_amdgcn_alignbit(h.hi, h.lo, 29);  // h ^= h >> 29
  h.hi ^= h.hi >> 29;
  return w64_mul_fast<kP3>(h);
}

template <typename T>
__device__ inline W64 hash_halves(uint32_t lo, uint32_t hi) {
  return xxh64_8_fast(lo, hi);  // LongType: hashLong; DoubleType: doubleToLongBits (canonical NaN upstream)
}

// Per-lane accumulators of the fast kernel.
struct FastAcc {
  uint32_t n_sel;      // selected rows (lane)
  uint32_t n_rows;     // rows visited (lane)
  uint64_t isum;       // Σ xm, wrapping (int64 columns)
  double s1, s2;       // Σd, Σd² with d = xm - c
  double fs, fc;       // compensated Σxm (fp64): the Sum, stand-ins included (removed at the end)
  double fmin, fmax;   // fp64: of x; int64: of d = x - c (exact, see fast_row), x = d + c at the end
  uint64_t pc;         // wave-uniform: Σ over visited rows of cmp(xm) (before negation)
};

constexpr uint64_t kMagic = 0x4338000000000000ull;  // 1.5 * 2^52 as a double


// One row: xm already neutralised (selected value or the shift).  MEMBER = the shift is a
// selected value (masking not needed); otherwise `m` (0 / ~0) masks min/max and the HLL rank.
// int64 statistics: for |x| < 2^51 the bits of xm + K (K = 1.5 * 2^52 as a double) ARE the
// double 1.5 * 2^52 + x, so d = x - c is one 64-bit integer add and one exact fp64 subtract of
// the constant cshift = 1.5 * 2^52 + c (no int64 -> double conversion).  An |x| >= 2^51 leaves
// the bits outside [2^52, 2^53), so its d is NaN, infinite or at least 2^51 - |c| > 2^50 away from
// 0 (|c| < 2^50): the workgroup sees it in min / max / Σd² at the end and redoes its statistics
// with EXACT (the conversion).
template <typename T, int PK, bool STATS, bool HLL, bool MEMBER, bool EXACT = false>
__device__ inline void fast_row(FastAcc& a, uint32_t lo, uint32_t hi, uint32_t m, double shift, double cshift,
                                double& dsum, int64_t lit_i, double lit_f, uint32_t* lregs, bool nan_possible) {
  constexpr bool INT = sizeof(T) == 8 && !__is_same(T, double);
  double xd = 0.0;
  if constexpr (INT) {
    if constexpr ((STATS && EXACT) || PK == PK_LT_F || PK == PK_EQ_F) xd = i64_to_f64(lo, hi);
  } else {
    xd = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  }
  if constexpr (STATS) {
    double d, xn;
    if constexpr (INT && !EXACT) {
      const uint64_t xm = ((uint64_t)hi << 32) | lo;
      a.isum += xm;
      const uint64_t bm = xm + kMagic;
      d = __builtin_bit_cast(double, bm) - cshift;
      xn = d;  // min / max of d
    } else {
      if constexpr (INT) a.isum += ((uint64_t)hi << 32) | lo;
      d = xd - shift;
      a.s1 += d;
      // fp64 Sum from the raw values (compensated per iteration by the caller), not from
      // n * c + Σd: x - c rounds when |x| >> |c|, and [1e308, -1e308, 5] must sum to 5
      if constexpr (!INT) dsum += xd;
      xn = xd;
    }
    a.s2 = fma(d, d, a.s2);
    if constexpr (!MEMBER) {  // a quiet NaN for an unselected row: v_min/v_max drop it
      const uint64_t xb = __builtin_bit_cast(uint64_t, xn);
      const uint32_t xh = sel32((uint32_t)(xb >> 32), m, 0x7ff80000u);
      xn = __builtin_bit_cast(double, ((uint64_t)xh << 32) | (uint32_t)xb);
    }
    a.fmin = vmin_f64(a.fmin, xn);
    a.fmax = vmax_f64(a.fmax, xn);
  }
  if constexpr (PK != PK_NONE) {
    bool c;
    if constexpr (PK == PK_LT_I) c = (int64_t)(((uint64_t)hi << 32) | lo) < lit_i;
    else if constexpr (PK == PK_EQ_I) c = (int64_t)(((uint64_t)hi << 32) | lo) == lit_i;
    else if constexpr (PK == PK_LT_F) c = xd < lit_f;
    else c = xd == lit_f;
    a.pc += __builtin_popcountll(__ballot(c));
  }
  if constexpr (HLL) {
    uint32_t hlo = lo, hhi = hi;
    if constexpr (!INT) {
      // Double.doubleToLongBits: every NaN hashes as the canonical one (rare: wave-uniform)
      if (nan_possible && is_nan_rare(xd)) {
        hlo = 0u;
        hhi = 0x7ff80000u;
      }
    }
    uint32_t off, s;
    hll_key_min(hash_halves<T>(hlo, hhi), off, s);
    if constexpr (!MEMBER) s |= ~m;  // an unselected row leaves the minimum alone
    lds_min(lregs, off, s);
  }
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#ifndef DQ_FAST_UNROLL
#define DQ_FAST_UNROLL 4
#endif
#ifndef DQ_FAST_WAVES
#define DQ_FAST_WAVES 1  // amdgpu_waves_per_eu minimum (register budget: 8 -> 64 VGPRs, 6 -> 80)
#endif
// The validity bytes keep the default policy: a 128-B bitmap line serves 1024 rows, i.e. eight
// wave-instructions of one workgroup, and read non-temporally it is fetched about twice (the
// known-bytes probes, tools/ubench/traffic_probe.hip: 0.508 vs 0.501 of the bytes; C2's PMC
// reads 33.3 -> 32.5 GB per launch, exactly the algorithmic bytes).
#ifndef DQ_VALID_AUX
#define DQ_VALID_AUX 0
#endif
constexpr int kFastUnroll = DQ_FAST_UNROLL;  // 16-byte loads (2 rows) per lane per iteration

// Streaming loads of a large pass go non-temporal (aux = 2: the bytes are read once and are far
// larger than the 256 MiB Infinity Cache; A/B 13.11 vs 13.22 ms on C2); a small table (C1's 10M
// rows) keeps the default policy, so a repeated pass over it is served from the Infinity Cache
// (nt there doubled C1's step, 0.5 -> 1.0 ms).
constexpr int64_t kNtMinRows = (int64_t)1 << 24;  // 128 MiB of 8-byte values per column
// The loads of iteration `it`: 4 x 16 B of values and the 4 validity bytes of the same rows.
// (Counting the selected rows from 16-byte bitmap words on the scalar unit instead of one VALU
// op per row measured slower: the words cost SGPRs and VGPRs, i.e. occupancy.)
struct FastLoad {
  v4u vec[kFastUnroll];
  uint32_t vb[kFastUnroll];
};

__device__ inline void fast_load(FastLoad& L, __amdgpu_buffer_rsrc_t rv, __amdgpu_buffer_rsrc_t rvalid, uint32_t it,
                                 bool nt) {
  constexpr uint32_t ROWS_PER_ITER = (uint32_t)kBlock * 2 * kFastUnroll;
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < kFastUnroll; ++u) {
    // (a load past the chunk -- the pipelined form's look-ahead -- reads 0 through the
    // descriptor's range check and is never used)
    const uint32_t r0 = it * ROWS_PER_ITER + ((uint32_t)u * kBlock + tid) * 2u;
    if (nt) {  // (wave-uniform)
      L.vec[u] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(r0 * 8u), 0, 2);
      L.vb[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rvalid, (int)(r0 >> 3), 0, DQ_VALID_AUX);
    } else {
      L.vec[u] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(r0 * 8u), 0, 0);
      L.vb[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rvalid, (int)(r0 >> 3), 0, 0);
    }
  }
}

template <typename T, int PK, bool STATS, bool HLL, bool MEMBER>
__device__ inline void fast_compute(FastAcc& a, const FastLoad& L, uint32_t no_valid, uint32_t sh_lo, uint32_t sh_hi,
                                    double shift, double cshift, int64_t lit_i, double lit_f, uint32_t* lregs,
                                    uint32_t* s_nan) {
  constexpr int UNROLL = kFastUnroll;
  constexpr bool FP = __is_same(T, double);
  const uint32_t bp = (threadIdx.x * 2u) & 7u;  // bit of the lane's first row in its validity byte
  uint32_t lo[UNROLL * 2], hi[UNROLL * 2], m[UNROLL * 2];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const uint32_t bits = L.vb[u] | no_valid;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = u * 2 + k;
      m[j] = (uint32_t)__builtin_amdgcn_sbfe((int32_t)bits, bp + (uint32_t)k, 1);
      lo[j] = sel32(L.vec[u][2 * k], m[j], sh_lo);
      hi[j] = sel32(L.vec[u][2 * k + 1], m[j], sh_hi);
      a.n_sel -= m[j];
    }
  }
  double dsum = -0.0;
  // statistics + predicate of all rows first: for fp64 the iteration's Σx tells whether a
  // selected NaN is present (it would be NaN), which the hash needs to know
#pragma unroll
  for (int j = 0; j < UNROLL * 2; ++j)
    fast_row<T, PK, STATS, false, MEMBER>(a, lo[j], hi[j], m[j], shift, cshift, dsum, lit_i, lit_f, lregs, false);
  bool nan_possible = false;
  if constexpr (FP && !STATS && HLL) {  // no Σd to look at: one ordered compare per row
    bool any = false;
#pragma unroll
    for (int j = 0; j < UNROLL * 2; ++j) {
      const double x = __builtin_bit_cast(double, ((uint64_t)hi[j] << 32) | lo[j]);
      any = any || (x != x);
    }
    nan_possible = __ballot(any) != 0;
  }
  if constexpr (FP && STATS) {
    nan_possible = __ballot(dsum != dsum) != 0;
    if (nan_possible) {  // rare; the flag lives in LDS so this stays a branch
#pragma unroll
      for (int j = 0; j < UNROLL * 2; ++j) {
        const double x = __builtin_bit_cast(double, ((uint64_t)hi[j] << 32) | lo[j]);
        if (m[j] && is_nan_rare(x)) *s_nan = 1u;
      }
    }
    neumaier_add(a.fs, a.fc, dsum);
  }
  if constexpr (HLL) {
    double unused = 0.0;
    if (FP && nan_possible) {  // wave-uniform and rare: the canonical-NaN form of the hash loop
#pragma unroll
      for (int j = 0; j < UNROLL * 2; ++j)
        fast_row<T, PK_NONE, false, true, MEMBER>(a, lo[j], hi[j], m[j], shift, cshift, unused, lit_i, lit_f, lregs, true);
    } else {
#pragma unroll
      for (int j = 0; j < UNROLL * 2; ++j)
        fast_row<T, PK_NONE, false, true, MEMBER>(a, lo[j], hi[j], m[j], shift, cshift, unused, lit_i, lit_f, lregs, false);
    }
  }
}

template <typename T, int PK, bool STATS, bool HLL, bool MEMBER>
__device__ inline void fast_main_loop(FastAcc& a, __amdgpu_buffer_rsrc_t rv, __amdgpu_buffer_rsrc_t rvalid,
                                      uint32_t no_valid, uint32_t full_iters, uint32_t sh_lo, uint32_t sh_hi,
                                      double shift, double cshift, int64_t lit_i, double lit_f, uint32_t* lregs,
                                      uint32_t* s_nan, bool nt) {
  // two-stage pipeline: iteration it + 1's loads are in flight while iteration it computes
  // (two register sets, the loop unrolled by two so no copies are needed)
  FastLoad A, B;
  uint32_t it = 0;
  if (full_iters > 0) fast_load(A, rv, rvalid, 0, nt);
#pragma unroll 1
  for (; it + 1 < full_iters; it += 2) {
    fast_load(B, rv, rvalid, it + 1, nt);
    fast_compute<T, PK, STATS, HLL, MEMBER>(a, A, no_valid, sh_lo, sh_hi, shift, cshift, lit_i, lit_f, lregs, s_nan);
    fast_load(A, rv, rvalid, it + 2, nt);
    fast_compute<T, PK, STATS, HLL, MEMBER>(a, B, no_valid, sh_lo, sh_hi, shift, cshift, lit_i, lit_f, lregs, s_nan);
  }
  if (it < full_iters) fast_compute<T, PK, STATS, HLL, MEMBER>(a, A, no_valid, sh_lo, sh_hi, shift, cshift, lit_i, lit_f, lregs, s_nan);
  a.n_rows += full_iters * kFastUnroll * 2;
}

// The ragged end of the chunk (first = full_iters * 2048), or -- with EXACT, HLL off -- the
// whole chunk again: one row per lane.
template <typename T, int PK, bool STATS, bool HLL, bool MEMBER, bool EXACT = false>
__device__ inline void fast_tail(FastAcc& a, __amdgpu_buffer_rsrc_t rv, __amdgpu_buffer_rsrc_t rvalid,
                                 uint32_t no_valid, uint32_t first, uint32_t span, uint32_t sh_lo, uint32_t sh_hi,
                                 double shift, double cshift, int64_t lit_i, double lit_f, uint32_t* lregs,
                                 uint32_t* s_nan) {
  double dsum = 0.0;
  for (uint32_t r = first + threadIdx.x; r < span; r += kBlock) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rv, (int)(r * 8u), 0, 0);
    const uint32_t bit = (((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rvalid, (int)(r >> 3), 0, 0) | no_valid) >>
                          (r & 7u)) & 1u;
    const uint32_t m = 0u - bit;
    const uint32_t lo = sel32((uint32_t)v[0], m, sh_lo), hi = sel32((uint32_t)v[1], m, sh_hi);
    a.n_sel += bit;
    a.n_rows += 1;
    fast_row<T, PK, STATS, false, MEMBER, EXACT>(a, lo, hi, m, shift, cshift, dsum, lit_i, lit_f, lregs, false);
    if constexpr (__is_same(T, double) && STATS) {
      const double x = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
      if (bit && x != x) *s_nan = 1u;
    }
    if constexpr (HLL) {
      double unused = 0.0;
      fast_row<T, PK_NONE, false, true, MEMBER>(a, lo, hi, m, shift, cshift, unused, lit_i, lit_f, lregs, true);
    }
  }
  if constexpr (__is_same(T, double) && STATS) neumaier_add(a.fs, a.fc, dsum);
}

__device__ inline void fast_acc_init(FastAcc& a) {
  a.n_sel = a.n_rows = 0u;
  a.isum = 0u;
  a.s1 = a.s2 = 0.0;
  a.fs = a.fc = 0.0;
  a.fmin = __builtin_huge_val();
  a.fmax = -__builtin_huge_val();
  a.pc = 0u;
}

}  // namespace

// Diagnostic build only (-DDQ_SCAN_DIAG): how often a workgroup re-reads its chunk -- the exact
// int64 statistics, the moments' cancellation guard, the HLL marker re-rank -- of all workgroups
// (printed per launch by launch_scan_fast).  The re-reads are the only reads beyond one pass.
#ifdef DQ_SCAN_DIAG
__device__ unsigned long long g_scan_diag[4];
#define DQ_SCAN_COUNT(i) do { if (threadIdx.x == 0) atomicAdd(&g_scan_diag[i], 1ull); } while (0)
#else
#define DQ_SCAN_COUNT(i) do { } while (0)
#endif

template <typename T, int PK, bool STATS, bool HLL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DQ_FAST_WAVES))) void dq_scan_fast_kernel(const ScanTask* __restrict__ tasks,
                                                              const int32_t* __restrict__ group,
                                                              const DevColumn* __restrict__ cols, int64_t n_rows,
                                                              ScanAcc* partials, uint32_t* __restrict__ hll_regs) {
  constexpr bool FP = __is_same(T, double);
  constexpr bool INT_STATS = !FP && STATS;
  const ScanTask& task = tasks[group[blockIdx.y]];
  int64_t row_begin, row_end;
  chunk_of_block(n_rows, row_begin, row_end);
  const bool nt = n_rows >= kNtMinRows;
  const uint32_t span = (uint32_t)(row_end - row_begin);  // host keeps span * 8 < 4 GiB
  __shared__ uint32_t lregs[kHllM];
  __shared__ uint32_t lflag[kHllM / 32];
  __shared__ uint32_t s_nan;  // a selected NaN seen (fp64 statistics)
  if constexpr (HLL) {
    for (int r = threadIdx.x; r < kHllM; r += kBlock) lregs[r] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) s_nan = 0u;
  __syncthreads();
  const DevColumn& col = cols[task.primary];
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(static_cast<const uint64_t*>(col.values) + row_begin, span * 8u);
  const bool has_valid = col.validity != nullptr;
  const uint32_t no_valid = has_valid ? 0u : 0xffu;
  const __amdgpu_buffer_rsrc_t rvalid =
      make_rsrc(has_valid ? col.validity + (row_begin >> 3) : nullptr, has_valid ? (span + 7u) >> 3 : 0u);
  int64_t lit_i = 0;
  double lit_f = 0.0;
  bool inv = false;
  if constexpr (PK != PK_NONE) {
    lit_i = task.preds[0].lit_i;
    lit_f = task.preds[0].lit_f;
    inv = (task.preds[0].cmp_sel & CS_INV) != 0;
  }

  // The wave's stand-in c: the first valid (finite, for fp) value among its first rows.  For
  // int64 statistics it must also satisfy |c| < 2^51 (the magic-number form); otherwise c = 0 and
  // the wave runs the masked loop.
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  uint32_t sh_lo = 0u, sh_hi = 0u;
  uint32_t any_lo = 0u, any_hi = 0u;  // the first valid value of any magnitude (exact int64 re-run)
  bool member = false, found_any = false;
  for (uint32_t probe = 0; probe < 8; ++probe) {
    const uint32_t r = (probe * (kBlock / 64) + wave) * 64u + lane;
    bool ok = false, okv = false;
    uint32_t vlo = 0u, vhi = 0u;
    if (r < span) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rv, (int)(r * 8u), 0, 0);
      vlo = (uint32_t)v[0];
      vhi = (uint32_t)v[1];
      const uint32_t bit = (((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rvalid, (int)(r >> 3), 0, 0) |
                             no_valid) >> (r & 7u)) & 1u;
      okv = bit != 0u;
      if (FP) {
        const double x = __builtin_bit_cast(double, ((uint64_t)vhi << 32) | vlo);
        // (finite and not near DBL_MAX: x - c must not overflow for values of the other sign)
        okv = okv && (x - x == 0.0) && fabs(x) <= 0x1p1000;
      }
      ok = okv;
      if (INT_STATS) {
        const int64_t x = (int64_t)(((uint64_t)vhi << 32) | vlo);
        ok = ok && x > -(1ll << 50) && x < (1ll << 50);
      }
    }
    const uint64_t bal_v = __ballot(okv);
    if (bal_v && !found_any) {
      const int src = __builtin_ctzll(bal_v);
      any_lo = (uint32_t)__shfl((int)vlo, src, 64);
      any_hi = (uint32_t)__shfl((int)vhi, src, 64);
      found_any = true;
    }
    const uint64_t bal = __ballot(ok);
    if (bal) {
      const int src = __builtin_ctzll(bal);
      sh_lo = (uint32_t)__shfl((int)vlo, src, 64);
      sh_hi = (uint32_t)__shfl((int)vhi, src, 64);
      member = true;
      break;
    }
  }
  // (wave-uniform: kept in SGPRs, every VGPR counts toward the occupancy the VALU-bound loop needs)
  sh_lo = __builtin_amdgcn_readfirstlane(sh_lo);
  sh_hi = __builtin_amdgcn_readfirstlane(sh_hi);
  const double shift = uniform_f64(FP ? __builtin_bit_cast(double, ((uint64_t)sh_hi << 32) | sh_lo)
                                      : i64_to_f64(sh_lo, sh_hi));
  const double cshift = uniform_f64(0x1.8p52 + shift);  // exact: |c| < 2^50
  const double shift_any = FP ? shift : i64_to_f64(any_lo, any_hi);

  FastAcc a;
  fast_acc_init(a);
  constexpr uint32_t ROWS_PER_ITER = (uint32_t)kBlock * 2u * kFastUnroll;
  const uint32_t full_iters = span / ROWS_PER_ITER;
  if (member) {
    fast_main_loop<T, PK, STATS, HLL, true>(a, rv, rvalid, no_valid, full_iters, sh_lo, sh_hi, shift, cshift, lit_i,
                                            lit_f, lregs, &s_nan, nt);
    fast_tail<T, PK, STATS, HLL, true>(a, rv, rvalid, no_valid, full_iters * ROWS_PER_ITER, span, sh_lo, sh_hi,
                                       shift, cshift, lit_i, lit_f, lregs, &s_nan);
  } else {
    fast_main_loop<T, PK, STATS, HLL, false>(a, rv, rvalid, no_valid, full_iters, sh_lo, sh_hi, shift, cshift, lit_i,
                                             lit_f, lregs, &s_nan, nt);
    fast_tail<T, PK, STATS, HLL, false>(a, rv, rvalid, no_valid, full_iters * ROWS_PER_ITER, span, sh_lo, sh_hi,
                                        shift, cshift, lit_i, lit_f, lregs, &s_nan);
  }

  // int64 statistics: d = x - c was exact if every |x| < 2^51 (|d| < 2^50 here) and a lane's Σd cannot
  // leave int64 (it is rebuilt from the wrapping sum: Σd = Σxm - rows * c).  Otherwise the whole
  // workgroup recomputes Σd, Σd², min, max with the int64 -> double conversion (rare: only
  // columns holding values beyond +-2^51).
  bool exact_stats = false;
  uint32_t mom_sel = a.n_sel;  // the lane's selected rows behind Σd, Σd² (the re-run visits other rows)
  if constexpr (INT_STATS) {
    const double dmax = (a.fmin <= a.fmax) ? fmax(fabs(a.fmin), fabs(a.fmax)) : 0.0;
    const bool bad = a.n_rows > 0 && (dmax >= 0x1p50 || dmax * (double)a.n_rows >= 0x1p62 || a.s2 != a.s2);
    if (__syncthreads_or(bad)) {
      DQ_SCAN_COUNT(0);
      exact_stats = true;
      FastAcc e;
      fast_acc_init(e);
      // (about the wave's first valid value of any magnitude, which also stands in for NULLs)
      if (found_any)
        fast_tail<T, PK_NONE, true, false, true, true>(e, rv, rvalid, no_valid, 0u, span, any_lo, any_hi, shift_any,
                                                       cshift, lit_i, lit_f, lregs, &s_nan);
      else
        fast_tail<T, PK_NONE, true, false, false, true>(e, rv, rvalid, no_valid, 0u, span, 0u, 0u, 0.0, cshift,
                                                        lit_i, lit_f, lregs, &s_nan);
      a.s1 = e.s1;
      a.s2 = e.s2;
      mom_sel = e.n_sel;
      a.fmin = e.fmin;
      a.fmax = e.fmax;
    } else {
      // back to x: min / max of the selected values, Σd of the lane
      a.fmin = a.fmin + shift;
      a.fmax = a.fmax + shift;
      a.s1 = (double)(int64_t)(a.isum - (uint64_t)a.n_rows * (((uint64_t)sh_hi << 32) | sh_lo));
    }
  }

  // The moments' cancellation guard (moments_cancel, dq_scan_common.h): a wave whose shift was an
  // outlier makes the workgroup redo Σd, Σd² of its chunk about the chunk's mean.  The re-run's
  // stand-in for unselected rows is that mean itself (as int64 bits / fp64 bits), so their d is
  // exactly 0; its min / max are not used (they saw the stand-in).
  const bool lane0 = lane == 0;
  double mom_shift = (INT_STATS && exact_stats) ? (found_any ? shift_any : 0.0) : shift;
  uint64_t mom_w = 0u;  // lane 0: the wave's rows behind S1, S2
  double S1 = 0.0, S2 = 0.0;
  if constexpr (STATS) {
    mom_w = wave_sum_u64(mom_sel);
    S1 = wave_sum_f64(a.s1);
    S2 = wave_sum_f64(a.s2);
    double wn = 0.0, wmean = 0.0;
    bool cancel = false;
    if (lane0 && mom_w > 0) {
      wn = (double)mom_w;
      wmean = mom_shift + S1 / wn;
      cancel = moments_cancel(wn, S1, S2);
    }
    if (__syncthreads_or(cancel)) {
      const double m = block_mean_of_waves(wn, wmean);
      if (fabs(m) < (FP ? 0x1p1000 : 0x1p62)) {
        uint32_t m_lo, m_hi;
        double m_shift;
        if constexpr (FP) {
          m_shift = m;
          const uint64_t b = __builtin_bit_cast(uint64_t, m);
          m_lo = (uint32_t)b;
          m_hi = (uint32_t)(b >> 32);
        } else {
          const uint64_t b = (uint64_t)(int64_t)rint(m);
          m_lo = (uint32_t)b;
          m_hi = (uint32_t)(b >> 32);
          m_shift = i64_to_f64(m_lo, m_hi);  // what the re-run converts a stand-in row to
        }
        DQ_SCAN_COUNT(1);
        FastAcc e;
        fast_acc_init(e);
        fast_tail<T, PK_NONE, true, false, true, true>(e, rv, rvalid, no_valid, 0u, span, m_lo, m_hi, m_shift, cshift,
                                                       lit_i, lit_f, lregs, &s_nan);
        mom_shift = m_shift;
        mom_w = wave_sum_u64(e.n_sel);
        S1 = wave_sum_f64(e.s1);
        S2 = wave_sum_f64(e.s2);
      }
    }
  }

  if constexpr (HLL) {
    __syncthreads();
    for (int r = threadIdx.x; r < kHllM; r += kBlock) lregs[r] = hll_min_to_rank(lregs[r]);
    __syncthreads();
    // Registers holding the marker: re-rank them exactly over this workgroup's rows (rare).
    bool mine = false;
    if (threadIdx.x < kHllM / 32) lflag[threadIdx.x] = 0u;
    __syncthreads();
    for (int r = threadIdx.x; r < kHllM; r += kBlock) {
      if (lregs[r] == kRankMarker) {
        atomicOr(&lflag[r >> 5], 1u << (r & 31));
        lregs[r] = 0u;
        mine = true;
      }
    }
    if (__syncthreads_or(mine)) {
      DQ_SCAN_COUNT(2);
      for (uint32_t r = threadIdx.x; r < span; r += kBlock) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rv, (int)(r * 8u), 0, 0);
        const uint32_t bit = (((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rvalid, (int)(r >> 3), 0, 0) |
                               no_valid) >> (r & 7u)) & 1u;
        uint32_t lo = (uint32_t)v[0], hi = (uint32_t)v[1];
        if (FP) {
          const double x = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
          if (x != x) {
            lo = 0u;
            hi = 0x7ff80000u;
          }
        }
        const W64 h = hash_halves<T>(lo, hi);
        const uint32_t idx = h.hi >> 23;
        if (bit && ((lflag[idx >> 5] >> (idx & 31)) & 1u)) atomicMax(&lregs[idx], hll_rank_exact(h));
      }
      __syncthreads();
    }
    uint32_t* out = hll_regs + (int64_t)task.hll * kHllM;
    for (int r = threadIdx.x; r < kHllM; r += kBlock) {
      const uint32_t v = lregs[r];
      if (v) atomicMax(&out[r], v);
    }
  }
  __syncthreads();  // s_nan complete
  DQ_SCAN_COUNT(3);

  // ---- lane accumulators -> the block's ScanAcc partial (same layout as dq_scan_values_kernel;
  // block_reduce_store sums / merges the lanes, so lane 0 carries the wave-level terms)
  const uint64_t rows_w = wave_sum_u64(a.n_rows);  // lane 0
  const uint64_t sel_w = wave_sum_u64(a.n_sel);    // lane 0
  const uint64_t unsel_w = rows_w - sel_w;
  const uint64_t sh_bits = ((uint64_t)sh_hi << 32) | sh_lo;
  uint64_t isum = 0u;
  double mean = 0.0, m2 = 0.0, fs = 0.0, fc = 0.0;
  if constexpr (STATS) {
    isum = a.isum;
    fs = a.fs;
    fc = a.fc;
    if (lane0) {
      if constexpr (!FP) isum -= unsel_w * sh_bits;  // the stand-in copies of unselected rows (wrapping)
      if (mom_w > 0) {
        const double n = (double)mom_w;
        mean = mom_shift + S1 / n;
        m2 = S2 - S1 * S1 / n;
        m2 = (m2 < 0.0) ? 0.0 : m2;  // rounding; NaN/Inf propagate
      }
      if constexpr (FP) {  // the stand-in copies out of Σx: - n_unsel * c, its rounding kept by an fma
        if (unsel_w > 0) {
          const double u = (double)unsel_w;
          const double p = u * shift;
          const double pe = (p - p == 0.0) ? fma(u, shift, -p) : 0.0;
          two_sum_merge(fs, fc, -p, -pe);
        }
      }
    }
  }
  uint64_t pm[1] = {0u}, pn[1] = {0u};
  if constexpr (PK != PK_NONE) {
    if (lane0) {
      bool pc_shift;  // pred(c): what each unselected row's stand-in contributed to the count
      if constexpr (PK == PK_LT_I) pc_shift = (int64_t)sh_bits < lit_i;
      else if constexpr (PK == PK_EQ_I) pc_shift = (int64_t)sh_bits == lit_i;
      else if constexpr (PK == PK_LT_F) pc_shift = shift < lit_f;
      else pc_shift = shift == lit_f;
      uint64_t c_all = inv ? rows_w - a.pc : a.pc;
      if (pc_shift != inv) c_all -= unsel_w;
      pm[0] = c_all;
      pn[0] = sel_w;  // `column CMP literal` is NULL exactly when the column is
    }
  }
  const bool block_nan = FP && STATS && s_nan != 0u;
  // (n_sel is also the moments' n, so it is the wave's count of the rows behind them; the block
  // total is the same either way)
  block_reduce_store<1>(lane0 ? rows_w : 0u, lane0 ? rows_w : 0u, lane0 ? mom_w : 0u,
                        (threadIdx.x == 0 && block_nan) ? 1u : 0u, (int64_t)isum, INT64_MAX, INT64_MIN, fs, fc,
                        a.fmin, a.fmax, mean, m2, pm, pn, PK != PK_NONE ? 1 : 0,
                        &partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x]);
}

// ----------------------------------------------------------------------------- launchers
template <typename T, bool STATS, bool HLL>
static const void* fast_ptr(int pk) {
  switch (pk) {
    case PK_LT_I: return reinterpret_cast<const void*>(&dq_scan_fast_kernel<T, PK_LT_I, STATS, HLL>);
    case PK_EQ_I: return reinterpret_cast<const void*>(&dq_scan_fast_kernel<T, PK_EQ_I, STATS, HLL>);
    case PK_LT_F: return reinterpret_cast<const void*>(&dq_scan_fast_kernel<T, PK_LT_F, STATS, HLL>);
    case PK_EQ_F: return reinterpret_cast<const void*>(&dq_scan_fast_kernel<T, PK_EQ_F, STATS, HLL>);
    default: return reinterpret_cast<const void*>(&dq_scan_fast_kernel<T, PK_NONE, STATS, HLL>);
  }
}

template <typename T>
static const void* fast_kernel(int variant) {
  const int pk = variant & 7;
  const bool stats = (variant & FAST_STATS) != 0, hll = (variant & FAST_HLL) != 0;
  if (stats && hll) return fast_ptr<T, true, true>(pk);
  if (stats) return fast_ptr<T, true, false>(pk);
  if (hll) return fast_ptr<T, false, true>(pk);
  return fast_ptr<T, false, false>(pk);
}

static const void* fast_kernel_for(int ptype, int variant) {
  if (ptype == DQ_T_INT64) return fast_kernel<int64_t>(variant);
  if (ptype == DQ_T_FLOAT64) {
    const int pk = variant & 7;
    if (pk == PK_LT_I || pk == PK_EQ_I) return nullptr;  // fp columns compare as fp
    return fast_kernel<double>(variant);
  }
  return nullptr;
}

hipError_t launch_scan_fast(int ptype, int variant, const ScanTask* d_tasks, const int32_t* d_group, int n_group,
                            const DevColumn* d_cols, int64_t n_rows, int blocks_per_task, ScanAcc* d_partials,
                            uint32_t* d_hll_regs, hipStream_t stream) {
  if (n_group <= 0) return hipSuccess;
  const void* fn = fast_kernel_for(ptype, variant);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {&d_tasks, &d_group, &d_cols, &n_rows, &d_partials, &d_hll_regs};
#ifdef DQ_SCAN_DIAG
  {
    unsigned long long z[4] = {0, 0, 0, 0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_scan_diag), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
    const hipError_t e = hipLaunchKernel(fn, dim3(blocks_per_task, n_group), dim3(kBlock), args, 0, stream);
    (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_scan_diag), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    std::fprintf(stderr, "[scan_diag] rows %lld blocks %llu (x%d tasks): exact-int64 redo %llu, moment-guard redo %llu, "
                 "HLL marker re-rank %llu\n", (long long)n_rows, z[3], n_group, z[0], z[1], z[2]);
    return e;
  }
#endif
  return hipLaunchKernel(fn, dim3(blocks_per_task, n_group), dim3(kBlock), args, 0, stream);
}

int scan_fast_blocks_per_cu(int ptype, int variant) {
  const void* fn = fast_kernel_for(ptype, variant);
  if (!fn) return 0;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kBlock, 0) != hipSuccess || nb < 1) return 0;
  return nb;
}

}  // namespace dq
