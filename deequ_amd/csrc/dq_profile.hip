// dq_profile.hip -- kernels for the ColumnProfiler path (ColumnProfiler.scala:220-251, 427-445).
//
// 1. DataType (DataType.scala:152-183, catalyst/StatefulDataType.scala:26-83): per row of the
//    column cast to string, classify it as NULL / Fractional / Integral / Boolean / String with
//    the reference's anchored regexes, tested in this order:
//        FRACTIONAL  ^(-|\+)? ?\d*\.\d*$        INTEGRAL  ^(-|\+)? ?\d*$        BOOLEAN  ^(true|false)$
//    (Java `\d` = [0-9]; Scala's `case R(_)` is a whole-string match.)  On utf8 bytes this is a
//    five-state DFA; numeric columns are classified from their value, as the string Spark's
//    Cast would produce (integers -> Integral; a float/double prints plain -- Fractional --
//    only for 0 and 1e-3 <= |x| < 1e7 and is "NaN"/"Infinity"/scientific -- String --
//    otherwise; booleans -> Boolean).  The five counts are integers: order independent.
// 2. Cast(StringType -> LongType / DoubleType) of the columns pass 1 typed as Integral /
//    Fractional (ColumnProfiler.castNumericStringColumns, :427-445), Spark 2.2.2 semantics:
//    long = UTF8String.toLong (optional sign, digits, optional '.' + digits truncated, no
//    whitespace, overflow -> NULL); double = java.lang.Double.parseDouble (whitespace trimmed,
//    sign, digits, '.', exponent, f/d suffix, NaN/Infinity, hexadecimal), correctly rounded for
//    every input (dq_numparse.h: Clinger's fast path, Eisel-Lemire, an exact big-integer
//    comparison near rounding boundaries).
#include "dq_parse.h"
#include "dq_strhash.h"

namespace dq {

namespace {

enum DtPos { DT_NULL = 0, DT_FRACTIONAL = 1, DT_INTEGRAL = 2, DT_BOOLEAN = 3, DT_STRING = 4 };

__device__ inline bool bit_at(const uint8_t* bm, int64_t row) { return (bm[row >> 3] >> (row & 7)) & 1u; }

template <typename Src>
__device__ int classify_utf8(const Src& p, int32_t n) {
  // DFA: 0 start, 1 after sign, 2 after the optional space, 3 integer digits, 4 after '.', 5 fail
  int st = 0;
  for (int32_t i = 0; i < n && st != 5; ++i) {
    const uint32_t c = p[i];
    const bool digit = c - '0' < 10u;
    switch (st) {
      case 0: st = (c == '-' || c == '+') ? 1 : c == ' ' ? 2 : digit ? 3 : c == '.' ? 4 : 5; break;
      case 1: st = c == ' ' ? 2 : digit ? 3 : c == '.' ? 4 : 5; break;
      case 2: case 3: st = digit ? 3 : c == '.' ? 4 : 5; break;
      default: st = digit ? 4 : 5; break;
    }
  }
  if (st == 4) return DT_FRACTIONAL;
  if (st != 5) return DT_INTEGRAL;
  if (n == 4 && p[0] == 't' && p[1] == 'r' && p[2] == 'u' && p[3] == 'e') return DT_BOOLEAN;
  if (n == 5 && p[0] == 'f' && p[1] == 'a' && p[2] == 'l' && p[3] == 's' && p[4] == 'e') return DT_BOOLEAN;
  return DT_STRING;
}

// The same classification, 8 bytes at a time, for strings of <= 24 bytes (the word-loaded
// form).  The DFA above accepts: an optional sign, then an optional single space, then a body of
// digits and '.' -- no '.' is Integral, exactly one is Fractional, anything else fails.  So the
// prefix is located from the first two bytes, and the body is tested with per-byte SWAR flags
// (bit 7 of each byte): non-digit, '.', and "inside [pos, n)".  No per-byte loop, no branches
// per byte.
__device__ inline uint64_t swar_nondigit(uint64_t x) {  // bit 7 set iff the byte is not '0'..'9'
  const uint64_t t = x ^ 0x3030303030303030ull;
  return (((t & 0x7f7f7f7f7f7f7f7full) + 0x7676767676767676ull) | t) & 0x8080808080808080ull;
}
__device__ inline uint64_t swar_is(uint64_t x, uint64_t rep) {  // bit 7 set iff the byte == rep's
  const uint64_t t = x ^ rep;
  return ~((((t & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | t)) & 0x8080808080808080ull;
}
__device__ inline uint64_t swar_bytes_below(int32_t m) {  // bytes [0, m) of a word (bit 7 flags)
  const uint64_t all = 0x8080808080808080ull;
  return m <= 0 ? 0ull : m >= 8 ? all : (all & ((1ull << (8 * m)) - 1ull));
}

// s0, s1, s2: the string's bytes 0..7, 8..15, 16..23 (s1 / s2 read only when n > 8 / 16).
__device__ int classify_shifted(uint64_t s0, uint64_t s1, uint64_t s2, int32_t n) {
  const uint32_t b0 = (uint32_t)s0 & 0xffu;
  int32_t pos = (n > 0 && (b0 == '+' || b0 == '-')) ? 1 : 0;
  if (pos < n && (((uint32_t)(s0 >> (8 * pos))) & 0xffu) == ' ') ++pos;
  // word 0: bytes [pos, n); later words: bytes below n only (pos <= 2)
  uint64_t in = swar_bytes_below(n) & ~swar_bytes_below(pos);
  uint64_t dot = swar_is(s0, 0x2e2e2e2e2e2e2e2eull) & in;
  uint64_t bad = swar_nondigit(s0) & in & ~dot;
  int dots = __builtin_popcountll(dot);
  if (n > 8 && bad == 0) {  // (a failed first word decides: String or Boolean from word 0)
    in = swar_bytes_below(n - 8);
    dot = swar_is(s1, 0x2e2e2e2e2e2e2e2eull) & in;
    bad |= swar_nondigit(s1) & in & ~dot;
    dots += __builtin_popcountll(dot);
    if (n > 16) {
      in = swar_bytes_below(n - 16);
      dot = swar_is(s2, 0x2e2e2e2e2e2e2e2eull) & in;
      bad |= swar_nondigit(s2) & in & ~dot;
      dots += __builtin_popcountll(dot);
    }
  }
  if (bad == 0 && dots <= 1) return dots ? DT_FRACTIONAL : DT_INTEGRAL;
  if (n == 4 && (uint32_t)s0 == 0x65757274u) return DT_BOOLEAN;                       // "true"
  if (n == 5 && (s0 & 0xffffffffffull) == 0x65736c6166ull) return DT_BOOLEAN;          // "false"
  return DT_STRING;
}

// The string's bytes 8k..8k+7 as one word (funnel shift of the aligned words).
__device__ inline uint64_t funnel(uint64_t lo, uint64_t hi, uint32_t sh_bits) {
  return sh_bits ? (lo >> sh_bits) | (hi << (64u - sh_bits)) : lo;
}

__device__ int classify_utf8_words(const WordSrc& ws, int32_t n) {
  const uint32_t sh = ws.sh * 8u;
  return classify_shifted(funnel(ws.w0, ws.w1, sh), funnel(ws.w1, ws.w2, sh), funnel(ws.w2, ws.w3, sh), n);
}

template <typename F>
__device__ inline int classify_float(F x) {
  // Double.toString / Float.toString: plain notation for 1e-3 <= |x| < 1e7 (and 0)
  if (!(x - x == x - x)) return DT_STRING;  // NaN, +-Infinity
  const F a = x < 0 ? -x : x;
  if (a == (F)0 || (a >= (F)1e-3 && a < (F)1e7)) return DT_FRACTIONAL;
  return DT_STRING;
}

__device__ int classify_row(const DevColumn& c, int64_t row) {
  switch (c.type) {
    case DQ_T_UTF8: {
      const int32_t b = c.offsets[row], e = c.offsets[row + 1];
      const uint8_t* p = static_cast<const uint8_t*>(c.values) + b;
      return e - b <= 24 ? classify_utf8_words(WordSrc(p, e - b), e - b) : classify_utf8(PtrSrc{p}, e - b);
    }
    case DQ_T_BOOL: return DT_BOOLEAN;
    case DQ_T_FLOAT32: return classify_float(static_cast<const float*>(c.values)[row]);
    case DQ_T_FLOAT64: return classify_float(static_cast<const double*>(c.values)[row]);
    default: return DT_INTEGRAL;  // int8..int64 print as [-]digits
  }
}

__device__ inline uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_down((unsigned long long)v, d, 64);
  return v;
}

}  // namespace

// blockIdx.y = task (column, where), blockIdx.x = row chunk; 5 counts per task, atomically
// added (integers: the result does not depend on the schedule).
__global__ __launch_bounds__(kBlock) void dq_datatype_kernel(const HllTask* __restrict__ tasks,
                                                             const DevColumn* __restrict__ cols,
                                                             const DevMask* __restrict__ masks,
                                                             int64_t n_rows, unsigned long long* counts) {
  const HllTask task = tasks[blockIdx.y];
  const DevColumn& col = cols[task.column];
  const uint8_t* wt = task.where_mask >= 0 ? reinterpret_cast<const uint8_t*>(masks[task.where_mask].t) : nullptr;
  const int64_t per_block = (n_rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(r0 + per_block, n_rows);
  uint64_t c[5] = {0, 0, 0, 0, 0};
  if (col.type == DQ_T_UTF8) {  // uniform
    // U rows per lane per step, every load of the step issued before any classification: the
    // string words come through a buffer descriptor over the (8-byte aligned) value bytes, so the
    // four word loads per row are unconditional (out of range reads 0) and overlap across rows.
    constexpr int U = 4;
    const uint8_t* vals = static_cast<const uint8_t*>(col.values);
    const uintptr_t al = (uintptr_t)vals & ~(uintptr_t)7;
    const uint32_t delta = (uint32_t)((uintptr_t)vals - al);
    const uint32_t span = (delta + (uint32_t)col.offsets[n_rows] + 7u) & ~7u;  // the last valid byte's word
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(al), 0, (int)span, 0x00020000);
    for (int64_t base = r0 + threadIdx.x; base < r1; base += U * kBlock) {
      int32_t ob[U], oe[U];
      bool sel[U];
      uint64_t w[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = base + (int64_t)u * kBlock;
        const bool in = row < r1;
        const int64_t rr = in ? row : r0;
        ob[u] = col.offsets[rr];
        oe[u] = col.offsets[rr + 1];
        sel[u] = in && (col.validity == nullptr || bit_at(col.validity, rr)) && (wt == nullptr || bit_at(wt, rr));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t a = (delta + (uint32_t)ob[u]) & ~7u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(a + 8u * k), 0, 0);
          w[u][k] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = base + (int64_t)u * kBlock;
        if (row >= r1) break;
        const int32_t n = oe[u] - ob[u];
        int k = DT_NULL;
        if (sel[u]) {
          k = n <= 24 ? classify_utf8_words(WordSrc(w[u][0], w[u][1], w[u][2], w[u][3], (delta + (uint32_t)ob[u]) & 7u), n)
                      : classify_utf8(PtrSrc{vals + ob[u]}, n);
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) c[i] += (k == i) ? 1u : 0u;
      }
    }
  } else
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
    // conditionalSelection: a row whose filter is not TRUE is a NULL input (Analyzer.scala:409-420)
    const bool valid = (col.validity == nullptr || bit_at(col.validity, row)) && (wt == nullptr || bit_at(wt, row));
    const int k = valid ? classify_row(col, row) : DT_NULL;
#pragma unroll
    for (int i = 0; i < 5; ++i) c[i] += (k == i) ? 1u : 0u;
  }
  __shared__ uint64_t part[kBlock / 64][5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint64_t s = wave_sum(c[i]);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    uint64_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += part[w][threadIdx.x];
    if (s) atomicAdd(&counts[(int64_t)task.reg_set * 5 + threadIdx.x], (unsigned long long)s);  // (reg_set = the task's count index)
  }
}

// Profiler pass 1 on utf8 columns: DataType (DataType.scala:152-183) and ApproxCountDistinct
// (StatefulHyperloglogPlus.scala:89-115) of the same (column, where) from ONE read of the
// strings -- the offsets, then four aligned 8-byte words per row through a buffer descriptor
// (unconditional: out of range reads 0), U rows per lane in flight; the words feed both the
// SWAR classifier and the word-form XXH64 (strings of <= 24 bytes; longer ones take the
// byte-pointer paths).  Every row is hashed and counted (rank 0 / DT_NULL when not selected),
// so lanes diverge only on the length.  Counts are integers and registers maxima: the result
// does not depend on the schedule.
#ifndef DQ_STR_U
#define DQ_STR_U 4
#endif
// Little-endian p[0..n) (n <= 8), zero padded, from the aligned words that hold those bytes only.
__device__ inline uint64_t ld_bytes(const uint8_t* p, uint32_t n) {
  if (n == 0) return 0;
  const uintptr_t a = (uintptr_t)p;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(a & 7) * 8u;
  uint64_t v = w[0] >> sh;
  if (sh && (a & 7) + n > 8) v |= w[1] << (64u - sh);
  return n >= 8 ? v : (v & ((1ull << (8u * n)) - 1ull));
}

// 24 bytes of a string heap (a descriptor over [0, heap_end)) from byte a: one unaligned 16-byte
// and one 8-byte buffer load at lo = min(a, heap_end - 24), always wholly in range -- a buffer
// load's range check is per dword counted from the load's own offset, so a load reaching past
// heap_end would zero whole dwords, string bytes included.  A string starting in the heap's last
// 24 bytes lands s = a - lo bytes into the words (s + n <= 24; returned): load24_fix shifts it
// down once the words have arrived (no memory access in that rare branch).  A heap of fewer than
// 24 bytes (uniform) is read byte-exactly.  The bytes past a string's end are not used.
// n = the string's length: a string of at most 16 bytes takes ONE 16-byte load at
// min(a, heap_end - 16) (w[2] = 0), so the common short string costs one memory instruction.
__device__ __forceinline__ uint32_t load24(__amdgpu_buffer_rsrc_t rs, const uint8_t* vals, uint32_t heap_end, uint32_t a,
                                           uint32_t n, uint64_t (&w)[3]) {
  if (heap_end >= 24u) {
    if (n <= 16u) {
      const uint32_t lo = min(a, heap_end - 16u);
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)lo, 0, 0);
      w[0] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
      w[1] = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
      w[2] = 0ull;
      return a - lo;
    }
    const uint32_t lo = min(a, heap_end - 24u);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)lo, 0, 0);
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(lo + 16u), 0, 0);
    w[0] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
    w[1] = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
    w[2] = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
    return a - lo;
  }
  const uint32_t m = a < heap_end ? heap_end - a : 0u;  // bytes of the heap from a (< 24)
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = m > 8u * k ? ld_bytes(vals + a + 8u * k, min(8u, m - 8u * k)) : 0ull;
  return 0u;
}
// w >>= 8 s bits (192-bit; s = load24's result, 1..24).
__device__ __forceinline__ void load24_fix(uint64_t (&w)[3], uint32_t s) {
  const uint32_t q = s >> 3, r = 8u * (s & 7u);
  const uint64_t d0 = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : 0ull;
  const uint64_t d1 = q == 0 ? w[1] : q == 1 ? w[2] : 0ull;
  const uint64_t d2 = q == 0 ? w[2] : 0ull;
  w[0] = r ? (d0 >> r) | (d1 << (64u - r)) : d0;
  w[1] = r ? (d1 >> r) | (d2 << (64u - r)) : d1;
  w[2] = r ? (d2 >> r) : d2;
}

// DT = false: the HLL alone (an ApproxCountDistinct without a DataType on the column), through
// the same batched word loads.
template <bool DT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void dq_string_pass_kernel(const StrTask* __restrict__ tasks,
                                                                const DevColumn* __restrict__ cols,
                                                                const DevMask* __restrict__ masks, int64_t n_rows,
                                                                uint32_t* registers, unsigned long long* counts) {
  __shared__ uint32_t regs[kHllM];
  __shared__ uint64_t part[kBlock / 64][5];
  const StrTask task = tasks[blockIdx.y];
  for (int r = threadIdx.x; r < kHllM; r += kBlock) regs[r] = 0u;
  __syncthreads();
  const int64_t n_chunks = (n_rows + kScanRowAlign - 1) / kScanRowAlign;
  const int64_t per_block = (n_chunks + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = min((int64_t)blockIdx.x * per_block * kScanRowAlign, n_rows);
  const int64_t r1 = min(r0 + per_block * kScanRowAlign, n_rows);
  const DevColumn& col = cols[task.column];
  const uint8_t* wt = task.where_mask >= 0 ? reinterpret_cast<const uint8_t*>(masks[task.where_mask].t) : nullptr;
  const uint8_t* vals = static_cast<const uint8_t*>(col.values);
  // each row's offset pair as one 8-byte buffer load, relative to the block's first row
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t*>(col.offsets + r0), 0, (int)(4u * (uint32_t)(r1 - r0 + 1)), 0x00020000);
  // the first 24 bytes of each string as three words (load24: unaligned, from its first byte)
  const uint32_t heap_end = (uint32_t)col.offsets[n_rows];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vals), 0, (int)heap_end, 0x00020000);
  uint64_t c[5] = {0, 0, 0, 0, 0};
  // the five type counts of this lane as 12-bit fields of one word (count k at bit 12 k: one
  // shift and one 64-bit add per row), folded into c[] before a field can reach 4096
  uint64_t packed = 0ull;
  uint32_t since_fold = 0u;
  constexpr int U = DQ_STR_U;
  // the offset pairs of a step's U rows (rows past the block read row r0's); the next step's are
  // loaded while this step's strings load and are hashed (round 5, as the cast kernel does), so
  // the offsets -> string bytes round trip is paid once per step, not twice
  int32_t ob[U], oe[U];
  auto load_offs = [&](int64_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + (int64_t)u * kBlock;
      const int64_t rr = row < r1 ? row : r0;
      const auto o = __builtin_amdgcn_raw_buffer_load_b64(ro, (int)(4u * (uint32_t)(rr - r0)), 0, 0);
      ob[u] = (int32_t)o[0];
      oe[u] = (int32_t)o[1];
    }
  };
  if (r0 + (int64_t)threadIdx.x < r1) load_offs(r0 + threadIdx.x);
  for (int64_t base = r0 + threadIdx.x; base < r1; base += U * kBlock) {
    if constexpr (DT) {
      if (since_fold >= 4096u - U) {
#pragma unroll
        for (int i = 0; i < 5; ++i) c[i] += (packed >> (12 * i)) & 0xFFFull;
        packed = 0ull;
        since_fold = 0u;
      }
      since_fold += U;
    }
    uint32_t sel[U], sh[U];
    uint64_t w[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + (int64_t)u * kBlock;
      const bool in = row < r1;
      const int64_t rr = in ? row : r0;
      sel[u] = (in && (col.validity == nullptr || bit_at(col.validity, rr)) && (wt == nullptr || bit_at(wt, rr))) ? 1u : 0u;
    }
    int32_t cb[U], ce[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cb[u] = ob[u];
      ce[u] = oe[u];
      sh[u] = load24(rs, vals, heap_end, (uint32_t)cb[u], (uint32_t)(ce[u] - cb[u]), w[u]);
    }
    if (base + U * kBlock < r1) load_offs(base + U * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + (int64_t)u * kBlock;
      if (row >= r1) break;
      const int32_t n = ce[u] - cb[u];
      int k;
      W64 h;
      if (n <= 24) {
        if (sh[u]) load24_fix(w[u], sh[u]);  // (a string in the heap's last 24 bytes)
        const uint64_t s[3] = {w[u][0], w[u][1], w[u][2]};
        k = (DT && sel[u]) ? classify_shifted(s[0], s[1], s[2], n) : DT_NULL;
        h = xxh64_words_dev(s, (uint32_t)n);
      } else {
        k = (DT && sel[u]) ? classify_utf8(PtrSrc{vals + cb[u]}, n) : DT_NULL;
        h = xxh64_utf8_dev(vals + cb[u], (uint32_t)n);
      }
      if constexpr (DT) packed += 1ull << (12u * (uint32_t)k);
      uint32_t idx, nlz, r;
      hll_slot(h, idx, nlz);
      asm("v_mad_u32_u24 %0, %1, %2, %2" : "=v"(r) : "v"(nlz), "v"(sel[u]));  // rank * sel
      __hip_atomic_fetch_max(&regs[idx], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  if constexpr (DT) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint64_t s = wave_sum(c[i] + ((packed >> (12 * i)) & 0xFFFull));
      if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6][i] = s;
    }
  }
  __syncthreads();
  if (DT && threadIdx.x < 5) {
    uint64_t s = 0;
    for (int wv = 0; wv < kBlock / 64; ++wv) s += part[wv][threadIdx.x];
    if (s) atomicAdd(&counts[(int64_t)task.dt_index * 5 + threadIdx.x], (unsigned long long)s);
  }
  uint32_t* out = registers + (int64_t)task.reg_set * kHllM;
  for (int r = threadIdx.x; r < kHllM; r += kBlock) {
    const uint32_t v = regs[r];
    if (v) atomicMax(&out[r], v);
  }
}

namespace {

// 8 ASCII digits (first digit in the low byte) -> their value: pairs, quads, then the 8-digit
// number, three multiply-adds on the whole word.
__device__ inline uint64_t swar_digits8(uint64_t x) {
  x -= 0x3030303030303030ull;
  x = (x * 10u + (x >> 8)) & 0x00ff00ff00ff00ffull;
  x = (x * 100u + (x >> 16)) & 0x0000ffff0000ffffull;
  return (x * 10000u + (x >> 32)) & 0xffffffffull;
}

// parse_long on the word-loaded form, with a fast path for the common shape: an optional sign
// and 1..16 digits (no '.', so no overflow is possible).  The digits are right-aligned in a
// 16-byte window padded with '0' and converted 8 at a time; anything else takes parse_long.
__device__ bool parse_long_words(const WordSrc& ws, int32_t n, int64_t* out) {
  if (n >= 1 && n <= 17) {
    const uint32_t sh = ws.sh * 8u;
    const uint64_t s0 = sh ? (ws.w0 >> sh) | (ws.w1 << (64u - sh)) : ws.w0;
    const uint64_t s1 = sh ? (ws.w1 >> sh) | (ws.w2 << (64u - sh)) : ws.w1;
    const uint64_t s2 = sh ? (ws.w2 >> sh) | (ws.w3 << (64u - sh)) : ws.w2;
    const uint32_t b0 = (uint32_t)s0 & 0xffu;
    const bool neg = b0 == '-';
    const int32_t start = (neg || b0 == '+') ? 1 : 0;
    const int32_t nd = n - start;
    if (nd >= 1 && nd <= 16) {
      const unsigned __int128 raw =
          start ? (((unsigned __int128)s2 << 120) | ((unsigned __int128)s1 << 56) | (unsigned __int128)(s0 >> 8))
                : (((unsigned __int128)s1 << 64) | (unsigned __int128)s0);
      const uint32_t pad = 8u * (uint32_t)(16 - nd);  // bits of '0' fill below the digits
      const unsigned __int128 zeros = ((unsigned __int128)0x3030303030303030ull << 64) | 0x3030303030303030ull;
      const unsigned __int128 fill = pad ? (zeros & ((((unsigned __int128)1) << pad) - 1)) : 0;
      const unsigned __int128 v = (raw << pad) | fill;
      const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
      if ((swar_nondigit(lo) | swar_nondigit(hi)) == 0) {
        const int64_t r = (int64_t)(swar_digits8(lo) * 100000000ull + swar_digits8(hi));
        *out = neg ? -r : r;
        return true;
      }
    }
  }
  return parse_long(ws, n, out);
}

template <int TO>
__device__ inline bool cast_one(const WordSrc& p, int32_t n, int64_t* lv, double* dv) {
  if constexpr (TO == DQ_T_INT64) return parse_long_words(p, n, lv);
  else return parse_double(p, n, dv) == 1;
}

template <int TO, typename Src>
__device__ inline bool cast_one(const Src& p, int32_t n, int64_t* lv, double* dv) {
  if constexpr (TO == DQ_T_INT64) return parse_long(p, n, lv);
  else return parse_double(p, n, dv) == 1;
}

}  // namespace

// One row per lane: values are written coalesced, and each wave's 64 validity bits (a ballot)
// are stored by its first lane -- one 8-byte word when the wave's rows are all in range.  One
// instantiation per target type: the string -> long cast does not carry the double parser's
// registers (its exact big-number path) into its occupancy.
#ifndef DQ_CAST_PIPE
#define DQ_CAST_PIPE 1
#endif
// Rows per lane per step of the cast: 2 (62 VGPRs, 8 waves per SIMD) measured 0.55 ms per
// 1e8-row column alone against 0.71 with 4 (114 VGPRs, 4 waves); 3 0.62, 6 0.85
// (profiles/r05_c5_cast_rows_ab.txt)
#ifndef DQ_CAST_U
#define DQ_CAST_U 2
#endif
template <int TO>
__global__ __launch_bounds__(kBlock) void dq_cast_utf8_kernel(DevColumn src, int64_t n_rows, void* values,
                                                              uint8_t* validity) {
  // U rows per lane per step, every load of the step issued before any parse: each row's offset
  // pair (one 8-byte load), its validity byte, and the first 24 bytes of the string (load24: a 16-
  // and an 8-byte unaligned buffer load).  Longer strings take the byte-pointer parser.
  constexpr int to_type = TO;
  constexpr int U = DQ_CAST_U;
  const uint32_t lane = threadIdx.x & 63u;
  const uint8_t* vals = static_cast<const uint8_t*>(src.values);
  const uint32_t heap_end = (uint32_t)src.offsets[n_rows];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vals), 0, (int)heap_end, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(src.offsets), 0, (int)(4u * (uint32_t)(n_rows + 1)), 0x00020000);
  // the offsets and validity bits of the NEXT step are loaded while this step's strings load and
  // parse (DQ_CAST_PIPE): the offsets -> string bytes round trip is paid once per step, not twice
  const int64_t stride = (int64_t)gridDim.x * kBlock * U;
  uint32_t ob[U], oe[U], sel = 0u;
  auto load_offs = [&](int64_t base, uint32_t (&b)[U], uint32_t (&e)[U], uint32_t& sl) {
    sl = 0u;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + (int64_t)u * kBlock + threadIdx.x;
      const auto o = __builtin_amdgcn_raw_buffer_load_b64(ro, (int)(4u * (uint32_t)row), 0, 0);
      b[u] = o[0];
      e[u] = o[1];
      if (row < n_rows && (src.validity == nullptr || bit_at(src.validity, row))) sl |= 1u << u;
    }
  };
  if ((int64_t)blockIdx.x * kBlock * U < n_rows) load_offs((int64_t)blockIdx.x * kBlock * U, ob, oe, sel);
  for (int64_t base = (int64_t)blockIdx.x * kBlock * U; base < n_rows; base += stride) {
    uint32_t sh[U];
    uint64_t w[U][3];
#if DQ_CAST_PIPE
#pragma unroll
    for (int u = 0; u < U; ++u) sh[u] = load24(rs, vals, heap_end, ob[u], oe[u] - ob[u], w[u]);
    uint32_t nob[U], noe[U], nsel = 0u;
    if (base + stride < n_rows) load_offs(base + stride, nob, noe, nsel);
#else
    if (base != (int64_t)blockIdx.x * kBlock * U) load_offs(base, ob, oe, sel);
#pragma unroll
    for (int u = 0; u < U; ++u) sh[u] = load24(rs, vals, heap_end, ob[u], oe[u] - ob[u], w[u]);
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + (int64_t)u * kBlock + threadIdx.x;
      int64_t lv = 0;
      double dv = 0.0;
      bool ok = false;
      if ((sel >> u) & 1u) {
        const int32_t n = (int32_t)(oe[u] - ob[u]);
        if (n <= 24) {
          if (sh[u]) load24_fix(w[u], sh[u]);  // (a string in the heap's last 24 bytes)
          ok = cast_one<TO>(WordSrc(w[u][0], w[u][1], w[u][2], 0ull, 0u), n, &lv, &dv);
        }
        else ok = cast_one<TO>(PtrSrc{vals + ob[u]}, n, &lv, &dv);
      }
      if (row < n_rows) {
        if (to_type == DQ_T_INT64) static_cast<int64_t*>(values)[row] = ok ? lv : 0;
        else static_cast<double*>(values)[row] = ok ? dv : 0.0;
      }
      const uint64_t mk = __ballot(ok);
      const int64_t row0 = row - (int64_t)lane;  // first row of the wave: a multiple of 64
      if (lane == 0 && row0 < n_rows) {
        if (row0 + 64 <= n_rows) {
          *reinterpret_cast<uint64_t*>(validity + (row0 >> 3)) = mk;
        } else {
          const int64_t nb = ((n_rows - row0) + 7) >> 3;
          for (int64_t k = 0; k < nb; ++k) validity[(row0 >> 3) + k] = (uint8_t)(mk >> (8 * k));
        }
      }
    }
#if DQ_CAST_PIPE
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ob[u] = nob[u];
      oe[u] = noe[u];
    }
    sel = nsel;
#endif
  }
}

hipError_t launch_string_pass(const StrTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                              int64_t n_rows, int blocks_per_task, uint32_t* d_registers, unsigned long long* d_counts,
                              hipStream_t stream) {
  if (n_tasks <= 0 || n_rows <= 0) return hipSuccess;
  if (d_counts)
    hipLaunchKernelGGL(dq_string_pass_kernel<true>, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream, d_tasks,
                       d_cols, d_masks, n_rows, d_registers, d_counts);
  else
    hipLaunchKernelGGL(dq_string_pass_kernel<false>, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream, d_tasks,
                       d_cols, d_masks, n_rows, d_registers, d_counts);
  return hipGetLastError();
}

// ApproxCountDistinct + DataType of a utf8 column from its distinct strings (dq_profile_string_groups):
// one thread per group hashes and classifies the key once; the DataType count is weighted by the
// group's count, the register update is the same maximum the per-row pass takes.
__global__ __launch_bounds__(kBlock) void dq_string_groups_kernel(const int64_t* __restrict__ counts,
                                                                  const int64_t* __restrict__ offs,
                                                                  const uint8_t* __restrict__ bytes, int64_t n,
                                                                  uint32_t* __restrict__ regs,
                                                                  unsigned long long* __restrict__ dtc) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = bytes + offs[i];
  const int64_t len = offs[i + 1] - offs[i];
  const int cls = classify_utf8(p, (int32_t)len);
  atomicAdd(&dtc[cls], (unsigned long long)counts[i]);
  uint32_t idx, pw;
  hll_idx_rank(xxh64_bytes(p, len, 42), &idx, &pw);
  atomicMax(&regs[idx], pw);
}

hipError_t launch_string_groups(const int64_t* d_counts, const int64_t* d_offs, const uint8_t* d_bytes, int64_t n,
                                uint32_t* d_regs, unsigned long long* d_dtc, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_string_groups_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                     d_counts, d_offs, d_bytes, n, d_regs, d_dtc);
  return hipGetLastError();
}

// The same from the few-groups kernel's compact list (dq_freq_small_merge_flat_kernel: key bytes
// 0..7 in k0, 8..14 and the length << 56 in k1, *n groups).
__global__ __launch_bounds__(kBlock) void dq_string_groups_words_kernel(const unsigned long long* __restrict__ k0,
                                                                        const unsigned long long* __restrict__ k1,
                                                                        const unsigned long long* __restrict__ counts,
                                                                        const uint32_t* __restrict__ n,
                                                                        uint32_t* __restrict__ regs,
                                                                        unsigned long long* __restrict__ dtc,
                                                                        uint32_t max_n) {
  const uint64_t y = blockIdx.y;  // the column
  k0 += y * max_n;
  k1 += y * max_n;
  counts += y * max_n;
  regs += y * kHllM;
  dtc += y * 8;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n[y]) return;
  const uint64_t w0 = k0[i], w1 = k1[i];
  const uint32_t len = (uint32_t)(w1 >> 56);
  uint8_t b[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    b[j] = (uint8_t)(w0 >> (8 * j));
    b[8 + j] = j < 7 ? (uint8_t)(w1 >> (8 * j)) : 0u;
  }
  const uint8_t* p = b;
  const int cls = classify_utf8(p, (int32_t)len);
  atomicAdd(&dtc[cls], counts[i]);
  uint32_t idx, pw;
  hll_idx_rank(xxh64_bytes(p, (int64_t)len, 42), &idx, &pw);
  atomicMax(&regs[idx], pw);
}

hipError_t launch_string_groups_words(const unsigned long long* d_k0, const unsigned long long* d_k1,
                                      const unsigned long long* d_counts, const uint32_t* d_n, uint32_t max_n, int n_cols,
                                      uint32_t* d_regs, unsigned long long* d_dtc, hipStream_t stream) {
  if (n_cols <= 0 || n_cols > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dq_string_groups_words_kernel, dim3((max_n + kBlock - 1) / kBlock, (unsigned)n_cols), dim3(kBlock), 0,
                     stream, d_k0, d_k1, d_counts, d_n, d_regs, d_dtc, max_n);
  return hipGetLastError();
}

hipError_t launch_datatype(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                           int64_t n_rows, int blocks_per_task, unsigned long long* d_counts, hipStream_t stream) {
  if (n_tasks <= 0 || n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_datatype_kernel, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream, d_tasks, d_cols,
                     d_masks, n_rows, d_counts);
  return hipGetLastError();
}

hipError_t launch_cast_utf8(const DevColumn& src, int64_t n_rows, int to_type, void* d_values, uint8_t* d_validity,
                            hipStream_t stream) {
  // chunks of at most 2^28 rows: the kernel's offsets descriptor spans 4 (rows + 1) bytes
  constexpr int64_t kChunk = (int64_t)1 << 28;
  for (int64_t start = 0; start < n_rows; start += kChunk) {
    const int64_t m = n_rows - start < kChunk ? n_rows - start : kChunk;
    DevColumn c = src;
    c.offsets = src.offsets + start;  // (offsets stay absolute into the bytes)
    if (c.validity) c.validity = src.validity + (start >> 3);
    uint8_t* vout = d_validity + (start >> 3);
    int64_t blocks = (m + DQ_CAST_U * kBlock - 1) / (DQ_CAST_U * kBlock);  // (DQ_CAST_U rows per lane per step)
    if (blocks > 8192) blocks = 8192;
    if (to_type == DQ_T_INT64)
      hipLaunchKernelGGL(dq_cast_utf8_kernel<DQ_T_INT64>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, c, m,
                         static_cast<void*>(static_cast<int64_t*>(d_values) + start), vout);
    else
      hipLaunchKernelGGL(dq_cast_utf8_kernel<DQ_T_FLOAT64>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, c, m,
                         static_cast<void*>(static_cast<double*>(d_values) + start), vout);
  }
  return hipGetLastError();
}

}  // namespace dq
