// dq_numparse.h -- java.lang.Double.parseDouble, correctly rounded for every input, as a host +
// device header (the cast kernel and the predicate interpreter run it on the GPU; a host build
// of the same code is checked against Python's correctly rounded float() on CPU, tests/).
//
// Spark 2.2.2's Cast(StringType -> DoubleType) is `s.toString.toDouble` = Double.parseDouble of
// the string (ColumnProfiler.scala:427-445 casts every Integral / Fractional-typed column this way;
// `item > 3` on a string column casts the same way, PromoteStrings).  Three tiers, each exact:
//   1. Clinger's fast path: <= 2^53 significand, |exponent| <= 22 -> one IEEE multiply / divide;
//   2. Eisel-Lemire: the first 19 significant digits w and exponent q, w * 5^q through a 128-bit
//      table (dq_pow5_table.h); with 128 bits the result is always correct for an exact w
//      (Mushtak & Lemire 2023).  When digits beyond 19 were dropped, w and w + 1 bracket the value:
//      equal results are the answer;
//   3. otherwise (a value within half an ulp of a rounding boundary) the exact comparison of the
//      decimal value with the halfway point between the two candidates, in big-integer arithmetic
//      over the first 800 significant digits (+ a sticky bit for the rest: more digits cannot
//      move a value off an exact tie other than upwards).
// Hexadecimal literals ("0x1.8p1") are rounded half-even from their bits.  Internal, not ABI.
#pragma once

#include <cstdint>

#include "dq_pow5_table.h"

#if defined(__HIPCC__)
#define DQ_HD __host__ __device__
#define DQ_HD_NOINLINE __host__ __device__ __attribute__((noinline))
#else
#define DQ_HD
#define DQ_HD_NOINLINE __attribute__((noinline))
#endif

namespace dq {
namespace numparse {

DQ_HD inline int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

DQ_HD inline void mul64x64(uint64_t a, uint64_t b, uint64_t* hi, uint64_t* lo) {
  const uint64_t a0 = (uint32_t)a, a1 = a >> 32, b0 = (uint32_t)b, b1 = b >> 32;
  const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
  const uint64_t mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;
  *lo = (mid << 32) | (uint32_t)p00;
  *hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}

// An IEEE binary64 under construction: mantissa without the implicit bit, biased exponent.
struct Adjusted {
  uint64_t mantissa;
  int32_t power2;  // 0x7FF = infinity
};

constexpr int kMantBits = 52;
constexpr int kMinExp = -1023;
constexpr int kInfPower = 0x7FF;

// Eisel-Lemire: w * 10^q rounded to nearest-even (w != 0, exact).
DQ_HD inline Adjusted eisel_lemire(int64_t q, uint64_t w) {
  Adjusted a;
  if (w == 0 || q < kPow5MinQ) {
    a.mantissa = 0;
    a.power2 = 0;
    return a;
  }
  if (q > kPow5MaxQ) {
    a.mantissa = 0;
    a.power2 = kInfPower;
    return a;
  }
  const int lz = clz64(w);
  w <<= lz;
  const int idx = 2 * (int)(q - kPow5MinQ);
  uint64_t hi, lo;
  mul64x64(w, kPow5Table[idx], &hi, &lo);
  constexpr uint64_t kPrecisionMask = 0xFFFFFFFFFFFFFFFFull >> (kMantBits + 3);
  if ((hi & kPrecisionMask) == kPrecisionMask) {  // the low word may carry into the bits kept
    uint64_t hi2, lo2;
    mul64x64(w, kPow5Table[idx + 1], &hi2, &lo2);
    lo += hi2;
    if (hi2 > lo) ++hi;
  }
  const int upper = (int)(hi >> 63);
  const int shift = upper + 64 - kMantBits - 3;
  a.mantissa = hi >> shift;
  // floor(log2(10^q)) + 63 = ((152170 + 65536) * q >> 16) + 63
  a.power2 = (int32_t)(((((152170 + 65536) * q) >> 16) + 63) + upper - lz - kMinExp);
  if (a.power2 <= 0) {  // subnormal (or zero)
    if (-a.power2 + 1 >= 64) {
      a.mantissa = 0;
      a.power2 = 0;
      return a;
    }
    a.mantissa >>= -a.power2 + 1;
    a.mantissa += (a.mantissa & 1);
    a.mantissa >>= 1;
    a.power2 = (a.mantissa < (1ull << kMantBits)) ? 0 : 1;
    return a;
  }
  // an exact product sitting on a tie rounds to even (only possible for small |q|)
  if (lo <= 1 && q >= -4 && q <= 23 && (a.mantissa & 3) == 1) {
    if ((a.mantissa << shift) == hi) a.mantissa &= ~1ull;
  }
  a.mantissa += (a.mantissa & 1);
  a.mantissa >>= 1;
  if (a.mantissa >= (2ull << kMantBits)) {
    a.mantissa = 1ull << kMantBits;
    ++a.power2;
  }
  a.mantissa &= ~(1ull << kMantBits);
  if (a.power2 >= kInfPower) {
    a.power2 = kInfPower;
    a.mantissa = 0;
  }
  return a;
}

DQ_HD inline uint64_t adjusted_bits(const Adjusted& a) { return a.mantissa | ((uint64_t)a.power2 << kMantBits); }

// ---- fixed-size big integers for tier 3 (little-endian 32-bit limbs)
constexpr int kBigLimbs = 112;  // 3584 bits: 800 digits (2658 bits) x 2^shift, or 54 bits x 5^1124 x 2^shift
struct Big {
  uint32_t w[kBigLimbs];
  int n;  // limbs in use (no high zero limbs)
};

DQ_HD inline void big_set(Big& b, uint64_t v) {
  b.w[0] = (uint32_t)v;
  b.w[1] = (uint32_t)(v >> 32);
  b.n = b.w[1] ? 2 : (b.w[0] ? 1 : 0);
}

DQ_HD inline bool big_muladd(Big& b, uint32_t m, uint32_t add) {  // false on overflow
  uint64_t carry = add;
  for (int i = 0; i < b.n; ++i) {
    const uint64_t t = (uint64_t)b.w[i] * m + carry;
    b.w[i] = (uint32_t)t;
    carry = t >> 32;
  }
  if (carry) {
    if (b.n == kBigLimbs) return false;
    b.w[b.n++] = (uint32_t)carry;
  }
  return true;
}

DQ_HD inline bool big_mul_pow5(Big& b, int64_t e) {
  while (e >= 13) {
    if (!big_muladd(b, 1220703125u, 0u)) return false;  // 5^13
    e -= 13;
  }
  uint32_t m = 1;
  for (int64_t i = 0; i < e; ++i) m *= 5u;
  return big_muladd(b, m, 0u);
}

DQ_HD inline bool big_shl(Big& b, int64_t s) {
  if (b.n == 0 || s == 0) return true;
  const int64_t limbs = s >> 5;
  const int bits = (int)(s & 31);
  if (b.n + limbs + 1 > kBigLimbs) return false;
  if (bits) {
    uint32_t carry = 0;
    for (int i = 0; i < b.n; ++i) {
      const uint32_t v = b.w[i];
      b.w[i] = (v << bits) | carry;
      carry = v >> (32 - bits);
    }
    if (carry) b.w[b.n++] = carry;
  }
  if (limbs) {
    for (int i = b.n - 1; i >= 0; --i) b.w[i + limbs] = b.w[i];
    for (int64_t i = 0; i < limbs; ++i) b.w[i] = 0u;
    b.n += (int)limbs;
  }
  return true;
}

DQ_HD inline int big_cmp(const Big& a, const Big& b) {
  if (a.n != b.n) return a.n < b.n ? -1 : 1;
  for (int i = a.n - 1; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}

// The digit string of a decimal literal: its significant digits are the bytes [i0, i1) (a '.' at
// `dot` is skipped, dot < 0: none) and value = int(digits) * 10^exp10.
struct DecimalSpan {
  int32_t i0, i1, dot;
  int64_t exp10;
};

constexpr int kMaxBigDigits = 800;

// Tier 3: the exact value compared with the halfway point above candidate `lo_bits` (the value
// lies in [lo, next(lo)] ); returns the correctly rounded bits.
template <typename Src>
DQ_HD_NOINLINE uint64_t decimal_slow(const Src& p, const DecimalSpan& d, uint64_t lo_bits) {
  Big a, b;
  a.n = 0;
  bool sticky = false;
  int kept = 0;
  int64_t dropped = 0;
  uint32_t chunk = 0, chunk_mul = 1;
  for (int32_t i = d.i0; i < d.i1; ++i) {
    if (i == d.dot) continue;
    const uint32_t dg = p[i] - 48u;
    if (kept < kMaxBigDigits) {
      chunk = chunk * 10u + dg;
      chunk_mul *= 10u;
      ++kept;
      if (chunk_mul == 1000000000u) {
        big_muladd(a, chunk_mul, chunk);
        chunk = 0;
        chunk_mul = 1;
      }
    } else {
      sticky = sticky || dg != 0;
      ++dropped;
    }
  }
  if (chunk_mul > 1) big_muladd(a, chunk_mul, chunk);
  const int64_t q = d.exp10 + dropped;  // value ~ a * 10^q (+ sticky)
  // halfway = (2m + 1) * 2^(e - 1), with lo = m * 2^e
  const uint64_t biased = (lo_bits >> kMantBits) & 0x7FF;
  const uint64_t frac = lo_bits & ((1ull << kMantBits) - 1);
  const uint64_t m = biased ? (frac | (1ull << kMantBits)) : frac;
  const int64_t e = biased ? (int64_t)biased - 1075 : -1074;
  big_set(b, 2 * m + 1);
  // compare a * 5^q * 2^q with b * 2^(e - 1)
  int64_t sh = q - (e - 1);  // a side's power of two relative to b's
  if (q >= 0) {
    big_mul_pow5(a, q);
  } else {
    big_mul_pow5(b, -q);
  }
  if (sh >= 0) big_shl(a, sh);
  else big_shl(b, -sh);
  const int c = big_cmp(a, b);
  if (c > 0 || (c == 0 && sticky)) return lo_bits + 1;
  if (c < 0) return lo_bits;
  return (m & 1) ? lo_bits + 1 : lo_bits;  // an exact tie: to even
}

// Hexadecimal significand [i0, i1) (a '.' at dot skipped), binary exponent bexp: round half-even.
template <typename Src>
DQ_HD inline uint64_t hex_bits(const Src& p, int32_t i0, int32_t i1, int32_t dot, int64_t bexp) {
  uint64_t m = 0;
  int32_t nd = 0;  // significant hex digits in m (<= 15)
  bool sticky = false, seen = false;
  int64_t e2 = bexp;
  for (int32_t i = i0; i < i1; ++i) {
    if (i == dot) continue;
    const uint32_t c = p[i];
    const uint32_t v = c <= '9' ? c - '0' : (c | 0x20u) - 'a' + 10u;
    const bool frac = dot >= 0 && i > dot;
    if (!seen && v == 0) {
      if (frac) e2 -= 4;
      continue;
    }
    seen = true;
    if (nd < 15) {
      m = (m << 4) | v;
      ++nd;
      if (frac) e2 -= 4;
    } else {
      sticky = sticky || v != 0;
      if (!frac) e2 += 4;
    }
  }
  if (m == 0) return 0;
  // value = m * 2^e2 (+ sticky below m's last bit), m normalised to [2^63, 2^64)
  const int lz = clz64(m);
  m <<= lz;
  e2 -= lz;
  int64_t lead = e2 + 63;  // exponent of the leading bit
  // significant bits kept: 53, fewer for a subnormal (the last kept bit weighs 2^-1074)
  const int64_t keep = lead >= -1022 ? 53 : 53 - (-1022 - lead);
  if (keep <= 0) {  // below 2^-1074: 2^-1075 exactly is a tie with 0 (even), above it the minimum
    return (keep == 0 && (m > (1ull << 63) || sticky)) ? 1ull : 0ull;
  }
  const int drop = 64 - (int)keep;
  uint64_t r = m >> drop;
  const uint64_t rem = m & ((1ull << drop) - 1), half = 1ull << (drop - 1);
  if (rem > half || (rem == half && (sticky || (r & 1)))) ++r;
  if (lead < -1022) return r;  // the subnormal's mantissa field (2^52 = the smallest normal)
  if (r >> 53) {
    r >>= 1;
    ++lead;
  }
  if (lead > 1023) return 0x7FF0000000000000ull;
  return (r & ((1ull << kMantBits) - 1)) | ((uint64_t)(lead + 1023) << kMantBits);
}

DQ_HD inline bool is_java_ws(uint32_t c) { return c <= 0x20u; }  // String.trim()

template <typename Src>
DQ_HD inline bool bytes_are(const Src& p, int32_t at, int32_t n, const char* w, int32_t len) {
  if (n != len) return false;
  for (int32_t k = 0; k < len; ++k)
    if (p[at + k] != (uint32_t)(uint8_t)w[k]) return false;
  return true;
}

DQ_HD inline double bits_double(uint64_t b) {
  union {
    uint64_t u;
    double d;
  } x;
  x.u = b;
  return x.d;
}

constexpr double kPow10Exact[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                    1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Double.parseDouble(s) (whitespace <= U+0020 trimmed): 0 = NumberFormatException (NULL in Spark),
// 1 = *out holds the correctly rounded value.
template <typename Src>
DQ_HD int parse_double(const Src& p, int32_t n, double* out) {
  int32_t i = 0, e = n;
  while (i < e && is_java_ws(p[i])) ++i;
  while (e > i && is_java_ws(p[e - 1])) --e;
  if (i == e) return 0;
  bool neg = false;
  if (p[i] == '+' || p[i] == '-') {
    neg = p[i] == '-';
    ++i;
  }
  const uint64_t sign = neg ? (1ull << 63) : 0ull;
  if (bytes_are(p, i, e - i, "NaN", 3)) {
    *out = bits_double(0x7ff8000000000000ull);
    return 1;
  }
  if (bytes_are(p, i, e - i, "Infinity", 8)) {
    *out = bits_double(sign | 0x7ff0000000000000ull);
    return 1;
  }
  if (e - i >= 2 && p[i] == '0' && (p[i + 1] == 'x' || p[i + 1] == 'X')) {
    // HexSignificand BinaryExponent [fFdD]: 0x h* [. h*] p [+-] d+  (at least one hex digit)
    int32_t j = i + 2, dot = -1, nh = 0;
    const int32_t h0 = j;
    for (; j < e; ++j) {
      const uint32_t c = p[j];
      if (c == '.') {
        if (dot >= 0) return 0;
        dot = j;
        continue;
      }
      const bool hx = (c - '0' < 10u) || ((c | 0x20u) - 'a' < 6u);
      if (!hx) break;
      ++nh;
    }
    const int32_t h1 = j;
    if (nh == 0 || j >= e || (p[j] | 0x20u) != 'p') return 0;
    ++j;
    bool eneg = false;
    if (j < e && (p[j] == '+' || p[j] == '-')) {
      eneg = p[j] == '-';
      ++j;
    }
    int32_t end = e;
    const uint32_t last = p[e - 1];
    if (last == 'f' || last == 'F' || last == 'd' || last == 'D') --end;
    if (j >= end) return 0;
    int64_t x = 0;
    for (; j < end; ++j) {
      const uint32_t dg = p[j] - 48u;
      if (dg > 9u) return 0;
      if (x < 100000000000ll) x = x * 10 + (int64_t)dg;
    }
    *out = bits_double(sign | hex_bits(p, h0, h1, dot, eneg ? -x : x));
    return 1;
  }
  const uint32_t last = p[e - 1];  // optional f/F/d/D type suffix
  if (last == 'f' || last == 'F' || last == 'd' || last == 'D') --e;
  DecimalSpan span;
  span.dot = -1;
  span.i0 = -1;
  uint64_t m = 0;
  int32_t sig = 0, ndig = 0;
  int64_t exp10 = 0;
  int64_t xexp = 0;  // the explicit exponent
  bool dropped = false, dot = false;
  while (i < e) {
    const uint32_t c = p[i];
    if (c == '.') {
      if (dot) return 0;
      dot = true;
      span.dot = i;
      ++i;
      continue;
    }
    const uint32_t dg = c - 48u;
    if (dg > 9u) break;
    ++ndig;
    if (m == 0 && dg == 0 && sig == 0) {  // leading zeros carry no significance
      if (dot) --exp10;
    } else {
      if (span.i0 < 0) span.i0 = i;
      if (sig < 19) {
        m = m * 10u + dg;
        if (dot) --exp10;
      } else {
        dropped = dropped || dg != 0;
        if (!dot) ++exp10;
      }
      ++sig;
    }
    ++i;
  }
  span.i1 = i;
  if (ndig == 0) return 0;
  if (i < e) {  // exponent
    const uint32_t c = p[i];
    if (c != 'e' && c != 'E') return 0;
    ++i;
    bool eneg = false;
    if (i < e && (p[i] == '+' || p[i] == '-')) {
      eneg = p[i] == '-';
      ++i;
    }
    if (i == e) return 0;
    int64_t x = 0;
    while (i < e) {
      const uint32_t dg = p[i] - 48u;
      if (dg > 9u) return 0;
      if (x < 100000000000ll) x = x * 10 + (int64_t)dg;
      ++i;
    }
    xexp = eneg ? -x : x;
    exp10 += xexp;
  }
  if (m == 0) {
    *out = bits_double(sign);
    return 1;
  }
  if (!dropped && m <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {  // tier 1
    double v = (double)m;  // exact
    v = exp10 >= 0 ? v * kPow10Exact[exp10] : v / kPow10Exact[-exp10];
    *out = neg ? -v : v;
    return 1;
  }
  const Adjusted a = eisel_lemire(exp10, m);  // tier 2
  uint64_t bits = adjusted_bits(a);
  if (dropped) {
    const Adjusted b = eisel_lemire(exp10, m + 1);
    const uint64_t bits_hi = adjusted_bits(b);
    if (bits_hi != bits) {  // tier 3: the value lies within [bits, bits_hi]
      // value = int(digits [i0, i1)) * 10^(X - digits of [i0, i1) after the point)
      // (zeros between the point and i0 are digits after the point too)
      const int64_t frac = (span.dot >= 0 && span.dot < span.i1) ? span.i1 - span.dot - 1 : 0;
      span.exp10 = xexp - frac;
      bits = decimal_slow(p, span, bits);
    }
  }
  *out = bits_double(sign | bits);
  return 1;
}

}  // namespace numparse
}  // namespace dq
