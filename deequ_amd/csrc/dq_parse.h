// dq_parse.h -- device parsers of Spark 2.2.2's string casts, shared by the ColumnProfiler cast
// kernel (dq_profile.hip) and the predicate interpreter's Cast(StringType -> DoubleType)
// (dq_pred.hip): java.lang.Double.parseDouble of the trimmed string, exact (correctly rounded) on
// the Clinger fast path, "well formed but off the fast path" reported separately so the caller
// can route the work to Spark instead of returning an inexact value.  Internal, not ABI.
#pragma once

#include "dq_internal.h"

namespace dq {
namespace {

// Byte sources for the parsers: a plain pointer, or (strings of <= 24 bytes) the aligned 8-byte
// words covering the string, loaded once -- 4 vector loads instead of one per byte.  Only words
// holding at least one byte of the string are read (never beyond the page of a valid byte).
struct PtrSrc {
  const uint8_t* p;
  __device__ uint32_t operator[](int32_t i) const { return p[i]; }
};
struct WordSrc {
  uint64_t w0, w1, w2, w3;
  uint32_t sh;
  __device__ WordSrc(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint32_t s)
      : w0(a), w1(b), w2(c), w3(d), sh(s) {}  // words already loaded (bytes past the string: any)
  __device__ WordSrc(const uint8_t* p, int32_t n) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
    sh = (uint32_t)(a & 7);
    const int32_t last = n > 0 ? (int32_t)(sh + n - 1) >> 3 : -1;
    w0 = last >= 0 ? w[0] : 0;
    w1 = last >= 1 ? w[1] : 0;
    w2 = last >= 2 ? w[2] : 0;
    w3 = last >= 3 ? w[3] : 0;
  }
  __device__ uint32_t operator[](int32_t i) const {
    const uint32_t j = sh + (uint32_t)i;
    const uint64_t w = (j >> 3) == 0 ? w0 : (j >> 3) == 1 ? w1 : (j >> 3) == 2 ? w2 : w3;
    return (uint32_t)(w >> ((j & 7u) * 8u)) & 0xffu;
  }
};


__device__ inline bool is_java_ws(uint32_t c) { return c <= 0x20u; }  // String.trim()

// UTF8String.toLong (Spark 2.2): [+-]digits[.digits]; the fraction is validated and dropped.
template <typename Src>
__device__ bool parse_long(const Src& p, int32_t n, int64_t* out) {
  if (n == 0) return false;
  int32_t i = 0;
  const bool neg = p[0] == '-';
  if (neg || p[0] == '+') {
    if (n == 1) return false;
    i = 1;
  }
  const int64_t stop = INT64_MIN / 10;
  int64_t r = 0;  // accumulated negatively, as the reference does, so INT64_MIN parses
  for (; i < n; ++i) {
    const uint32_t b = p[i];
    if (b == '.') {
      ++i;
      break;
    }
    if (b - '0' >= 10u) return false;
    // the reference detects overflow after a wrapping step; here it is checked before the
    // step (no signed overflow): r * 10 - digit >= INT64_MIN
    if (r < stop || (r == stop && (int64_t)(b - '0') > -(INT64_MIN % 10))) return false;
    r = r * 10 - (int64_t)(b - '0');
  }
  for (; i < n; ++i)
    if ((uint32_t)p[i] - '0' >= 10u) return false;
  if (!neg) {
    if (r == INT64_MIN) return false;  // 9223372036854775808 does not fit
    r = -r;
  }
  *out = r;
  return true;
}

__device__ const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

template <typename Src>
__device__ inline bool bytes_are(const Src& p, int32_t at, int32_t n, const char* w, int32_t len) {
  if (n != len) return false;
  for (int32_t k = 0; k < len; ++k)
    if (p[at + k] != (uint32_t)(uint8_t)w[k]) return false;
  return true;
}

// 0 = NULL (NumberFormatException), 1 = value, 2 = well formed but off the exact fast path
template <typename Src>
__device__ int parse_double(const Src& p, int32_t n, double* out) {
  int32_t i = 0, e = n;
  while (i < e && is_java_ws(p[i])) ++i;
  while (e > i && is_java_ws(p[e - 1])) --e;
  if (i == e) return 0;
  bool neg = false;
  if (p[i] == '+' || p[i] == '-') {
    neg = p[i] == '-';
    ++i;
  }
  if (bytes_are(p, i, e - i, "NaN", 3)) {
    *out = __builtin_nan("");
    return 1;
  }
  if (bytes_are(p, i, e - i, "Infinity", 8)) {
    *out = neg ? -__builtin_huge_val() : __builtin_huge_val();
    return 1;
  }
  if (e - i >= 2 && p[i] == '0' && (p[i + 1] == 'x' || p[i + 1] == 'X')) return 2;  // hex float
  const uint32_t last = p[e - 1];  // optional f/F/d/D type suffix
  if (last == 'f' || last == 'F' || last == 'd' || last == 'D') --e;
  uint64_t m = 0;
  int32_t sig = 0, exp10 = 0, ndig = 0;
  bool dropped = false, dot = false;
  while (i < e) {
    const uint32_t c = p[i];
    if (c == '.') {
      if (dot) return 0;
      dot = true;
      ++i;
      continue;
    }
    const uint32_t dg = c - 48u;
    if (dg > 9u) break;
    ++ndig;
    ++i;
    if (m == 0 && dg == 0) {  // leading zeros carry no significance
      if (dot) --exp10;
    } else if (sig < 19) {
      m = m * 10u + dg;
      ++sig;
      if (dot) --exp10;
    } else {
      dropped = dropped || dg != 0;
      if (!dot) ++exp10;
    }
  }
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
    int32_t x = 0;
    while (i < e) {
      const uint32_t dg = p[i] - 48u;
      if (dg > 9u) return 0;
      if (x < 100000) x = x * 10 + (int32_t)dg;
      ++i;
    }
    exp10 += eneg ? -x : x;
  }
  if (m == 0) {
    *out = neg ? -0.0 : 0.0;
    return 1;
  }
  if (dropped || m > (1ull << 53) || exp10 < -22 || exp10 > 22) return 2;
  double v = (double)m;  // exact: m <= 2^53
  v = exp10 >= 0 ? v * kPow10[exp10] : v / kPow10[-exp10];  // one correctly rounded operation
  *out = neg ? -v : v;
  return 1;
}

}  // namespace
}  // namespace dq
