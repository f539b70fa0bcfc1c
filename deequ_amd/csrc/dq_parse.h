// dq_parse.h -- device parsers of Spark 2.2.2's string casts, shared by the ColumnProfiler cast
// kernel (dq_profile.hip) and the predicate interpreter's Cast(StringType -> DoubleType)
// (dq_pred.hip): UTF8String.toLong, and java.lang.Double.parseDouble of the trimmed string,
// correctly rounded for every input (dq_numparse.h).  Internal, not ABI.
#pragma once

#include "dq_internal.h"
#include "dq_numparse.h"

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

// Double.parseDouble: 0 = NumberFormatException (NULL), 1 = value (correctly rounded)
template <typename Src>
__device__ inline int parse_double(const Src& p, int32_t n, double* out) {
  return numparse::parse_double(p, n, out);
}

}  // namespace
}  // namespace dq
