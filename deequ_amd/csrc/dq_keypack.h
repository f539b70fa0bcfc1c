// dq_keypack.h -- digit-string grouping keys in one 8-byte word (host + device).
//
// The partition path of the group-by (dq_freq.hip) moves every staged record three times
// (stage -> level-1 regions, -> slice regions, -> aggregation).  Keys of at most 15 ASCII
// digits -- decimal ids, the shape of C4's 12-digit keys -- pack into ONE word, so those
// stagings move 8-byte records instead of 16-byte ones:
//   bits 4i .. 4i+3 : byte i of the key minus '0' (0..9), i < 15; nibbles past the key are 0
//   bits 60 .. 63   : the key's length (0..15)
// Codes no digit key packs to (nibble 0 is 0xA..0xF):
//   kPackNull    = Histogram's "NullValue" group (Histogram.scala:63-64), so a NULL-as-key
//                  staging stays packed;
//   kPackEmpty   = a free LDS slot;
//   kPackForeign = an LDS slot holding a table group that is not a digit key (never matches).
// The table itself keeps the key bytes (k0/k1 little-endian, as every other path writes them).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DQ_KP_FN __host__ __device__ inline
#else
#define DQ_KP_FN inline
#endif

namespace dq {

constexpr uint64_t kPackNull = 0xAull;
constexpr uint64_t kPackEmpty = ~0ull;
constexpr uint64_t kPackForeign = ~0ull - 1ull;
constexpr uint64_t kNullK0 = 0x756c61566c6c754eull;  // "NullValu"
constexpr uint64_t kNullK1 = 0x65ull;                // "e"

// 32-bit halves throughout: the VALU is 32 bits wide, so the work is done per 4-byte word.
// Low n bytes of a word (n clamped to 0..4), the rest '0'.
DQ_KP_FN uint32_t kp_pad4(uint32_t w, int32_t n) {
  const uint32_t m = n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
  return (w & m) | (0x30303030u & ~m);
}

// 0 if every byte of y (padded) is an ASCII digit, else bit 7 of some byte.
DQ_KP_FN uint32_t kp_nondigit4(uint32_t y) {
  // per byte b < 0x80: (b | 0x80) - 0x30 keeps bit 7 iff b >= '0'; b + 0x46 sets it iff b > '9'
  const uint32_t ge0 = (y | 0x80808080u) - 0x30303030u;
  const uint32_t gt9 = y + 0x46464646u;  // (a byte >= 0x80 carries; it is caught by y itself)
  return (~ge0 | gt9 | y) & 0x80808080u;
}

// 4 digit bytes -> 4 nibbles (byte i -> bits 4i..4i+3).
DQ_KP_FN uint32_t kp_nib4(uint32_t y) {
  const uint32_t d = y - 0x30303030u;  // bytes 0..9, no borrow
  const uint32_t t = d | (d >> 4);      // bytes 0 and 2 hold the pairs
  return (t & 0xFFu) | ((t >> 8) & 0xFF00u);
}

// 4 nibbles -> 4 digit bytes, the bytes from n on zero.
DQ_KP_FN uint32_t kp_spread4(uint32_t nib, int32_t n) {
  uint32_t x = nib & 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x += 0x30303030u;
  const uint32_t m = n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
  return x & m;
}

// The packed word of an inline key (k0/k1 little-endian key bytes, len <= 15), if it is a digit
// string (false otherwise; "NullValue" is not one -- see kp_pack_record).
DQ_KP_FN bool kp_pack(uint64_t k0, uint64_t k1, uint32_t len, uint64_t* p) {
  if (len > 15) return false;
  const int32_t n = (int32_t)len;
  const uint32_t y0 = kp_pad4((uint32_t)k0, n), y1 = kp_pad4((uint32_t)(k0 >> 32), n - 4);
  const uint32_t y2 = kp_pad4((uint32_t)k1, n - 8), y3 = kp_pad4((uint32_t)(k1 >> 32), n - 12);
  if (kp_nondigit4(y0) | kp_nondigit4(y1) | kp_nondigit4(y2) | kp_nondigit4(y3)) return false;
  const uint32_t lo = kp_nib4(y0) | (kp_nib4(y1) << 16);
  const uint32_t hi = kp_nib4(y2) | (kp_nib4(y3) << 16) | (len << 28);  // (nibble 15 is 0: len <= 15)
  *p = (uint64_t)lo | ((uint64_t)hi << 32);
  return true;
}

// A staged record's word: a digit key, or Histogram's "NullValue" (kPackNull).
DQ_KP_FN bool kp_pack_record(uint64_t k0, uint64_t k1, uint32_t len, uint64_t* p) {
  if (kp_pack(k0, k1, len, p)) return true;
  if (len == 9 && k0 == kNullK0 && k1 == kNullK1) {
    *p = kPackNull;
    return true;
  }
  return false;
}

DQ_KP_FN void kp_unpack(uint64_t p, uint64_t* k0, uint64_t* k1, uint32_t* len) {
  if (p == kPackNull) {
    *k0 = kNullK0;
    *k1 = kNullK1;
    *len = 9;
    return;
  }
  const uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
  const int32_t n = (int32_t)(hi >> 28);
  *len = (uint32_t)n;
  *k0 = (uint64_t)kp_spread4(lo, n) | ((uint64_t)kp_spread4(lo >> 16, n - 4) << 32);
  *k1 = (uint64_t)kp_spread4(hi, n - 8) | ((uint64_t)kp_spread4((hi >> 16) & 0x0FFFu, n - 12) << 32);
}

}  // namespace dq
