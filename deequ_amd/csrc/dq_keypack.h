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

// The bytes of x below n (n <= 8; the rest ignored): all ASCII digits?  *nib = their values as
// 8 nibbles (byte i -> bits 4i..4i+3; bytes >= n -> 0).
DQ_KP_FN bool kp_digits8(uint64_t x, uint32_t n, uint32_t* nib) {
  const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8u * n)) - 1ull);
  const uint64_t y = (x & m) | (0x3030303030303030ull & ~m);  // pad with '0'
  if (y & 0x8080808080808080ull) return false;                 // not ASCII (the adds below carry)
  // per byte b < 0x80: (b | 0x80) - 0x30 has bit 7 iff b >= '0'; b + 0x46 has bit 7 iff b > '9'
  const uint64_t ge0 = (y | 0x8080808080808080ull) - 0x3030303030303030ull;
  const uint64_t gt9 = y + 0x4646464646464646ull;
  if ((ge0 & ~gt9 & 0x8080808080808080ull) != 0x8080808080808080ull) return false;
  const uint64_t d = y - 0x3030303030303030ull;                // bytes 0..9
  uint64_t t = (d | (d >> 4)) & 0x00FF00FF00FF00FFull;         // byte pairs -> one byte each
  t = (t | (t >> 8)) & 0x0000FFFF0000FFFFull;
  t = (t | (t >> 16)) & 0x00000000FFFFFFFFull;
  *nib = (uint32_t)t;
  return true;
}

// 8 nibbles -> 8 digit bytes, the bytes from n on zero.
DQ_KP_FN uint64_t kp_spread8(uint32_t nib, uint32_t n) {
  uint64_t x = nib;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x += 0x3030303030303030ull;
  return n >= 8 ? x : (n ? x & ((1ull << (8u * n)) - 1ull) : 0ull);
}

// The packed word of an inline key (k0/k1 little-endian key bytes, len <= 15), if it is a digit
// string (false otherwise; "NullValue" is not one -- see kp_pack_record).
DQ_KP_FN bool kp_pack(uint64_t k0, uint64_t k1, uint32_t len, uint64_t* p) {
  if (len > 15) return false;
  uint32_t a, b;
  if (!kp_digits8(k0, len < 8 ? len : 8, &a)) return false;
  if (!kp_digits8(k1, len > 8 ? len - 8 : 0, &b)) return false;
  *p = (uint64_t)a | ((uint64_t)b << 32) | ((uint64_t)len << 60);
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
  const uint32_t n = (uint32_t)(p >> 60);
  *len = n;
  *k0 = kp_spread8((uint32_t)p, n < 8 ? n : 8);
  *k1 = kp_spread8((uint32_t)(p >> 32) & 0x0FFFFFFFu, n > 8 ? n - 8 : 0);
}

}  // namespace dq
