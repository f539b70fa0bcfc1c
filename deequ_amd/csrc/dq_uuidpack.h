// dq_uuidpack.h -- canonical UUID grouping keys in two 8-byte words (host + device).
//
// isUnique / isPrimaryKey / hasUniqueness (Check.scala:140-230) are most often asked of id
// columns holding UUID text: 36 bytes, "xxxxxxxx-xxxx-xxxx-xxxx-xxxxxxxxxxxx" with x a lowercase
// hex digit (java.util.UUID.toString, Python's str(uuid)).  Such a key is longer than a 16-byte
// record holds, so in general it would have to travel by reference into a copy of its bytes --
// and every row of a group would then have to be compared byte for byte against the group's
// first row, two random reads per row.  Its 32 hex digits are exactly 128 bits, though, so the
// partition path stages a canonical UUID as its two words {lo, hi} and groups, compares and
// splits them in registers and LDS like any other 16-byte record; the text is written once per
// GROUP, into the table's key heap, when the aggregation writes the group out.
//   lo bits 16 g .. 16 g + 15 (g < 4): hex group g -- text bytes 0-3, 4-7, 9-12, 14-17
//   hi bits 16 g .. 16 g + 15 (g < 4): hex group 4 + g -- text bytes 19-22, 24-27, 28-31, 32-35
//   inside a group, nibble i (bits 4 i .. 4 i + 3) is the value of the group's byte i.
// The map is a bijection between canonical lowercase UUID strings and 128-bit values; any other
// 36-byte string (uppercase, a misplaced dash, a non-hex byte) does not pack and keeps the
// general path.  The table's hash of a key that packs is hash_raw of its words (dq_freq.hip,
// hash_uuid), wherever the key is hashed -- so it hashes alike as a packed record or as bytes.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DQ_UP_FN __host__ __device__ inline
#else
#define DQ_UP_FN inline
#endif

namespace dq {

constexpr uint32_t kUuidLen = 36;

// 0 if every byte of y is a lowercase hex digit ('0'-'9', 'a'-'f'), else bit 7 of some byte.
DQ_UP_FN uint32_t up_nonhex4(uint32_t y) {
  // per byte b < 0x80: (b | 0x80) - lo keeps bit 7 iff b >= lo; b + (0x7F - hi) sets it iff b > hi
  const uint32_t ge0 = (y | 0x80808080u) - 0x30303030u, gt9 = y + 0x46464646u;  // '0'..'9'
  const uint32_t gea = (y | 0x80808080u) - 0x61616161u, gtf = y + 0x19191919u;  // 'a'..'f'
  const uint32_t digit = ge0 & ~gt9, alpha = gea & ~gtf;
  return (~(digit | alpha) & 0x80808080u) | (y & 0x80808080u);
}

// 4 hex digit bytes (validated) -> 16 bits, byte i -> nibble i.
DQ_UP_FN uint32_t up_nib4(uint32_t y) {
  const uint32_t d = (y & 0x0F0F0F0Fu) + ((y >> 6) & 0x01010101u) * 9u;  // bit 6: a letter
  const uint32_t t = d | (d >> 4);
  return (t & 0xFFu) | ((t >> 8) & 0xFF00u);
}

// 16 bits -> 4 lowercase hex digit bytes (nibble i -> byte i).
DQ_UP_FN uint32_t up_hex4(uint32_t nib) {
  uint32_t x = nib & 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  return x + 0x30303030u + (((x + 0x06060606u) >> 4) & 0x01010101u) * 0x27u;
}

DQ_UP_FN uint32_t up_align(uint32_t hi, uint32_t lo, uint32_t sh) {  // (hi:lo) >> sh, sh in 1..31
  return (lo >> sh) | (hi << (32u - sh));
}

// The 36 text bytes as nine little-endian 32-bit words -> {lo, hi}; false if not canonical.
DQ_UP_FN bool uuid_pack(const uint32_t (&w)[9], uint64_t* lo, uint64_t* hi) {
  const uint32_t g2 = up_align(w[3], w[2], 8), g3 = up_align(w[4], w[3], 16), g4 = up_align(w[5], w[4], 24);
  const uint32_t dashes = (w[2] & 0xFFu) | (w[3] & 0xFF00u) | (w[4] & 0xFF0000u) | (w[5] & 0xFF000000u);
  const uint32_t bad = up_nonhex4(w[0]) | up_nonhex4(w[1]) | up_nonhex4(g2) | up_nonhex4(g3) | up_nonhex4(g4) |
                       up_nonhex4(w[6]) | up_nonhex4(w[7]) | up_nonhex4(w[8]);
  if (bad || dashes != 0x2D2D2D2Du) return false;
  *lo = (uint64_t)(up_nib4(w[0]) | (up_nib4(w[1]) << 16)) | ((uint64_t)(up_nib4(g2) | (up_nib4(g3) << 16)) << 32);
  *hi = (uint64_t)(up_nib4(g4) | (up_nib4(w[6]) << 16)) | ((uint64_t)(up_nib4(w[7]) | (up_nib4(w[8]) << 16)) << 32);
  return true;
}

// {lo, hi} -> the 36 text bytes as nine words (w[9], the heap's padding word, is 0).
DQ_UP_FN void uuid_unpack(uint64_t lo, uint64_t hi, uint32_t (&w)[10]) {
  const uint32_t c0 = up_hex4((uint32_t)lo), c1 = up_hex4((uint32_t)(lo >> 16));
  const uint32_t c2 = up_hex4((uint32_t)(lo >> 32)), c3 = up_hex4((uint32_t)(lo >> 48));
  const uint32_t c4 = up_hex4((uint32_t)hi), c5 = up_hex4((uint32_t)(hi >> 16));
  const uint32_t c6 = up_hex4((uint32_t)(hi >> 32)), c7 = up_hex4((uint32_t)(hi >> 48));
  w[0] = c0;
  w[1] = c1;
  w[2] = 0x2Du | (c2 << 8);
  w[3] = (c2 >> 24) | 0x2D00u | (c3 << 16);
  w[4] = (c3 >> 16) | 0x2D0000u | (c4 << 24);
  w[5] = (c4 >> 8) | 0x2D000000u;
  w[6] = c5;
  w[7] = c6;
  w[8] = c7;
  w[9] = 0u;
}

// A key given as bytes (any length): its packed words if it is a canonical UUID.
DQ_UP_FN bool uuid_pack_bytes(const uint8_t* p, uint32_t len, uint64_t* lo, uint64_t* hi) {
  if (len != kUuidLen) return false;
  uint32_t w[9];
  for (int i = 0; i < 9; ++i)
    w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
           ((uint32_t)p[4 * i + 3] << 24);
  return uuid_pack(w, lo, hi);
}

}  // namespace dq
