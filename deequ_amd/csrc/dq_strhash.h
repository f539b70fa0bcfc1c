// dq_strhash.h -- Spark XXH64.hashUnsafeBytes (seed 42) of utf8 strings on the device, shared
// by the HLL kernel (dq_hll.hip) and the fused profiler string pass (dq_profile.hip).
// Reference: catalyst/StatefulHyperloglogPlus.scala:89-115 (XxHash64Function over the UTF-8
// bytes), Spark 2.2.2 XXH64.hashUnsafeBytes.
#pragma once
#include "dq_internal.h"

namespace dq {
namespace {

// Unaligned little-endian loads that only touch aligned words containing at least one byte
// of [p, end): such a word never leaves the page of that byte, so this is memory safe.
__device__ inline uint64_t ld64(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(a & 7) * 8u;
  if (sh == 0) return w[0];
  return (w[0] >> sh) | (w[1] << (64u - sh));
}
__device__ inline uint32_t ld32(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8u;
  if (sh == 0) return w[0];
  return (w[0] >> sh) | (w[1] << (32u - sh));
}

// [p, p + n), n <= 7, little-endian and zero padded: the one or two aligned 8-byte words that
// hold a byte of the range (never a word without one, so never beyond the page of a valid byte).
__device__ inline uint64_t ld_tail(const uint8_t* p, uint32_t n) {
  const uintptr_t a = (uintptr_t)p;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(a & 7) * 8u;
  uint64_t v = w[0] >> sh;
  if (sh && (a & 7) + n > 8) v |= w[1] << (64u - sh);
  return v & ((1ull << (8u * n)) - 1ull);
}

// XXH64 (Spark XXH64.hashUnsafeBytes) over [p, p + len).
__device__ uint64_t xxh64_bytes(const uint8_t* p, int64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xxh_round(v1, ld64(p));
      v2 = xxh_round(v2, ld64(p + 8));
      v3 = xxh_round(v3, ld64(p + 16));
      v4 = xxh_round(v4, ld64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h ^= xxh_round(0, v1); h = h * kP1 + kP4;
    h ^= xxh_round(0, v2); h = h * kP1 + kP4;
    h ^= xxh_round(0, v3); h = h * kP1 + kP4;
    h ^= xxh_round(0, v4); h = h * kP1 + kP4;
  } else {
    h = seed + kP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xxh_round(0, ld64(p));
    h = rotl64(h, 27) * kP1 + kP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)ld32(p) * kP1;
    h = rotl64(h, 23) * kP2 + kP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * kP5;
    h = rotl64(h, 11) * kP1;
    ++p;
  }
  return xxh_avalanche(h);
}

// Spark XXH64.hashUnsafeBytes (seed 42) of a string shorter than 32 bytes, on 32-bit halves
// like the scan kernel's hashLong (dq_internal.h), returned in the pre-final form hll_slot
// reads.  Same steps as xxh64_bytes below 32 bytes: h = seed + P5 + len, one round per 8-byte
// word, then a 4-byte word, then single bytes, then the avalanche.  The first two 8-byte words
// come in preloaded (q[0], q[1]; valid when len >= 8 / 16).
__device__ inline W64 xxh64_short_dev(const uint8_t* p, uint32_t len, const uint64_t* q) {
  const uint64_t h0 = 42ull + kP5 + len;
  W64 h = {(uint32_t)h0, (uint32_t)(h0 >> 32)};
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    const uint64_t w = i < 16 ? q[i >> 3] : ld64(p + i);
    const W64 k = w64_mul<kP1>(w64_rotl<31>(w64_mul<kP2>({(uint32_t)w, (uint32_t)(w >> 32)})));
    h.lo ^= k.lo;
    h.hi ^= k.hi;
    h = w64_mul<kP1, kP4>(w64_rotl<27>(h));
  }
  // the < 8-byte tail: loaded once (the aligned words holding it), its 4-byte word and single
  // bytes then come out of that register instead of one memory access each
  uint64_t tail = i < len ? ld_tail(p + i, len - i) : 0ull;
  if (i + 4 <= len) {
    const uint32_t w = (uint32_t)tail;
    tail >>= 32;
    const uint64_t pr = (uint64_t)w * (uint32_t)kP1;
    h.lo ^= (uint32_t)pr;
    h.hi ^= (uint32_t)(pr >> 32) + w * (uint32_t)(kP1 >> 32);
    h = w64_mul<kP2, kP3>(w64_rotl<23>(h));
    i += 4;
  }
  for (; i < len; ++i, tail >>= 8) {
    const uint32_t b = (uint32_t)tail & 0xffu;
    const uint64_t pr = (uint64_t)b * (uint32_t)kP5;
    h.lo ^= (uint32_t)pr;
    h.hi ^= (uint32_t)(pr >> 32) + b * (uint32_t)(kP5 >> 32);
    h = w64_mul<kP1>(w64_rotl<11>(h));
  }
  return w64_avalanche_pre32(h);
}

// The same hash of a string of n <= 24 bytes whose bytes 8k..8k+7 are s[k] (already funnel
// shifted out of the aligned words; bytes past n are masked here), in the pre-final form.
__device__ inline W64 xxh64_words_dev(const uint64_t (&s)[3], uint32_t len) {
  const uint64_t h0 = 42ull + kP5 + len;
  W64 h = {(uint32_t)h0, (uint32_t)(h0 >> 32)};
  uint32_t i = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (i + 8 <= len) {
      const uint64_t w = s[k];
      const W64 kk = w64_mul<kP1>(w64_rotl<31>(w64_mul<kP2>({(uint32_t)w, (uint32_t)(w >> 32)})));
      h.lo ^= kk.lo;
      h.hi ^= kk.hi;
      h = w64_mul<kP1, kP4>(w64_rotl<27>(h));
      i += 8;
    }
  }
  uint64_t tail = 0ull;
  if (i < len) {
    const uint32_t r = len - i;  // 1..7
    const uint64_t w = i == 0 ? s[0] : (i == 8 ? s[1] : s[2]);
    tail = w & ((1ull << (8u * r)) - 1ull);
  }
  if (i + 4 <= len) {
    const uint32_t w = (uint32_t)tail;
    tail >>= 32;
    const uint64_t pr = (uint64_t)w * (uint32_t)kP1;
    h.lo ^= (uint32_t)pr;
    h.hi ^= (uint32_t)(pr >> 32) + w * (uint32_t)(kP1 >> 32);
    h = w64_mul<kP2, kP3>(w64_rotl<23>(h));
    i += 4;
  }
  for (; i < len; ++i, tail >>= 8) {
    const uint32_t b = (uint32_t)tail & 0xffu;
    const uint64_t pr = (uint64_t)b * (uint32_t)kP5;
    h.lo ^= (uint32_t)pr;
    h.hi ^= (uint32_t)(pr >> 32) + b * (uint32_t)(kP5 >> 32);
    h = w64_mul<kP1>(w64_rotl<11>(h));
  }
  return w64_avalanche_pre32(h);
}

// Any length, from memory (the pre-final form).
__device__ inline W64 xxh64_utf8_dev(const uint8_t* p, uint32_t len) {
  if (len < 32) {
    const uint64_t q[2] = {len >= 8 ? ld64(p) : 0ull, len >= 16 ? ld64(p + 8) : 0ull};
    return xxh64_short_dev(p, len, q);
  }
  const uint64_t x = xxh64_bytes(p, (int64_t)len, 42);
  return {(uint32_t)x ^ (uint32_t)(x >> 32), (uint32_t)(x >> 32)};
}

}  // namespace
}  // namespace dq
