/* Search for values whose Spark XXH64 (seed 42) lands on the rare branches of the device HLL
 * slot computation (deequ_amd/csrc/dq_internal.h hll_slot): x = hash, w = (x << 9) | 0x100,
 *   rare1: bits 54..32 of x are zero (the high word of x << 9 comes only from the low word),
 *   rare2: bits 54..23 of x are zero (the high word of w is zero; nlz >= 32).
 * Prints "<kind> <width> <value>" lines; width 8 = hashLong of an int64 (or the bits of a double),
 * width 4 = hashInt of an int32.  Test-fixture generator only (tests/golden/make_hll_rare.py). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define P1 0x9E3779B185EBCA87ull
#define P2 0xC2B2AE3D27D4EB4Full
#define P3 0x165667B19E3779F9ull
#define P4 0x85EBCA77C2B2AE63ull
#define P5 0x27D4EB2F165667C5ull
static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t aval(uint64_t h) {
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32; return h;
}
static inline uint64_t h8(uint64_t v) {
  uint64_t h = 42 + P5 + 8;
  h ^= rotl(v * P2, 31) * P1;
  return aval(rotl(h, 27) * P1 + P4);
}
static inline uint64_t h4(uint32_t v) {
  uint64_t h = 42 + P5 + 4;
  h ^= (uint64_t)v * P1;
  return aval(rotl(h, 23) * P2 + P3);
}
static int kind(uint64_t x) {
  if (((x >> 23) & ((1ull << 32) - 1)) == 0) return 2;
  if (((x >> 32) & ((1ull << 23) - 1)) == 0) return 1;
  return 0;
}

int main(int argc, char** argv) {
  const uint64_t base8 = argc > 1 ? strtoull(argv[1], 0, 0) : 0;
  const uint64_t n8 = argc > 2 ? strtoull(argv[2], 0, 0) : (1ull << 33);
  int found1 = 0, found2 = 0;
  for (uint64_t i = 0; i < n8 && (found1 < 4 || found2 < 2); ++i) {
    const uint64_t v = base8 + i;
    const int k = kind(h8(v));
    if (k == 1 && found1 < 4) { printf("rare1 8 %llu\n", (unsigned long long)v); ++found1; }
    if (k == 2 && found2 < 2) { printf("rare2 8 %llu\n", (unsigned long long)v); ++found2; }
  }
  int f4_1 = 0, f4_2 = 0;
  for (uint64_t v = 0; v < (1ull << 32) && (f4_1 < 4 || f4_2 < 1); ++v) {
    const int k = kind(h4((uint32_t)v));
    if (k == 1 && f4_1 < 4) { printf("rare1 4 %lld\n", (long long)(int32_t)(uint32_t)v); ++f4_1; }
    if (k == 2 && f4_2 < 1) { printf("rare2 4 %lld\n", (long long)(int32_t)(uint32_t)v); ++f4_2; }
  }
  return 0;
}
