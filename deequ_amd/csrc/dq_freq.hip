// dq_freq.hip -- GPU hash group-by for the frequency-based analyzers.
//
// Replaces FrequencyBasedAnalyzer.computeFrequencies (analyzers/GroupingAnalyzers.scala:53-80):
//   SELECT cols, COUNT(*) FROM data WHERE cols NOT NULL GROUP BY cols
// and the group-by of Histogram.computeStateFrom (Histogram.scala:54-69, NULL -> "NullValue").
// The metrics (Uniqueness, Distinctness, CountDistinct, UniqueValueRatio, Entropy,
// Histogram) depend only on the multiset of group counts, so after the group-by a second
// kernel builds a count-of-counts histogram (integer, order independent); the host turns it
// into metrics in a fixed order -- bitwise reproducible whatever the insert schedule.
//
// Table: open addressing with linear probing in HBM, 32-byte slots
//   ctrl  = tag(32) << 32 | READY | HEAP | len(24)     (0 = empty)
//   count = number of rows in the group
//   k0,k1 = the key bytes when len <= 16, else {heap offset, 0} into the key heap
// Every access to another workgroup's slot is a device-scope atomic RMW (CAS to probe/claim,
// atomic exchange to write the key, fetch-or to read it, fetch-add for the count): RMW
// atomics are coherent across the eight XCDs, plain loads of another XCD's stores are not
// (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement & inter-workgroup visibility").
//
// Each workgroup first aggregates in an LDS table (kLdsSlots keys); rows whose key does not
// find room there go straight to the global table.  Low-cardinality / skewed columns therefore
// cost one global atomic per (workgroup, key) instead of one per row.
#include "dq_internal.h"
#include "dq_keypack.h"
#include "dq_uuidpack.h"

#include <cstdio>
#include <cstring>
#include <type_traits>

namespace dq {

namespace {

constexpr unsigned long long kReady = 1ull << 31;
constexpr unsigned long long kHeapKey = 1ull << 30;
constexpr unsigned long long kLenMask = (1ull << 24) - 1;
constexpr int kLdsSlots = 1024;       // LDS pre-aggregation slots per workgroup
constexpr int kLdsProbe = 8;          // linear probes in LDS before going global
#ifndef DQ_INSERT_R
#define DQ_INSERT_R 4
#endif

__device__ inline unsigned long long atom_or(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long atom_read(unsigned long long* p) { return atom_or(p, 0ull); }

// Unaligned little-endian 8-byte read of p[0..n) (n <= 8), zero padded, touching only aligned
// words that contain at least one byte of the range (never leaves the page of a valid byte).
__device__ inline uint64_t ld_partial(const uint8_t* p, uint32_t n) {
  if (n == 0) return 0;
  const uintptr_t a = (uintptr_t)p;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(a & 7) * 8u;
  uint64_t v = w[0] >> sh;
  if (sh && (a & 7) + n > 8) v |= w[1] << (64u - sh);
  return n >= 8 ? v : (v & ((1ull << (8u * n)) - 1ull));
}

__device__ uint64_t xxh64_any(const uint8_t* p, uint32_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    while (p + 32 <= end) {
      v1 = xxh_round(v1, ld_partial(p, 8));
      v2 = xxh_round(v2, ld_partial(p + 8, 8));
      v3 = xxh_round(v3, ld_partial(p + 16, 8));
      v4 = xxh_round(v4, ld_partial(p + 24, 8));
      p += 32;
    }
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
    h ^= xxh_round(0, ld_partial(p, 8));
    h = rotl64(h, 27) * kP1 + kP4;
    p += 8;
  }
  if (p < end) {  // tail <= 7 bytes folded as one word (a deterministic variant, not XXH64)
    h ^= ld_partial(p, (uint32_t)(end - p)) * kP5;
    h = rotl64(h, 11) * kP1;
  }
  return xxh_avalanche(h);
}

// The table hash of an inline key (len <= 16).  It only places groups (slice, first probe, tag,
// owner rank) -- keys are always compared exactly -- so it is the table's own function, not
// Spark's: three 64-bit multiplies (each key word once, then one finalising multiply) instead
// of XXH64's eight, since the stage, the level-2 split and the slice aggregation each hash every
// record.  Its bins measured Poisson-spread (std/sqrt(mean) 0.97-1.0) over the slice, slot and
// region bits for C4's 12-digit keys, sequential decimal strings and small / shifted integers.
// (The length goes into k1's top byte, which an inline key of <= 15 bytes leaves zero.)
__device__ inline uint64_t hash_raw(uint64_t k0, uint64_t k1, uint32_t len) {
  const uint64_t a = (k0 + 0x165667B19E3779F9ull) * 0x9E3779B97F4A7C15ull;
  const uint64_t b = (k1 ^ ((uint64_t)len << 56) ^ 0x27D4EB2F165667C5ull) * 0xC2B2AE3D27D4EB4Full;
  uint64_t h = a ^ ((b << 32) | (b >> 32));
  h ^= h >> 29;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

// The table hash of a key that packs into one word (a digit string, or Histogram's NULL group;
// dq_keypack.h): two 64-bit multiplies of the packed word, each followed by a fold of the high
// half into the low one.  The partition path's level-2 split and its slice aggregation hash
// every record, so a packed record is hashed as it is (round 3 unpacked it and ran hash_raw:
// ~75 VALU instructions per record against ~13).  Bins measured Poisson-spread over the slice,
// probe, tag and owner bits for C4's 12-digit keys and sequential decimal strings.
__device__ inline uint64_t hash_record_packed(uint64_t p) {
  uint64_t x = p + 0x9E3779B97F4A7C15ull;
  x ^= x >> 32;
  x *= 0xD6E8FEB86659FD93ull;
  x ^= x >> 32;
  x *= 0xD6E8FEB86659FD93ull;
  return x ^ (x >> 32);
}

// The table hash of an inline key, wherever a key is hashed (stage, splits, aggregations,
// inserts, imports, lookups, rehash, owner ranks): a key that packs is hashed as its packed
// word, so a digit key hashes alike whether it travels as a packed or a 16-byte record.
__device__ inline uint64_t hash_inline(uint64_t k0, uint64_t k1, uint32_t len) {
  uint64_t p;
  if (kp_pack_record(k0, k1, len, &p)) return hash_record_packed(p);
  return hash_raw(k0, k1, len);
}

// The table hash of a canonical UUID key (dq_uuidpack.h) from its packed words: the partition
// path stages, splits and aggregates such keys as {lo, hi} and hashes each record in every pass,
// so -- as a digit key is hashed as its packed word -- a UUID is hashed as its words (three
// multiplies) rather than as 36 bytes of XXH64 (~25).
__device__ inline uint64_t hash_uuid(uint64_t lo, uint64_t hi) { return hash_raw(lo, hi, kUuidLen); }

// The table hash of a key of more than 16 bytes, wherever one is hashed (make_key, lookups,
// imports, rehash, inserts from the heap): a canonical UUID hashes as its packed words, any other
// key by xxh64_any.  A function of the key bytes alone, so every path agrees.
__device__ inline uint64_t hash_long(const uint8_t* p, uint32_t len) {
  if (len == kUuidLen) {
    uint32_t w[9];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t v = ld_partial(p + 8 * i, 8);
      w[2 * i] = (uint32_t)v;
      w[2 * i + 1] = (uint32_t)(v >> 32);
    }
    w[8] = (uint32_t)ld_partial(p + 32, 4);
    uint64_t lo, hi;
    if (uuid_pack(w, &lo, &hi)) return hash_uuid(lo, hi);
  }
  return xxh64_any(p, len, 42);
}

// One row's grouping key.  Inline (len <= 16) keys live in k0/k1; longer keys point at their
// bytes (`ptr`, in the batch or in thread-local scratch).
struct Key {
  uint64_t k0, k1;
  const uint8_t* ptr;
  uint32_t len;
  uint64_t hash;
};

__device__ inline bool col_valid(const DevColumn& c, int64_t row) {
  return c.validity == nullptr || ((c.validity[row >> 3] >> (row & 7)) & 1u);
}

__device__ inline int width_of(int t) {
  switch (t) {
    case DQ_T_BOOL: case DQ_T_INT8: return 1;
    case DQ_T_INT16: return 2;
    case DQ_T_INT32: case DQ_T_FLOAT32: return 4;
    default: return 8;
  }
}

__device__ inline uint64_t fixed_bits(const DevColumn& c, int64_t row) {
  switch (c.type) {
    case DQ_T_BOOL: return (static_cast<const uint8_t*>(c.values)[row >> 3] >> (row & 7)) & 1u;
    case DQ_T_INT8: return static_cast<const uint8_t*>(c.values)[row];
    case DQ_T_INT16: return static_cast<const uint16_t*>(c.values)[row];
    case DQ_T_INT32: case DQ_T_FLOAT32: return static_cast<const uint32_t*>(c.values)[row];
    default: return static_cast<const uint64_t*>(c.values)[row];
  }
}

// Builds the key of `row`; false if the row is excluded (a NULL grouping value and NULLs are
// not a key).  Encodings: fixed-width columns = little-endian value bits (floats as raw bits,
// Spark 2.2 groups by UnsafeRow bytes); strings = UTF-8 bytes, prefixed by a u32 length when
// several columns are combined; Histogram NULLs = "NullValue" for strings (merging with a
// literal "NullValue", Histogram.scala:63-64) and the empty key for other types.
// want_hash = false: an inline key (len <= 16, k.ptr == nullptr) is returned without its table
// hash (k.hash = 0) -- the LDS pre-aggregation only needs a cheap one (lds_hash below), and
// most rows of a low-cardinality column never reach the global table.
__device__ bool make_key(const FreqKeySpec& ks, const DevColumn* cols, int64_t row, Key& k,
                         uint8_t* scratch, bool& too_long, bool want_hash = true) {
  k.k0 = k.k1 = 0;
  k.ptr = nullptr;
  k.len = 0;
  too_long = false;
  if (ks.n_keys == 1) {
    const DevColumn& c = cols[ks.key_cols[0]];
    const bool valid = col_valid(c, row);
    if (!valid && !ks.null_as_key) return false;
    if (c.type == DQ_T_UTF8) {
      const uint8_t* p;
      uint32_t n;
      if (!valid) {
        p = reinterpret_cast<const uint8_t*>("NullValue");
        n = 9;
      } else {
        const int32_t b = c.offsets[row], e = c.offsets[row + 1];
        p = static_cast<const uint8_t*>(c.values) + b;
        n = (uint32_t)(e - b);
      }
      k.len = n;
      if (n <= 16) {
        k.k0 = ld_partial(p, n < 8 ? n : 8);
        k.k1 = n > 8 ? ld_partial(p + 8, n - 8) : 0;
        k.hash = want_hash ? hash_inline(k.k0, k.k1, n) : 0;
      } else {
        k.ptr = p;
        k.hash = hash_long(p, n);
      }
      return true;
    }
    if (!valid) {  // Histogram NULL of a non-string column: the empty key
      k.hash = want_hash ? hash_inline(0, 0, 0) : 0;
      return true;
    }
    k.k0 = fixed_bits(c, row);
    if (ks.null_as_key) {  // Histogram groups cast-to-string values: every NaN is "NaN"
      if (c.type == DQ_T_FLOAT64 && (k.k0 & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) k.k0 = 0x7ff8000000000000ull;
      if (c.type == DQ_T_FLOAT32 && (k.k0 & 0x7fffffffull) > 0x7f800000ull) k.k0 = 0x7fc00000ull;
    }
    k.len = (uint32_t)width_of(c.type);
    k.hash = want_hash ? hash_inline(k.k0, 0, k.len) : 0;
    return true;
  }
  // several columns: concatenate into scratch
  uint32_t n = 0;
  for (int i = 0; i < ks.n_keys; ++i) {
    const DevColumn& c = cols[ks.key_cols[i]];
    if (!col_valid(c, row)) return false;
    if (c.type == DQ_T_UTF8) {
      const int32_t b = c.offsets[row], e = c.offsets[row + 1];
      const uint32_t sl = (uint32_t)(e - b);
      if (n + 4 + sl > (uint32_t)kMaxLocalKey) {
        too_long = true;
        return false;
      }
      for (int j = 0; j < 4; ++j) scratch[n + j] = (uint8_t)(sl >> (8 * j));
      n += 4;
      const uint8_t* p = static_cast<const uint8_t*>(c.values) + b;
      for (uint32_t j = 0; j < sl; ++j) scratch[n + j] = p[j];
      n += sl;
    } else {
      const int w = width_of(c.type);
      const uint64_t bits = fixed_bits(c, row);
      for (int j = 0; j < w; ++j) scratch[n + j] = (uint8_t)(bits >> (8 * j));
      n += (uint32_t)w;
    }
  }
  k.len = n;
  if (n <= 16) {
    for (uint32_t j = 0; j < n && j < 8; ++j) k.k0 |= (uint64_t)scratch[j] << (8 * j);
    for (uint32_t j = 8; j < n; ++j) k.k1 |= (uint64_t)scratch[j] << (8 * (j - 8));
    k.hash = hash_inline(k.k0, k.k1, n);
  } else {
    k.ptr = scratch;
    k.hash = hash_long(scratch, n);
  }
  return true;
}

// Keys of G rows (row_j = base + j * stride, j < G) of ONE utf8 key column, with the loads of
// all G rows issued together: the validity bits and offsets first, then the (at most 3) aligned
// words of each key of <= 15 bytes.  Per row: sel = in range and a key (a NULL is a key only for
// Histogram: "NullValue"); lng = a selected key longer than 15 bytes (the caller builds it with
// make_key).  Words past a key are never loaded (they could lie past the buffer).
template <int G>
__device__ inline void string_keys(const DevColumn& c0, bool null_as_key, int64_t base, int64_t stride,
                                   int64_t end, uint64_t (&k0)[G], uint64_t (&k1)[G], uint32_t (&len)[G],
                                   uint32_t& sel, uint32_t& lng) {
  const uint8_t* bytes = static_cast<const uint8_t*>(c0.values);
  int32_t ob[G], oe[G];
  uint32_t valid = 0u, inr = 0u;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int64_t row = base + j * stride;
    ob[j] = oe[j] = 0;
    if (row < end) {
      inr |= 1u << j;
      ob[j] = c0.offsets[row];
      oe[j] = c0.offsets[row + 1];
      if (col_valid(c0, row)) valid |= 1u << j;
    }
  }
  uint64_t w0[G], w1[G], w2[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const uint32_t n = (uint32_t)(oe[j] - ob[j]);
    const uintptr_t a = (uintptr_t)(bytes + ob[j]);
    const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
    const uint32_t span = (uint32_t)(a & 7) + n;  // bytes from the first word's start
    w0[j] = w1[j] = w2[j] = 0;
    if (((valid >> j) & 1u) && n > 0 && n <= 15) {
      w0[j] = w[0];
      if (span > 8) w1[j] = w[1];
      if (span > 16) w2[j] = w[2];
    }
  }
  sel = 0u;
  lng = 0u;
#pragma unroll
  for (int j = 0; j < G; ++j) {
    k0[j] = k1[j] = 0ull;
    len[j] = 0u;
    if (!((inr >> j) & 1u)) continue;
    if ((valid >> j) & 1u) {
      const uint32_t n = (uint32_t)(oe[j] - ob[j]);
      sel |= 1u << j;
      len[j] = n;
      if (n > 15) {
        lng |= 1u << j;
        continue;
      }
      const uint32_t sh = (uint32_t)((uintptr_t)(bytes + ob[j]) & 7) * 8u;
      // bytes 0..7 and 8..15 of the key from the three words, then masked to n bytes
      const uint64_t lo = sh ? (w0[j] >> sh) | (w1[j] << (64u - sh)) : w0[j];
      const uint64_t hi = sh ? (w1[j] >> sh) | (w2[j] << (64u - sh)) : w1[j];
      k0[j] = n >= 8 ? lo : (n ? lo & ((1ull << (8u * n)) - 1ull) : 0ull);
      k1[j] = n > 8 ? hi & ((1ull << (8u * (n - 8u))) - 1ull) : 0ull;
    } else if (null_as_key) {  // Histogram NULL: "NullValue"
      sel |= 1u << j;
      len[j] = 9;
      k0[j] = 0x756c61566c6c754eull;  // "NullValu"
      k1[j] = 0x65ull;                // "e"
    }
  }
}

// Hash bit use: the top bucket_bits select the slice, the low kFreqSliceLog bits the first
// probe, bits 12..43 the 32-bit tag kept in ctrl (independent of both).
__device__ inline uint32_t tag_of(uint64_t h) {
  const uint32_t t = (uint32_t)(h >> 12);
  return t ? t : 1u;
}

__device__ inline uint64_t slice_of(const FreqTable& T, uint64_t h) {
  return T.bucket_bits ? (h >> (64 - T.bucket_bits)) : 0ull;
}

__device__ inline uint64_t probe_slot(const FreqTable& T, uint64_t h, uint64_t i) {
  return (slice_of(T, h) << kFreqSliceLog) | ((h + i) & (kFreqSliceSlots - 1));
}

// Compare a long key with heap bytes (heap words written by atomic exchange: read coherently).
__device__ bool heap_equal(const FreqTable& T, uint64_t off, const uint8_t* p, uint32_t len) {
  unsigned long long* hw = reinterpret_cast<unsigned long long*>(T.heap) + (off >> 3);
  for (uint32_t i = 0; i < len; i += 8) {
    const uint32_t n = len - i < 8 ? len - i : 8;
    if (atom_read(hw + (i >> 3)) != ld_partial(p + i, n)) return false;
  }
  return true;
}

// Insert `cnt` rows of key k into the global table.  Returns false on table/heap overflow.
// kFlagOverflow = false: a full slice is reported only by the return value (the sorted path
// hands such rows back for a retry after the table grows).
// kKeyInHeap: a long key's bytes already lie in T's heap at k.ptr (the hashed path's stage put
// them there): a claimed slot refers to them instead of copying them again.
template <bool kFlagOverflow = true, bool kKeyInHeap = false>
__device__ bool global_insert(const FreqTable& T, const Key& k, unsigned long long cnt) {
  // Every action happens inside the loop iteration and the loop ends only through `state`: a
  // lane that waits for another lane of its own wave to publish a slot must see that publish in
  // its next iteration.  (With the publish on an exit path -- `return` right after it -- the
  // compiler may move it behind the loop, after the lanes that wait for it.)
  const uint32_t tag = tag_of(k.hash);
  const bool inl = k.len <= 16;
  const unsigned long long want = ((unsigned long long)tag << 32) | (inl ? 0ull : kHeapKey) | k.len;
  uint64_t probes = 0;
  uint64_t slot = probe_slot(T, k.hash, 0);
  uint32_t waits = 0;
  int state = 0;  // 0 = probing, 1 = counted, 2 = no room in the slice, 3 = key heap full, 4 = wait timeout
  while (state == 0) {
    FreqSlot* e = &T.slots[slot];
    const unsigned long long c = atomicCAS(&e->ctrl, 0ull, want);
    bool next = false;
    if (c == 0ull) {  // claimed: publish key, count, then READY
      bool heap_ok = true;
      if (inl) {
        atomicExch(&e->k0, (unsigned long long)k.k0);
        atomicExch(&e->k1, (unsigned long long)k.k1);
      } else if (kKeyInHeap) {
        atomicExch(&e->k0, (unsigned long long)(k.ptr - T.heap));
      } else {
        const unsigned long long bytes = ((unsigned long long)k.len + 7ull) & ~7ull;
        const unsigned long long off = atomicAdd(T.heap_used, bytes);
        if (off + bytes > T.heap_cap) {  // publish anyway so that no reader waits on the slot
          atomicOr(T.overflow, 2u);
          atomicExch(&e->k0, ~0ull);
          heap_ok = false;
        } else {
          unsigned long long* hw = reinterpret_cast<unsigned long long*>(T.heap) + (off >> 3);
          for (uint32_t i = 0; i < k.len; i += 8) {
            const uint32_t n = k.len - i < 8 ? k.len - i : 8;
            atomicExch(hw + (i >> 3), (unsigned long long)ld_partial(k.ptr + i, n));
          }
          atomicExch(&e->k0, off);
        }
      }
      atomicAdd(&e->count, cnt);
      if (heap_ok) atomicAdd(T.n_groups, 1ull);
      if (!(T.test_flags & kFreqTestNoPublish))
        __hip_atomic_fetch_or(&e->ctrl, kReady, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      state = heap_ok ? 1 : 3;  // (3: heap full, flagged above with bit 2 only)
    } else if ((uint32_t)(c >> 32) == tag && (c & (kLenMask | kHeapKey)) == (want & (kLenMask | kHeapKey))) {
      if (!(c & kReady)) {  // being published by another lane/wave: look at this slot again
        // (a wait that never ends is a failure -- its own overflow bit, reported as an error by
        // every caller -- never a full slice that would send the rows to a retry)
        if (++waits > (1u << 22)) state = 4;
        else __builtin_amdgcn_s_sleep(1);
      } else {
        bool eq;
        if (inl) {
          eq = atom_read(&e->k0) == k.k0 && atom_read(&e->k1) == k.k1;
        } else {
          const unsigned long long off = atom_read(&e->k0);
          eq = off + k.len <= T.heap_cap && heap_equal(T, off, k.ptr, k.len);
        }
        if (eq) {
          atomicAdd(&e->count, cnt);
          state = 1;
        } else {
          next = true;
        }
      }
    } else {
      next = true;
    }
    if (next) {
      if (++probes < kFreqSliceSlots) slot = probe_slot(T, k.hash, probes);
      else state = 2;
    }
  }
  if (state == 2 && kFlagOverflow) atomicOr(T.overflow, 1u);
  if (state == 4) atomicOr(T.overflow, kFreqWaitTimeout);
  return state == 1;
}

// Slot and tag of an inline key in a workgroup's LDS table: a 32-bit mix (two 32-bit multiplies
// instead of XXH64's six 64-bit ones); keys are compared exactly, so any spread will do.
__device__ inline uint32_t lds_hash(uint64_t k0, uint64_t k1, uint32_t len) {
  uint32_t a = ((uint32_t)k0 ^ (uint32_t)(k1 >> 32)) * 0x9E3779B1u;
  uint32_t b = ((uint32_t)(k0 >> 32) ^ (uint32_t)k1 ^ (len << 24)) * 0x85EBCA77u;
  uint32_t h = a ^ __builtin_amdgcn_alignbit(b, b, 13);
  h ^= h >> 15;
  h *= 0xC2B2AE3Du;
  return h ^ (h >> 13);
}

// Structure of arrays: a wave's 64 random slots spread over all 64 LDS banks (32-byte slot
// records put every slot of a wave on 8 of them).
struct LdsTable {
  unsigned long long ctrl[kLdsSlots];  // as the global ctrl (READY unused: LDS keys are written before ctrl)
  unsigned long long k0[kLdsSlots], k1[kLdsSlots];
  unsigned int count[kLdsSlots];
};
#define DQ_LDS(f, i) lds.f[i]

}  // namespace

// Group-by of one batch: LDS pre-aggregation per workgroup, overflow rows to the global table.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void dq_freq_insert_kernel(FreqKeySpec ks,
                                                                const DevColumn* __restrict__ cols,
                                                                int64_t n_rows, FreqTable T) {
  __shared__ LdsTable lds;
  __shared__ int lds_open;
  for (int i = threadIdx.x; i < kLdsSlots; i += kBlock) {
    DQ_LDS(ctrl, i) = 0;
    DQ_LDS(count, i) = 0;
  }
  if (threadIdx.x == 0) lds_open = 1;
  __syncthreads();

  const int64_t per_block = (n_rows + gridDim.x - 1) / gridDim.x;
  const int64_t row_begin = (int64_t)blockIdx.x * per_block;
  const int64_t row_end = row_begin + per_block < n_rows ? row_begin + per_block : n_rows;
  alignas(8) uint8_t scratch[kMaxLocalKey];
  unsigned long long lds_misses = 0;
  // One row through the LDS table (claiming, probing) and, failing that, the global table.
  // Returns false on a global table overflow.
  auto insert_row = [&](Key& k) -> bool {
    const bool lazy = k.ptr == nullptr && k.len <= 16;  // inline key: k.hash not computed yet
    bool done = false;
    if (lazy && lds_open) {
      // LDS table: claim by CAS on ctrl after the key words are known; a racing claimer of the
      // same slot either wins (and writes the same-or-other key) or re-probes.  LDS slots publish
      // k0/k1 under a per-slot two-phase (ctrl = BUSY, then ctrl = want) and readers re-probe
      // the slot while BUSY.
      const uint32_t lh = lds_hash(k.k0, k.k1, k.len);
      const unsigned long long want = ((unsigned long long)lh << 32) | kReady | k.len;
      uint32_t s = lh & (kLdsSlots - 1);
      for (int probe = 0; probe < kLdsProbe * 4 && !done; ) {
        unsigned long long c = __hip_atomic_load(&DQ_LDS(ctrl, s), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c == 0ull) c = atomicCAS(&DQ_LDS(ctrl, s), 0ull, 1ull);  // 1 = BUSY
        if (c == 0ull) {
          DQ_LDS(k0, s) = k.k0;
          DQ_LDS(k1, s) = k.k1;
          atomicAdd(&DQ_LDS(count, s), 1u);
          __threadfence_block();
          atomicExch(&DQ_LDS(ctrl, s), want);
          done = true;
        } else if (c == 1ull) {
          ++probe;  // another lane is publishing this slot: look again
        } else if (c == want && __hip_atomic_load(&DQ_LDS(k0, s), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == k.k0 &&
                   __hip_atomic_load(&DQ_LDS(k1, s), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == k.k1) {
          atomicAdd(&DQ_LDS(count, s), 1u);
          done = true;
        } else {
          s = (s + 1) & (kLdsSlots - 1);
          probe += 4;
        }
      }
      if (!done && ++lds_misses > 32) lds_open = 0;  // LDS is full of other keys: stop probing it
    }
    if (!done) {
      if (lazy) k.hash = hash_inline(k.k0, k.k1, k.len);
      if (!global_insert(T, k, 1ull)) return false;
    }
    return true;
  };
  if (ks.n_keys == 1) {
    // Single-column keys (no scratch): R rows per lane per step, the common case -- the key is
    // already in its home slot -- as independent loads (R slot words read together, ONE acquire
    // fence, R key compares, R counter adds), so the LDS round trips overlap instead of chaining
    // row after row.  Anything else (empty or busy slot, collision) takes insert_row.
    constexpr int R = DQ_INSERT_R;
    bool overflowed = false;
    const bool one_string = cols[ks.key_cols[0]].type == DQ_T_UTF8;
    for (int64_t base = row_begin; base < row_end && !overflowed; base += (int64_t)kBlock * R) {
      Key k[R];
      bool ok[R];
      uint32_t slot[R];
      unsigned long long want[R], c[R];
      uint32_t s_sel = 0u, s_lng = 0u;
      uint64_t sk0[R], sk1[R];
      uint32_t slen[R];
      if (one_string)  // all R rows' offsets, then all their key words, in flight together
        string_keys<R>(cols[ks.key_cols[0]], ks.null_as_key != 0, base + threadIdx.x, kBlock, row_end, sk0, sk1,
                       slen, s_sel, s_lng);
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int64_t row = base + (int64_t)j * kBlock + threadIdx.x;
        bool too_long = false;
        if (one_string && !((s_lng >> j) & 1u)) {
          ok[j] = (s_sel >> j) & 1u;
          k[j].k0 = sk0[j];
          k[j].k1 = sk1[j];
          k[j].len = slen[j];
          k[j].ptr = nullptr;
          k[j].hash = 0;
        } else {
          ok[j] = row < row_end && make_key(ks, cols, row, k[j], scratch, too_long, false);
        }
        if (!ok[j] && too_long) atomicOr(T.overflow, 4u);
        const bool fast = ok[j] && k[j].ptr == nullptr && k[j].len <= 16 && lds_open;
        const uint32_t lh = fast ? lds_hash(k[j].k0, k[j].k1, k[j].len) : 0u;
        want[j] = fast ? (((unsigned long long)lh << 32) | kReady | k[j].len) : 0ull;
        slot[j] = lh & (kLdsSlots - 1);
      }
#pragma unroll
      for (int j = 0; j < R; ++j)
        c[j] = want[j] ? __hip_atomic_load(&DQ_LDS(ctrl, slot[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0ull;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the keys published before those ctrl words
#pragma unroll
      for (int j = 0; j < R; ++j) {
        bool hit = false;
        if (want[j] && c[j] == want[j])
          hit = __hip_atomic_load(&DQ_LDS(k0, slot[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == k[j].k0 &&
                __hip_atomic_load(&DQ_LDS(k1, slot[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == k[j].k1;
        if (hit) atomicAdd(&DQ_LDS(count, slot[j]), 1u);
        else if (ok[j] && !insert_row(k[j])) overflowed = true;
      }
    }
  } else {
    for (int64_t row = row_begin + threadIdx.x; row < row_end; row += kBlock) {
      Key k;
      bool too_long;
      if (!make_key(ks, cols, row, k, scratch, too_long, false)) {
        if (too_long) atomicOr(T.overflow, 4u);
        continue;
      }
      if (!insert_row(k)) break;
    }
  }
  __syncthreads();
  // flush the LDS groups
  for (int i = threadIdx.x; i < kLdsSlots; i += kBlock) {
    const unsigned long long c = DQ_LDS(ctrl, i);
    if (c > 1ull && DQ_LDS(count, i)) {
      Key k;
      k.k0 = DQ_LDS(k0, i);
      k.k1 = DQ_LDS(k1, i);
      k.len = (uint32_t)(c & kLenMask);
      k.ptr = nullptr;
      k.hash = hash_inline(k.k0, k.k1, k.len);
      global_insert(T, k, DQ_LDS(count, i));
    }
  }
}

// Count-of-counts over the table: hist[c] for c < kFreqHist, larger counts appended to a list.
__global__ __launch_bounds__(kBlock) void dq_freq_hist_kernel(FreqTable T, unsigned long long* hist,
                                                              unsigned long long* big,
                                                              unsigned long long* n_big,
                                                              unsigned long long big_cap) {
  __shared__ unsigned int lh[kFreqLdsHist];
  for (int i = threadIdx.x; i < kFreqLdsHist; i += kBlock) lh[i] = 0;
  __syncthreads();
  const uint64_t n = T.mask + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (uint64_t)gridDim.x * kBlock) {
    const FreqSlot& e = T.slots[s];
    if (e.ctrl & kReady) {
      const unsigned long long c = e.count;  // launch boundary: all inserts are visible
      if (c < (unsigned long long)kFreqLdsHist) {
        atomicAdd(&lh[c], 1u);
      } else if (c < (unsigned long long)kFreqHist) {
        atomicAdd(&hist[c], 1ull);
      } else {
        const unsigned long long i = atomicAdd(n_big, 1ull);
        if (i < big_cap) big[i] = c;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kFreqLdsHist; i += kBlock)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

// Export groups: slots with count >= min_count (and, for count == tie_count, all of them).
// smax (optional): the largest count of each slice; slices below min_count are not read.
__global__ __launch_bounds__(kBlock) void dq_freq_export_slices_kernel(FreqTable T, unsigned long long min_count,
                                                                       const uint32_t* __restrict__ smax, FreqOut out) {
  const uint64_t n_slices = (T.mask + 1) >> kFreqSliceLog;
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    if ((unsigned long long)smax[b] < min_count) continue;
    const FreqSlot* slice = T.slots + (b << kFreqSliceLog);
    for (uint32_t s = threadIdx.x; s < (uint32_t)kFreqSliceSlots; s += kBlock) {
      const FreqSlot& e = slice[s];
      if ((e.ctrl & kReady) && e.count >= min_count) {
        const unsigned long long i = atomicAdd(out.n, 1ull);
        if (i < out.cap) {
          out.ctrl[i] = e.ctrl;
          out.count[i] = e.count;
          out.k0[i] = e.k0;
          out.k1[i] = e.k1;
        }
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void dq_freq_export_kernel(FreqTable T, unsigned long long min_count,
                                                                FreqOut out) {
  const uint64_t n = T.mask + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < n; s += (uint64_t)gridDim.x * kBlock) {
    const FreqSlot& e = T.slots[s];
    if ((e.ctrl & kReady) && e.count >= min_count) {
      const unsigned long long i = atomicAdd(out.n, 1ull);
      if (i < out.cap) {
        out.ctrl[i] = e.ctrl;
        out.count[i] = e.count;
        out.k0[i] = e.k0;
        out.k1[i] = e.k1;
      }
    }
  }
}

// Insert exported groups (another table, a loaded state, another GPU's partition).
__global__ __launch_bounds__(kBlock) void dq_freq_import_kernel(FreqTable T, FreqIn in) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < in.n; i += (uint64_t)gridDim.x * kBlock) {
    Key k;
    const uint64_t j = i * in.stride;
    k.len = (uint32_t)(in.ctrl[j] & kLenMask);
    if (in.ctrl[j] & kHeapKey) {
      k.ptr = in.heap + in.k0[j];
      k.k0 = k.k1 = 0;
      k.hash = hash_long(k.ptr, k.len);
    } else {
      k.ptr = nullptr;
      k.k0 = in.k0[j];
      k.k1 = in.k1[j];
      k.hash = hash_inline(k.k0, k.k1, k.len);
    }
    if (!global_insert(T, k, in.count[j])) return;
  }
}

// ---- Flat (columnar) export and import: dq_freq_export_flat / dq_freq_import_flat.
// The export lists every group in SLOT order (deterministic: the same table exports the same
// columns), as the Arrow layout of the state's DataFrame wants it: counts[i], and key i's bytes
// at [offs[i], offs[i + 1]) of one byte array.  No per-group record on the host.
constexpr uint32_t kFlatRounds = 16;
constexpr uint32_t kFlatChunk = (uint32_t)kBlock * kFlatRounds;  // slots per workgroup

// chunk_n[b] = the groups among slots [b kFlatChunk, (b + 1) kFlatChunk); chunk_n[n_chunks] = 0
// (the exclusive scan's total lands there).
__global__ __launch_bounds__(kBlock) void dq_flat_count_kernel(FreqTable T, unsigned long long* chunk_n,
                                                               uint64_t n_chunks) {
  __shared__ uint32_t ws[kBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kFlatChunk;
  uint32_t c = 0;
#pragma unroll 4
  for (uint32_t r = 0; r < kFlatRounds; ++r) {
    const uint64_t s = base + (uint64_t)r * kBlock + threadIdx.x;
    if (s <= T.mask && (T.slots[s].ctrl & kReady)) ++c;
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += ws[w];
    chunk_n[blockIdx.x] = s;
    if (blockIdx.x == 0) chunk_n[n_chunks] = 0ull;
  }
}

// Each workgroup writes its chunk's groups from position chunk_base[b], in slot order: per round
// of kBlock slots a ballot gives each ready slot its rank within the wave, LDS the waves' offsets.
// lens[i] = key length (the exclusive scan turns it into the byte offsets); lens[n] = 0.
__global__ __launch_bounds__(kBlock) void dq_flat_fill_kernel(FreqTable T, const unsigned long long* __restrict__ chunk_base,
                                                              uint64_t n, unsigned long long* __restrict__ ctrl,
                                                              unsigned long long* __restrict__ count,
                                                              unsigned long long* __restrict__ k0,
                                                              unsigned long long* __restrict__ k1,
                                                              unsigned long long* __restrict__ lens) {
  __shared__ uint32_t ws[kBlock / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kFlatChunk;
  uint64_t pos = chunk_base[blockIdx.x];
  if (blockIdx.x == 0 && threadIdx.x == 0) lens[n] = 0ull;
  for (uint32_t r = 0; r < kFlatRounds; ++r) {
    const uint64_t s = base + (uint64_t)r * kBlock + threadIdx.x;
    FreqSlot e;
    bool ready = false;
    if (s <= T.mask) {
      e = T.slots[s];
      ready = (e.ctrl & kReady) != 0;
    }
    const uint64_t b = __ballot(ready);
    const uint32_t below = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) ws[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (uint32_t w = 0; w < (uint32_t)(kBlock / 64); ++w) {
      off += w < wave ? ws[w] : 0u;
      tot += ws[w];
    }
    if (ready) {
      const uint64_t i = pos + off + below;
      if (i < n) {
        ctrl[i] = e.ctrl;
        count[i] = e.count;
        k0[i] = e.k0;
        k1[i] = e.k1;
        lens[i] = e.ctrl & kLenMask;
      }
    }
    pos += tot;
    __syncthreads();  // (ws is rewritten by the next round)
  }
}

// Key bytes of group i at out[offs[i] ..]: inline keys from k0 / k1, long keys from the heap.
__global__ __launch_bounds__(kBlock) void dq_flat_keys_kernel(FreqTable T, const unsigned long long* __restrict__ ctrl,
                                                              const unsigned long long* __restrict__ k0,
                                                              const unsigned long long* __restrict__ k1,
                                                              const unsigned long long* __restrict__ offs, uint64_t n,
                                                              uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const unsigned long long c = ctrl[i];
    const uint32_t len = (uint32_t)(c & kLenMask);
    uint8_t* dst = out + offs[i];
    if (c & kHeapKey) {
      const uint8_t* src = T.heap + k0[i];
      for (uint32_t j = 0; j < len; ++j) dst[j] = src[j];
    } else {
      const uint64_t a = k0[i], b = k1[i];
      for (uint32_t j = 0; j < len; ++j) dst[j] = (uint8_t)((j < 8 ? a >> (8 * j) : b >> (8 * (j - 8))) & 0xFFu);
    }
  }
}

// Insert flat groups (a loaded state): group i = (counts[i], bytes[offs[i] .. offs[i + 1])).
__global__ __launch_bounds__(kBlock) void dq_freq_import_flat_kernel(FreqTable T, const long long* __restrict__ counts,
                                                                     const long long* __restrict__ offs,
                                                                     const uint8_t* __restrict__ bytes, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint64_t o = (uint64_t)offs[i];
    Key k;
    k.len = (uint32_t)((uint64_t)offs[i + 1] - o);
    if (k.len > 16u) {
      k.ptr = bytes + o;
      k.k0 = k.k1 = 0;
      k.hash = hash_long(k.ptr, k.len);
    } else {
      k.ptr = nullptr;
      k.k0 = ld_partial(bytes + o, k.len < 8u ? k.len : 8u);
      k.k1 = k.len > 8u ? ld_partial(bytes + o + 8, k.len - 8u) : 0ull;
      k.hash = hash_inline(k.k0, k.k1, k.len);
    }
    if (!global_insert(T, k, (unsigned long long)counts[i])) return;
  }
}

// Count of one encoded key (0 if absent): a single-thread probe of the key's slice.
// cmp.slots != nullptr: a compacted table -- the key's slice's groups are scanned (by the wave's
// 64 lanes) instead of probed.
__global__ void dq_freq_lookup_kernel(FreqTable T, const uint8_t* key, uint32_t len, unsigned long long* out,
                                      FreqCompact cmp) {
  if (blockIdx.x != 0) return;
  if (cmp.slots) {
    Key k;
    k.len = len;
    k.k0 = len <= 16 ? ld_partial(key, len < 8 ? len : 8) : 0ull;
    k.k1 = len > 8 && len <= 16 ? ld_partial(key + 8, len - 8) : 0ull;
    k.hash = len <= 16 ? hash_inline(k.k0, k.k1, len) : hash_long(key, len);
    const uint32_t tag = tag_of(k.hash);
    const uint64_t b = slice_of(T, k.hash);
    const FreqSlot* g = cmp.slots + cmp.base[b];
    const uint32_t n = cmp.num[b];
    if (threadIdx.x == 0) *out = 0ull;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const FreqSlot e = g[i];
      if ((uint32_t)(e.ctrl >> 32) != tag || (uint32_t)(e.ctrl & kLenMask) != len) continue;
      bool eq;
      if (len <= 16 && !(e.ctrl & kHeapKey)) {
        eq = e.k0 == k.k0 && e.k1 == k.k1;
      } else {
        eq = (e.ctrl & kHeapKey) != 0;
        for (uint32_t j = 0; eq && j < len; ++j) eq = T.heap[e.k0 + j] == key[j];
      }
      if (eq) *out = e.count;  // (one group holds the key)
    }
    return;
  }
  if (threadIdx.x != 0) return;
  Key k;
  k.len = len;
  k.k0 = k.k1 = 0;
  k.ptr = nullptr;
  if (len <= 16) {
    k.k0 = ld_partial(key, len < 8 ? len : 8);
    k.k1 = len > 8 ? ld_partial(key + 8, len - 8) : 0;
    k.hash = hash_inline(k.k0, k.k1, len);
  } else {
    k.ptr = key;
    k.hash = hash_long(key, len);
  }
  const uint32_t tag = tag_of(k.hash);
  *out = 0ull;
  for (uint64_t i = 0; i < kFreqSliceSlots; ++i) {
    const FreqSlot& e = T.slots[probe_slot(T, k.hash, i)];
    if (e.ctrl == 0ull) return;  // launch boundary: the table is complete and visible
    if ((uint32_t)(e.ctrl >> 32) != tag || (uint32_t)(e.ctrl & kLenMask) != len) continue;
    if (len <= 16 && !(e.ctrl & kHeapKey)) {
      if (e.k0 != k.k0 || e.k1 != k.k1) continue;
    } else {
      bool eq = (e.ctrl & kHeapKey) != 0;
      for (uint32_t j = 0; eq && j < len; ++j) eq = T.heap[e.k0 + j] == key[j];
      if (!eq) continue;
    }
    *out = e.count;
    return;
  }
}

// ---- multi-GPU key-hash partitioning (owner = a function of hash bits the table does not use
// for its slot index, so every owner's keys still spread over its whole table): bits 11..30,
// above the first probe (bits 0..10) and below any slice index (the top <= 22 bits); they
// overlap only the 32-bit tag, which then loses log2(n_parts) bits of its spread per owner.
__device__ inline uint32_t freq_owner(uint64_t h, uint32_t n_parts) {
  return (uint32_t)((((h >> 11) & 0xFFFFFull) * n_parts) >> 20);
}

__device__ inline uint64_t slot_hash(const FreqTable& T, const FreqSlot& e, uint32_t len) {
  return (e.ctrl & kHeapKey) ? hash_long(T.heap + e.k0, len) : hash_inline(e.k0, e.k1, len);
}

// ---- sorted-bucket path ---------------------------------------------------------------------
// High-cardinality group-by without a device-scope atomic per row:
//  1. stage (one streaming pass): every selected row becomes a 16-B record and feeds an HLL
//     sketch of the hashes that sizes the table.  A workgroup owns a contiguous row range and
//     reserves its output with ONE atomic (its rows are counted from the validity bitmaps
//     first), so no address takes an atomic per wave;
//  2. bucket split: the records grouped by slice (the top log2(#slices) hash bits) with exact
//     counts, two LDS multi-split levels (dq_freq_split_kernel below);
//  3. agg: one work item per slice's bucket.  A bucket of at most kFreqAggPiece records is one work
//     item: its slice is loaded into LDS, the records are counted there and the slice is written
//     back with plain stores (the workgroup owns it).  A larger bucket (a hot key, or Histogram's
//     NULL group) is cut into pieces of kFreqAggPiece records; each piece is pre-aggregated in LDS and
//     merged into the slice with device-scope atomics, so a skewed key spreads over many CUs
//     instead of serialising one workgroup.
// Keys of up to 15 bytes (the length lives in the top byte of the record's second word).
constexpr unsigned long long kRecLenShift = 56;
constexpr unsigned long long kRecKeyMask = (1ull << kRecLenShift) - 1;
constexpr uint32_t kRecHole = 0xFFu;  // length byte of a record that holds no row

// Staged records are written once and read once by the next pass (plain loads/stores: measured,
// non-temporal records cost C4 3-4 ms because the next pass re-reads them from L2 / MALL).
__device__ inline FreqRec ld_rec(const FreqRec* p) { return *p; }

__device__ inline void rec_unpack(const FreqRec& r, unsigned long long* k1, uint32_t* len) {
  *len = (uint32_t)(r.k1 >> kRecLenShift);
  *k1 = r.k1 & kRecKeyMask;
}

// HLL sketch of the staged hashes (p = 9): an estimate of the number of distinct keys, used
// only to size the table before aggregation.  (Sketching a 1/8 hash-based sample instead
// measured no faster on C4: 1.341 vs 1.341 ms per stage launch.)
__device__ inline void sketch_update(uint32_t* regs, uint64_t h) {
  uint32_t idx, pw;
  hll_idx_rank(h, &idx, &pw);
  if (pw > regs[idx]) atomicMax(&regs[idx], pw);
}

// The rows make_key accepts, from the validity bitmaps alone (the host routes a batch here only
// when every accepted key is at most 15 bytes long).
__device__ inline bool row_selected(const FreqKeySpec& ks, const DevColumn* cols, int64_t row) {
  if (ks.n_keys == 1) return ks.null_as_key || col_valid(cols[ks.key_cols[0]], row);
  for (int i = 0; i < ks.n_keys; ++i)
    if (!col_valid(cols[ks.key_cols[i]], row)) return false;
  return true;
}


// Each wave stages a contiguous run of the block's rows: a first pass counts the wave's selected
// rows (validity only), one atomicAdd per block reserves the block's records, and the second
// pass writes every selected row at its ballot prefix -- no block barrier inside either loop.
__global__ __launch_bounds__(kBlock) void dq_freq_stage_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                               int64_t n_rows, FreqRec* out,
                                                               unsigned long long* cursor, uint32_t* hll,
                                                               unsigned long long* long_key) {
  __shared__ uint32_t regs[kHllM];
  __shared__ uint32_t wcount[kBlock / 64];
  __shared__ unsigned long long base_s;
  for (int i = threadIdx.x; i < kHllM; i += kBlock) regs[i] = 0u;
  const int64_t per = (((n_rows + gridDim.x - 1) / gridDim.x) + kBlock - 1) & ~(int64_t)(kBlock - 1);
  const int64_t r0 = min((int64_t)blockIdx.x * per, n_rows);
  const int64_t r1 = min(r0 + per, n_rows);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const int64_t wper = per / (kBlock / 64);  // a multiple of 64
  const int64_t w0 = min(r0 + (int64_t)wave * wper, r1);
  const int64_t w1 = min(w0 + wper, r1);
  uint32_t cnt = 0;
  for (int64_t b = w0; b < w1; b += 64) {
    const int64_t row = b + lane;
    cnt += (uint32_t)__popcll(__ballot(row < w1 && row_selected(ks, cols, row)));
  }
  if (lane == 0) wcount[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t total = 0;
    for (int v = 0; v < kBlock / 64; ++v) total += wcount[v];
    base_s = total ? atomicAdd(cursor, (unsigned long long)total) : 0ull;
  }
  __syncthreads();
  unsigned long long w = base_s;
  for (uint32_t v = 0; v < wave; ++v) w += wcount[v];
  alignas(8) uint8_t scratch[kMaxLocalKey];
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (int64_t b = w0; b < w1; b += 64) {
    const int64_t row = b + lane;
    const bool sel = row < w1 && row_selected(ks, cols, row);
    const uint64_t m = __ballot(sel);
    if (sel) {
      const unsigned long long pos = w + (unsigned long long)__popcll(m & lt_mask);
      Key k;
      bool too_long;
      FreqRec r;
      if (make_key(ks, cols, row, k, scratch, too_long) && k.len <= 15 && k.ptr == nullptr) {
        r.k0 = k.k0;
        r.k1 = k.k1 | ((unsigned long long)k.len << kRecLenShift);
        sketch_update(regs, k.hash);
      } else {  // a key longer than 15 bytes: the host rolls this batch back to the general path
        r.k0 = 0;
        r.k1 = (unsigned long long)kRecHole << kRecLenShift;
        atomicMax(long_key, (unsigned long long)(k.len > 15 ? k.len : 16));
      }
      out[pos] = r;
    }
    w += (unsigned long long)__popcll(m);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHllM; i += kBlock)
    if (regs[i]) atomicMax(&hll[i], regs[i]);
}

// LDS slot words: K1 = EMPTY / BUSY (being published) / FOREIGN (a group this path cannot hold:
// a long or 16-byte key) / the record's k1 (length in the top byte); K0 = low key bytes;
// C = rows counted in this work item.
constexpr unsigned long long kLdsEmpty = ~0ull;
constexpr unsigned long long kLdsBusy = ~0ull - 1ull;
constexpr unsigned long long kLdsForeign = 0xFEull << kRecLenShift;

__device__ inline void emit_retry(FreqRec* retry, unsigned long long* n_retry, const FreqRec& r,
                                  unsigned long long copies) {
  const unsigned long long at = atomicAdd(n_retry, copies);
  for (unsigned long long j = 0; j < copies; ++j) retry[at + j] = r;
}

// The LDS image of one slice (dq_freq_agg_kernel, dq_freq_agg_region_kernel).
constexpr int kAggLdsHist = 512;  // count-of-counts bins kept in LDS by a tracking aggregation
struct AggLds {
  unsigned long long K0[kFreqSliceSlots], K1[kFreqSliceSlots];
  uint32_t C[kFreqSliceSlots];
  uint32_t G[kFreqSliceSlots];  // the table tag of a slot claimed in this work item
  int overflow;
  uint32_t fresh;
  uint32_t cmax;
  unsigned long long retry_base;
  unsigned long long cbase;     // (compacted write-out)
  uint32_t wsum[8];
  uint32_t hist[kAggLdsHist];
};

// One tile's multi-split: each thread holds kPartPerThread records and their LDS bins (bin <
// 2^bin_bits, or kPartNoBin for none); output region of a bin = base_id + bin.  Ranks come from
// LDS atomics, the room in each region from ONE device atomic per (tile, non-empty bin), and the
// records are written from an LDS image sorted by bin, kPartSub at a time (coalesced runs).
// A workgroup barrier for LDS only: the LDS writes before it complete (lgkmcnt) but global loads
// and stores stay in flight across it -- __syncthreads() would wait for every outstanding vector
// memory operation (the write-out's stores, the reservation's no-return atomics, loads already
// issued) at each of a tile's barriers.  Used where the barrier orders LDS data only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Exclusive prefix of v over a workgroup of NT threads (NT / 64 <= 8 waves; wsum holds NT / 64); *total = the sum.
// Every thread must call it (it holds a barrier).
template <int NT>
__device__ inline uint32_t block_prefix(uint32_t v, uint32_t* wsum, uint32_t* total) {
  static_assert(NT % 64 == 0 && NT / 64 <= 8, "block_prefix: up to eight waves");
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63u) wsum[wave] = x;
  lds_barrier();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    before += (uint32_t)w < wave ? wsum[w] : 0u;
    tot += wsum[w];
  }
  *total = tot;
  return before + x - v;
}

// What a partition-path aggregation into an EMPTY table also produces (nullptr / 0 = off):
// the count-of-counts histogram of the new groups (so the metrics need no table scan), the
// largest count of each slice (so a top-N export skips slices below its threshold), and every
// slot of every slice written (zeros included), so the table needs no clearing beforehand.
struct AggTrack {
  unsigned long long* hist;   // kFreqHist bins
  unsigned long long* big;    // counts >= kFreqHist
  unsigned long long* n_big;
  unsigned long long big_cap;
  uint32_t* smax;             // per slice
  int write_all;
  FreqCompact cmp;            // cmp.slots != nullptr: write the occupied slots only (packed aggregation)
};

__device__ inline void track_count(AggLds& L, const AggTrack& tr, uint32_t c) {
  atomicMax(&L.cmax, c);
  if (!tr.hist) return;
  if (c < (uint32_t)kAggLdsHist) {
    atomicAdd(&L.hist[c], 1u);
  } else if (c < (uint32_t)kFreqHist) {
    atomicAdd(&tr.hist[c], 1ull);
  } else {
    const unsigned long long i = atomicAdd(tr.n_big, 1ull);
    if (i < tr.big_cap) tr.big[i] = c;
  }
}

#ifndef DQ_AGG_BATCH
#define DQ_AGG_BATCH 8
#endif
constexpr int kAggBatch = DQ_AGG_BATCH;  // records per thread loaded together

// Count record r (table hash h) in the LDS slice image; false if the image is full.  (The
// publishing lane's stores stay inside the loop iteration, with `done` tested by the loop: a
// lane of the same wave spinning on BUSY must see them in its next iteration, so the publish
// must not be sunk behind the loop -- an early return there hung the wave.)
__device__ inline bool lds_count(unsigned long long* K0, unsigned long long* K1, uint32_t* C, uint32_t* G,
                                 const FreqRec& r, uint64_t h) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  uint32_t s = (uint32_t)(h & (S - 1));
  bool done = false;
  for (uint32_t probe = 0; probe < S && !done;) {
    const unsigned long long c = atomicCAS(&K1[s], kLdsEmpty, kLdsBusy);
    if (c == kLdsEmpty) {  // claimed: publish the key, then count
      K0[s] = r.k0;
      G[s] = tag_of(h);  // (written back with the slot: no second hash of the key)
      __threadfence_block();
      atomicExch(&K1[s], r.k1);
      atomicAdd(&C[s], 1u);
      done = true;
    } else if (c == kLdsBusy) {
      // another lane is publishing this slot: look at it again
    } else if (c == r.k1 && __hip_atomic_load(&K0[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == r.k0) {
      atomicAdd(&C[s], 1u);
      done = true;
    } else {
      s = (s + 1) & (S - 1);
      ++probe;
    }
  }
  return done;
}

// A piece holding more keys than LDS: the row goes straight to the slice (rare; not inlined).
__device__ __noinline__ void piece_spill(const FreqTable& T, const FreqRec& r, unsigned long long k1, uint32_t len,
                                         uint64_t h, FreqRec* retry, unsigned long long* n_retry) {
  Key k;
  k.k0 = r.k0;
  k.k1 = k1;
  k.len = len;
  k.ptr = nullptr;
  k.hash = h;
  if (!global_insert<false>(T, k, 1ull)) emit_retry(retry, n_retry, r, 1ull);
}

// Aggregate records [r0, r1) of slice b.  owner: the work item holds the slice's whole bucket
// (load the slice, count in LDS, write it back with plain stores); otherwise it is one piece of a
// split bucket (count in LDS, merge into the slice with device-scope atomics).
template <int NT, bool OWNER_ONLY>
__device__ void agg_item(AggLds& L, const FreqTable& T, const FreqRec* __restrict__ recs, uint64_t r0, uint64_t r1,
                         uint64_t b, bool owner, int table_empty, FreqRec* retry, unsigned long long* n_retry,
                         unsigned long long* new_groups, const AggTrack* tr = nullptr) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  unsigned long long* K0 = L.K0;
  unsigned long long* K1 = L.K1;
  uint32_t* C = L.C;
  int& overflow = L.overflow;
  uint32_t& fresh = L.fresh;
  unsigned long long& retry_base = L.retry_base;
  {
    FreqSlot* slice = T.slots + (b << kFreqSliceLog);
    for (uint32_t s = threadIdx.x; s < S; s += NT) {
      if (owner && !table_empty) {
        const FreqSlot e = slice[s];
        const uint32_t len = (uint32_t)(e.ctrl & kLenMask);
        if (!(e.ctrl & kReady)) {
          K1[s] = kLdsEmpty;
        } else if ((e.ctrl & kHeapKey) || len > 15) {
          K1[s] = kLdsForeign;
        } else {
          K0[s] = e.k0;
          K1[s] = e.k1 | ((unsigned long long)len << kRecLenShift);
        }
      } else {
        K1[s] = kLdsEmpty;
      }
      C[s] = 0u;
    }
    if (threadIdx.x == 0) {
      overflow = 0;
      fresh = 0u;
      L.cmax = 0u;
    }
    __syncthreads();
    // records are loaded kAggBatch per thread at a time, all loads in flight together (one
    // dependent load per record made the loop latency-bound)
    FreqRec rb[kAggBatch];
    for (uint64_t base = r0; base < r1; base += (uint64_t)NT * kAggBatch) {
#pragma unroll
      for (int j = 0; j < kAggBatch; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i < r1) rb[j] = ld_rec(recs + i);
      }
#pragma unroll
      for (int j = 0; j < kAggBatch; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i >= r1) continue;
        const FreqRec r = rb[j];
        unsigned long long k1;
        uint32_t len;
        rec_unpack(r, &k1, &len);
        if (len == kRecHole) continue;
        const uint64_t h = hash_inline(r.k0, k1, len);
        if (!lds_count(K0, K1, C, L.G, r, h)) {
          if (OWNER_ONLY || owner) overflow = 1;
          else piece_spill(T, r, k1, len, h, retry, n_retry);
        }
      }
    }
    __syncthreads();
    if (!OWNER_ONLY && !owner) {  // merge the piece's counts into the shared slice
      for (uint32_t s = threadIdx.x; s < S; s += NT) {
        const uint32_t c = C[s];
        if (!c) continue;
        const unsigned long long kk1 = K1[s];
        Key k;
        k.k0 = K0[s];
        k.k1 = kk1 & kRecKeyMask;
        k.len = (uint32_t)(kk1 >> kRecLenShift);
        k.ptr = nullptr;
        k.hash = hash_inline(k.k0, k.k1, k.len);
        if (!global_insert<false>(T, k, (unsigned long long)c)) {
          FreqRec r;
          r.k0 = k.k0;
          r.k1 = kk1;
          emit_retry(retry, n_retry, r, (unsigned long long)c);
        }
      }
    } else if (overflow) {  // the slice is full: leave it untouched, hand the bucket's rows back
      if (threadIdx.x == 0) retry_base = atomicAdd(n_retry, (unsigned long long)(r1 - r0));
      __syncthreads();
      for (uint64_t i = r0 + threadIdx.x; i < r1; i += NT) retry[retry_base + (i - r0)] = recs[i];
      if (tr && tr->cmp.slots) {
        if (threadIdx.x == 0) tr->cmp.num[b] = 0u;  // (the slice starts out empty)
      } else if (tr && tr->write_all) {  // (the table was not cleared: the slice starts out empty)
        for (uint32_t s = threadIdx.x; s < S; s += NT) slice[s] = FreqSlot{0ull, 0ull, 0ull, 0ull};
      }
      if (tr && tr->smax && threadIdx.x == 0) tr->smax[b] = 0xFFFFFFFFu;  // unknown: never skipped
    } else if (tr && tr->cmp.slots) {
      // Occupied slots only (an empty table; as dq_freq_agg_packed_kernel): thread t owns slots
      // PER t .. PER t + PER - 1, its groups stored at consecutive places in slot order.
      constexpr uint32_t PER = S / (uint32_t)NT;
      static_assert(PER == 4u || PER == 8u, "four or eight slots per thread");
      const uint32_t t = threadIdx.x;
      uint32_t occ = 0u;
#pragma unroll
      for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t c = C[PER * t + j];
        if (!c) continue;
        occ |= 1u << j;
        track_count(L, *tr, c);
      }
      uint32_t tot;
      const uint32_t k = block_prefix<NT>((uint32_t)__builtin_popcount(occ), L.wsum, &tot);
      if constexpr (PER == 8u) {
        tr->cmp.bits[(b << 8) + t] = (uint8_t)occ;
      } else {
        const uint32_t hi = __shfl_down(occ, 1, 64);
        if (!(t & 1u)) tr->cmp.bits[(b << 8) + (t >> 1)] = (uint8_t)(occ | (hi << 4));
      }
      if (t == 0) {
        const unsigned long long at = atomicAdd(tr->cmp.cursor, (unsigned long long)tot);
        L.cbase = at;
        tr->cmp.base[b] = at;
        tr->cmp.num[b] = tot;
        if (tot) atomicAdd(new_groups, (unsigned long long)tot);
      }
      __syncthreads();
      FreqSlot* out = tr->cmp.slots + L.cbase + k;
#pragma unroll
      for (uint32_t j = 0; j < PER; ++j) {
        if (!(occ & (1u << j))) continue;
        const uint32_t s = PER * t + j;
        const unsigned long long k1 = K1[s];
        *out++ = FreqSlot{((unsigned long long)L.G[s] << 32) | kReady | (uint32_t)(k1 >> kRecLenShift),
                          (unsigned long long)C[s], K0[s], k1 & kRecKeyMask};
      }
      if (tr->smax && t == 0) tr->smax[b] = L.cmax;
    } else {
      for (uint32_t s = threadIdx.x; s < S; s += NT) {
        const uint32_t c = C[s];
        if (!c) {
          if (tr && tr->write_all) slice[s] = FreqSlot{0ull, 0ull, 0ull, 0ull};
          continue;
        }
        if (tr) track_count(L, *tr, c);
        FreqSlot& e = slice[s];
        bool is_new = false;
        if (!table_empty && (e.ctrl & kReady)) {
          e.count += c;
        } else {
          const unsigned long long k1 = K1[s];
          const uint32_t len = (uint32_t)(k1 >> kRecLenShift);
          FreqSlot n;
          n.ctrl = ((unsigned long long)L.G[s] << 32) | kReady | len;
          n.count = c;
          n.k0 = K0[s];
          n.k1 = k1 & kRecKeyMask;
          e = n;
          is_new = true;
        }
        const uint64_t nb = __ballot(is_new);  // one LDS add per wave, not one per new group
        if (nb && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(nb)) atomicAdd(&fresh, (uint32_t)__popcll(nb));
      }
      __syncthreads();
      if (threadIdx.x == 0 && fresh) atomicAdd(new_groups, (unsigned long long)fresh);
      if (tr && tr->smax && threadIdx.x == 0) tr->smax[b] = L.cmax;
    }
    __syncthreads();  // LDS is reused by the next work item
  }
}

__global__ __launch_bounds__(kBlock) void dq_freq_agg_kernel(FreqTable T, const FreqRec* __restrict__ recs,
                                                             const uint64_t* __restrict__ off,
                                                             const uint32_t* __restrict__ piece_start,
                                                             uint64_t n_buckets, int table_empty, FreqRec* retry,
                                                             unsigned long long* n_retry,
                                                             unsigned long long* new_groups) {
  __shared__ AggLds L;
  const uint32_t n_items = piece_start[n_buckets];
  for (uint32_t w = blockIdx.x; w < n_items; w += gridDim.x) {
    // the bucket of work item w: piece_start[b] <= w < piece_start[b + 1]
    uint64_t lo = 0, hi = n_buckets;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (piece_start[mid] <= w) lo = mid;
      else hi = mid;
    }
    const uint64_t b = lo;
    const bool owner = piece_start[b + 1] - piece_start[b] == 1u;
    const uint64_t r0 = off[b] + (uint64_t)(w - piece_start[b]) * kFreqAggPiece;
    const uint64_t r1 = min(off[b + 1], r0 + kFreqAggPiece);
    agg_item<kBlock, false>(L, T, recs, r0, r1, b, owner, table_empty, retry, n_retry, new_groups);
  }
}

// ---- partition path (large stagings: no counting pass, fixed-capacity regions) -------------
// Two passes of an LDS multi-split put every staged record into the region of its slice:
//  P1: stage array -> 2^b1 level-1 regions (top b1 bits of the table hash);
//  P2: each level-1 region -> the 2^(bits-b1) slice regions under it.
// A region has a fixed capacity (its expected share + a 6-sigma margin, sized on the host from
// the row count and the sketch's distinct estimate); a workgroup reserves its records' room in a
// region with ONE atomic per (tile, region), writes them from an LDS image sorted by region (runs
// of ~32 records, coalesced), and records beyond a region's capacity go to an overflow list that
// the sort path aggregates afterwards (skewed data).  Then dq_freq_agg_region_kernel aggregates
// each slice region in LDS as the owner of its slice.  Per pass: 16 B read + 16 B written per
// record (the sort moved 20 B keyed records three times, plus a key histogram pass).
#ifndef DQ_PART_NT
#define DQ_PART_NT 512
#endif
#ifndef DQ_PART_SUB
#define DQ_PART_SUB 2048
#endif
// 512-thread workgroups with LDS images of 2048 records: two workgroups per CU (registers allow
// 4 waves per SIMD), so one workgroup's load / reservation latency hides behind the other's
// LDS scatter and writes.
constexpr int kPartThreads = DQ_PART_NT;
constexpr int kPartPerThread = 16;
constexpr uint32_t kPartTile = (uint32_t)kPartThreads * kPartPerThread;  // records per tile
constexpr uint32_t kPartSub = DQ_PART_SUB;                               // records per LDS round
#ifndef DQ_PARTP_PER
#define DQ_PARTP_PER 24
#endif
#ifndef DQ_PARTP_SUB
#define DQ_PARTP_SUB 6144
#endif
// packed (8-byte) records: per thread and per LDS round of the level-2 split
constexpr int kPartPerThreadP = DQ_PARTP_PER;
constexpr uint32_t kPartTileP = (uint32_t)kPartThreads * kPartPerThreadP;
constexpr uint32_t kPartSubP = DQ_PARTP_SUB;
constexpr int kPartMaxBinBits = kPartMaxBits;
constexpr int kStageBinBits = 9;  // the level-1 split of the fused stage (dq_freq_api.inc kRegionBits)
constexpr uint32_t kPartNoBin = 0xFFFFu;
#ifndef DQ_STAGE_PER
#define DQ_STAGE_PER 12
#endif
constexpr int kStagePer = DQ_STAGE_PER;   // rows per thread per fused-stage tile (register budget)
// The fused stage's workgroups: 384 threads (6 waves) at 3 waves per SIMD -- two workgroups per
// CU, and 168 VGPRs per lane: a tile's 12 rows of key words in flight plus the next tile's offsets
// fit without spills (at 4 waves per SIMD, 128 VGPRs, they do not).
#ifndef DQ_STAGE_NT
#define DQ_STAGE_NT 512
#endif
constexpr int kStageThreads = DQ_STAGE_NT;
constexpr uint32_t kStageTile = (uint32_t)kStageThreads * kStagePer;
#ifndef DQ_STAGEP_SUB
#define DQ_STAGEP_SUB kStageTile
#endif
constexpr uint32_t kStageSubP = DQ_STAGEP_SUB;  // packed records per LDS round of the fused stage
#ifndef DQ_STAGE_SUB16
#define DQ_STAGE_SUB16 3072  // (2048: 33.3 ms per alnum C4 step, 3072: 32.4, 6144: 32.8 -- profiles/r06g_c4_alnum_stage_sub_ab.txt)
#endif
constexpr uint32_t kStageSub16 = DQ_STAGE_SUB16;  // 16-byte records per LDS round of the fused stage

// R: the record type of the regions -- FreqRec (16 B: key bytes + length) or, for a staging of
// digit keys, its packed word (uint64_t, dq_keypack.h).
template <int MAXB, typename R = FreqRec, uint32_t SUBN = (sizeof(R) == 8 ? kPartSubP : kPartSub)>
struct PartLdsT {
  static constexpr uint32_t SUB = SUBN;
  R rec[SUB];
  uint16_t bin[SUB];
  alignas(16) uint32_t hist[MAXB];
  alignas(16) uint32_t start[MAXB];
  unsigned long long gbase[MAXB];  // per bin: output index of the tile's position 0 (see part_tile)
  uint32_t lim[MAXB];              // per bin: tile positions below lim fit the bin's region
  uint32_t total;
};

__device__ inline uint64_t rec_hash(const FreqRec& r, bool* hole) {
  unsigned long long k1;
  uint32_t len;
  rec_unpack(r, &k1, &len);
  *hole = len == kRecHole;
  return hash_inline(r.k0, k1, len);
}
__device__ inline uint64_t rec_hash(uint64_t p, bool* hole) {
  *hole = p == kPackEmpty;  // (a row the row-order staging left empty)
  return hash_record_packed(p);
}

__device__ inline uint64_t rec_hash(const HashRec& r, bool* hole) {
  *hole = r.ref == kHashHole;
  return r.h;
}
__device__ inline uint64_t rec_hash(const UuidRec& r, bool* hole) {
  *hole = false;  // (the UUID stage is fused with the level-1 split: no row-order holes)
  return hash_uuid(r.lo, r.hi);
}
__device__ inline uint64_t rec_hash(const Raw16Rec& r, bool* hole) {
  *hole = false;  // (as UuidRec)
  return hash_inline(r.lo, r.hi, 16u);
}

// A record in the 16-byte form (what the overflow and retry lists and the sort path hold; a
// hashed record keeps its bits: the hashed path's lists are read by dq_freq_insert_hashed_kernel).
__device__ inline FreqRec rec_raw(const FreqRec& r) { return r; }
__device__ inline FreqRec rec_raw(const HashRec& r) {
  FreqRec f;
  f.k0 = r.h;
  f.k1 = r.ref;
  return f;
}
__device__ inline FreqRec rec_raw(const UuidRec& r) {  // (its bits; the host converts such lists)
  FreqRec f;
  f.k0 = r.lo;
  f.k1 = r.hi;
  return f;
}
__device__ inline FreqRec rec_raw(const Raw16Rec& r) {  // (as UuidRec)
  FreqRec f;
  f.k0 = r.lo;
  f.k1 = r.hi;
  return f;
}
__device__ inline FreqRec rec_raw(uint64_t p) {
  uint64_t k0, k1;
  uint32_t len;
  kp_unpack(p, &k0, &k1, &len);
  FreqRec r;
  r.k0 = k0;
  r.k1 = k1 | ((unsigned long long)len << kRecLenShift);
  return r;
}

// Phase timing of the fused stage (a diagnostic build only, -DDQ_STAGE_PROF): thread 0 of every
// workgroup adds the clock cycles of each phase of each tile to g_stage_prof (read back and
// printed per launch by launch_freq_stage_part).
#ifdef DQ_STAGE_PROF
__device__ unsigned long long g_stage_prof[8];
__device__ unsigned long long g_stage_blk[4096][2];  // per workgroup: wall-clock start, end
#define DQ_PROF_MARK(PROF, i)                                                        \
  do {                                                                               \
    if (PROF && threadIdx.x == 0) {                                                  \
      const unsigned long long now_ = wall_clock64();                                \
      if (i > 0) atomicAdd(&g_stage_prof[i - 1], now_ - prof_t_);                    \
      prof_t_ = now_;                                                                \
    }                                                                                \
  } while (0)
#else
#define DQ_PROF_MARK(PROF, i) do { } while (0)
#endif


struct NoMid {
  __device__ void operator()() const {}
};
// pre_res(): called as the tile's room is reserved (the fused stage reads its abort flag there).
template <int PER, int MAXB, typename R, uint32_t SUBN, bool PROF = false, int WOUT_UNROLL = 0,
          bool REC_LDS = false, int NT = kPartThreads, typename PreRes = NoMid>
__device__ inline void part_tile(PartLdsT<MAXB, R, SUBN>& L, const R (&rec)[PER], uint32_t (&bin)[PER],
                                 uint32_t nb, uint64_t base_id, R* __restrict__ out, uint64_t out_cap,
                                 unsigned long long* out_fill, FreqRec* ovf, unsigned long long* ovf_n,
                                 uint64_t ovf_cap, unsigned int* flag, unsigned long long* staged,
                                 const unsigned long long* region_start = nullptr, unsigned long long prof_t_ = 0,
                                 const PreRes& pre_res = PreRes()) {
  // region_start != nullptr: exact regions -- output region id starts at record region_start[id]
  // of `out` (sizes counted beforehand: nothing can overflow), out_fill is its cursor
  constexpr uint32_t SUB = SUBN;
  const uint32_t t = threadIdx.x;
  DQ_PROF_MARK(PROF, 1);
  for (uint32_t i = t; i < nb; i += NT) L.hist[i] = 0u;
  lds_barrier();
  DQ_PROF_MARK(PROF, 2);
  // rank of each record within its bin (LDS atomics), packed with the bin: rank << 16 | bin
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (bin[i] != kPartNoBin) bin[i] |= atomicAdd(&L.hist[bin[i]], 1u) << 16;
  lds_barrier();
  DQ_PROF_MARK(PROF, 3);
  // exclusive scan of the bins by wave 0 (nb / 64 consecutive bins per lane; 512 bins -- the
  // fused stage's level-1 split -- as two 16-byte LDS reads and writes per lane)
  if (t < 64) {
    if (nb == 512u && MAXB >= 512) {
      const uint4 h0 = reinterpret_cast<const uint4*>(L.hist)[2 * t], h1 = reinterpret_cast<const uint4*>(L.hist)[2 * t + 1];
      const uint32_t s = h0.x + h0.y + h0.z + h0.w + h1.x + h1.y + h1.z + h1.w;
      uint32_t incl = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if ((int)t >= d) incl += o;
      }
      uint4 s0, s1;
      s0.x = incl - s;
      s0.y = s0.x + h0.x;
      s0.z = s0.y + h0.y;
      s0.w = s0.z + h0.z;
      s1.x = s0.w + h0.w;
      s1.y = s1.x + h1.x;
      s1.z = s1.y + h1.y;
      s1.w = s1.z + h1.z;
      reinterpret_cast<uint4*>(L.start)[2 * t] = s0;
      reinterpret_cast<uint4*>(L.start)[2 * t + 1] = s1;
      if (t == 63) {
        L.total = incl;
        if (staged && incl) atomicAdd(staged, (unsigned long long)incl);
      }
    } else {
      const uint32_t per = (nb + 63u) / 64u;
      uint32_t s = 0;
      for (uint32_t k = 0; k < per; ++k) {
        const uint32_t b = t * per + k;
        if (b < nb) s += L.hist[b];
      }
      uint32_t incl = s;
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if ((int)t >= d) incl += o;
      }
      uint32_t run = incl - s;
      for (uint32_t k = 0; k < per; ++k) {
        const uint32_t b = t * per + k;
        if (b < nb) {
          L.start[b] = run;
          run += L.hist[b];
        }
      }
      if (t == 63) {
        L.total = incl;
        if (staged && incl) atomicAdd(staged, (unsigned long long)incl);
      }
    }
  }
  lds_barrier();
  DQ_PROF_MARK(PROF, 4);
  pre_res();  // (the fused stage's flag read: its latency overlaps the reservation atomics')
  // The tile's room in each bin's region: ONE device atomic per non-empty bin, issued here and
  // published to LDS only after the records are placed in the image, so the atomics' latency
  // overlaps that work.  Published per bin: gbase = the output index of tile position 0 (the
  // bin's first record sits at position start[b]) and lim = the positions that fit the region.
  constexpr int GB = (MAXB + NT - 1) / NT;
  unsigned long long room[GB];
#pragma unroll
  for (int k = 0; k < GB; ++k) {
    const uint32_t b = t + (uint32_t)k * NT;
    room[k] = 0ull;
    if (b < nb) {
      const uint32_t c = L.hist[b];
      if (c) room[k] = atomicAdd(&out_fill[base_id + b], (unsigned long long)c);
    }
  }
  auto publish = [&]() {
#pragma unroll
    for (int k = 0; k < GB; ++k) {
      const uint32_t b = t + (uint32_t)k * NT;
      if (b < nb) {
        const uint64_t st = L.start[b], fill = room[k];
        if (region_start) {
          L.gbase[b] = region_start[base_id + b] + fill - st;
          L.lim[b] = 0xFFFFFFFFu;
        } else {
          L.gbase[b] = (base_id + b) * out_cap + fill - st;
          const uint64_t lim = out_cap + st > fill ? out_cap + st - fill : 0ull;
          L.lim[b] = lim < 0xFFFFFFFFull ? (uint32_t)lim : 0xFFFFFFFFu;
        }
      }
    }
  };
  const uint32_t total = L.total;
  DQ_PROF_MARK(PROF, 5);
  // REC_LDS: the caller left the records in L.rec in row order (record i of thread t at
  // i * NT + t; registers are short while the keys load): read back, then sorted
  R rl[PER];
  if constexpr (REC_LDS) {
    static_assert(SUB >= (uint32_t)PER * (uint32_t)NT, "a tile's records in one image");
#pragma unroll
    for (int i = 0; i < PER; ++i) rl[i] = L.rec[i * NT + t];
    lds_barrier();
  }
  for (uint32_t r0 = 0; r0 < total; r0 += SUB) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if ((bin[i] & 0xFFFFu) == kPartNoBin) continue;
      const uint32_t b = bin[i] & 0xFFFFu;
      const uint32_t p = L.start[b] + (bin[i] >> 16) - r0;
      if (p < SUB) {
        L.rec[p] = REC_LDS ? rl[i] : rec[i];
        L.bin[p] = (uint16_t)b;
      }
    }
    if (r0 == 0) publish();
    lds_barrier();
    DQ_PROF_MARK(PROF, 6);
    const uint32_t m = min(SUB, total - r0);
    auto put = [&](uint32_t j) {
      const uint32_t b = L.bin[j];
      const uint32_t pos = r0 + j;  // the record's tile position
      const R r = L.rec[j];
      if (pos < L.lim[b]) {
        out[L.gbase[b] + pos] = r;
      } else {  // the region is full: the overflow list (16-B records, aggregated by the sort path)
        const unsigned long long k = atomicAdd(ovf_n, 1ull);
        if (k < ovf_cap) ovf[k] = rec_raw(r);
        else atomicOr(flag, 1u);
      }
    };
    if constexpr (WOUT_UNROLL > 0) {
      // (a bounded unroll: the fused stage's registers)
#pragma unroll WOUT_UNROLL
      for (uint32_t j = t; j < m; j += NT) put(j);
    } else {  // the compiler's choice (the level-2 passes: no loop-carried state to keep)
      for (uint32_t j = t; j < m; j += NT) put(j);
    }
    lds_barrier();
    DQ_PROF_MARK(PROF, 7);
    // an image that holds a whole tile: one round, so rec[] is dead once it is in LDS
    if constexpr (SUB >= (uint32_t)PER * (uint32_t)NT) break;
  }
}

// in_fill == nullptr: level 1, tile blockIdx.x of in[0, in_n).  Otherwise level 2: tile
// blockIdx.x of region blockIdx.y (in + y * in_cap, min(in_fill[y], in_cap) records).
// A record's output region = the top id_bits of its hash; its LDS bin = the low bin_bits of
// that id (the higher id bits are the input region's, uniform over the tile).
#ifndef DQ_PARTP_WAVES
#define DQ_PARTP_WAVES 4
#endif
// MAXB: LDS bin arrays for up to that many bins (512 when bin_bits <= 9: more LDS for the image).
template <typename R, int MAXB>
__global__ __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(MAXB <= 512 ? DQ_PARTP_WAVES : 1))) void dq_freq_part_kernel(
    const R* __restrict__ in, uint64_t in_n, const unsigned long long* __restrict__ in_fill, uint64_t in_cap,
    int id_bits, int bin_bits, R* __restrict__ out, uint64_t out_cap, unsigned long long* out_fill,
    FreqRec* ovf, unsigned long long* ovf_n, uint64_t ovf_cap, unsigned int* flag, unsigned long long* staged) {
  // (2048 bins: the smaller LDS rounds keep two workgroups per CU)
  __shared__ PartLdsT<MAXB, R, (sizeof(R) == 8 && MAXB <= 512 ? kPartSubP : kPartSub)> L;
  constexpr uint32_t TILE = sizeof(R) == 8 ? kPartTileP : kPartTile;
  const uint32_t t = threadIdx.x;
  const uint32_t nb = 1u << bin_bits;
  uint64_t base_id = 0, begin, count;
  if (in_fill) {
    const uint64_t r = blockIdx.y;
    const unsigned long long f = in_fill[r];
    const uint64_t have = f < in_cap ? f : in_cap;
    begin = (uint64_t)blockIdx.x * TILE;
    if (begin >= have) return;
    count = min((uint64_t)TILE, have - begin);
    begin += r * in_cap;
    base_id = r << bin_bits;
  } else {
    begin = (uint64_t)blockIdx.x * TILE;
    if (begin >= in_n) return;
    count = min((uint64_t)TILE, in_n - begin);
  }
  constexpr int PER = sizeof(R) == 8 ? kPartPerThreadP : kPartPerThread;
  R rec[PER];
  uint32_t bin[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t j = (uint32_t)i * kPartThreads + t;
    if (j < count) rec[i] = in[begin + j];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t j = (uint32_t)i * kPartThreads + t;
    bin[i] = kPartNoBin;
    if (j < count) {
      bool hole;
      const uint64_t h = rec_hash(rec[i], &hole);
      if (!hole) bin[i] = (uint32_t)(h >> (64 - id_bits)) & (nb - 1u);
    }
  }
  part_tile(L, rec, bin, nb, base_id, out, out_cap, out_fill, ovf, ovf_n, ovf_cap, flag, staged);
}

// ---- bucket split: the sort path's grouping of staged records by slice (small stagings, and the
// partition path's retry / skew fall-backs), hand-written on the same LDS multi-split: a slice id
// of `bits` (<= 22) hash bits is split in two levels, b1 = min(bits, 11) high bits, then the low
// b2 = bits - b1 bits inside each level-1 region.  Each level COUNTS first (one device atomic per
// (tile, non-empty bin)), the counts are scanned into exact region starts, and the SCATTER pass
// writes every record inside its region (one atomic cursor add per (tile, bin)): nothing can
// overflow, a hot key costs one atomic per tile, and level 2's counts are the per-slice record
// counts the aggregation's work items come from.  Holes (length byte 0xFF) are dropped.
//   level 1 (in_off == nullptr): tile blockIdx.x of in[0, n), bin = slice >> b2, id = bin;
//   level 2: tile blockIdx.x of region y = blockIdx.y, in[in_off[y], in_off[y + 1]),
//            bin = slice & (2^b2 - 1), id = (y << b2) | bin = the slice.
// count != nullptr: add the bins' counts to count[id]; else scatter to out (region_start, cursor).
__global__ __launch_bounds__(kPartThreads) void dq_freq_split_kernel(
    const FreqRec* __restrict__ in, uint64_t n, const unsigned long long* __restrict__ in_off, int bits, int b2,
    unsigned long long* count, FreqRec* __restrict__ out, const unsigned long long* __restrict__ region_start,
    unsigned long long* cursor) {
  __shared__ PartLdsT<(1 << kPartMaxBinBits)> L;
  const uint32_t t = threadIdx.x;
  const bool level2 = in_off != nullptr;
  const uint32_t nb = level2 ? (1u << b2) : (1u << (bits - b2));
  uint64_t begin, end, base_id = 0;
  if (level2) {
    begin = in_off[blockIdx.y] + (uint64_t)blockIdx.x * kPartTile;
    end = in_off[blockIdx.y + 1];
    base_id = (uint64_t)blockIdx.y << b2;
  } else {
    begin = (uint64_t)blockIdx.x * kPartTile;
    end = n;
  }
  if (begin >= end) return;
  const uint64_t cnt_in = min((uint64_t)kPartTile, end - begin);
  FreqRec rec[kPartPerThread];
  uint32_t bin[kPartPerThread];
#pragma unroll
  for (int i = 0; i < kPartPerThread; ++i) {
    const uint32_t j = (uint32_t)i * kPartThreads + t;
    if (j < cnt_in) rec[i] = ld_rec(in + begin + j);
  }
#pragma unroll
  for (int i = 0; i < kPartPerThread; ++i) {
    const uint32_t j = (uint32_t)i * kPartThreads + t;
    bin[i] = kPartNoBin;
    if (j < cnt_in) {
      bool hole;
      const uint64_t h = rec_hash(rec[i], &hole);
      const uint32_t slice = bits ? (uint32_t)(h >> (64 - bits)) : 0u;
      if (!hole) bin[i] = level2 ? (slice & (nb - 1u)) : (slice >> b2);
    }
  }
  if (count) {  // counting pass: LDS histogram, one device atomic per non-empty bin
    for (uint32_t i = t; i < nb; i += kPartThreads) L.hist[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPartPerThread; ++i)
      if (bin[i] != kPartNoBin) atomicAdd(&L.hist[bin[i]], 1u);
    __syncthreads();
    for (uint32_t b = t; b < nb; b += kPartThreads) {
      const uint32_t c = L.hist[b];
      if (c) atomicAdd(&count[base_id + b], (unsigned long long)c);
    }
    return;
  }
  part_tile(L, rec, bin, nb, base_id, out, ~0ull, cursor, nullptr, nullptr, 0, nullptr, nullptr, region_start);
}

// Exclusive scan of n counts (in place, 64-bit): chunks of kScanChunk by one block each, the chunk
// sums scanned by one block, then added back.  (The bucket split's region starts and the
// aggregation's work-item numbering.)
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 4;
constexpr uint32_t kScanChunk = (uint32_t)kScanThreads * kScanPer;

template <typename T>
__device__ inline T block_exclusive_scan(T v, T* warp_sums, T* total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  T incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(incl, d, 64);
    if ((int)lane >= d) incl += o;
  }
  if (lane == 63) warp_sums[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    const uint32_t nw = blockDim.x >> 6;
    T w = lane < nw ? warp_sums[lane] : (T)0;
    T wi = w;
    for (int d = 1; d < 64; d <<= 1) {
      const T o = __shfl_up(wi, d, 64);
      if ((int)lane >= d) wi += o;
    }
    if (lane < nw) warp_sums[lane] = wi - w;
    if (lane == nw - 1) *total = wi;
  }
  __syncthreads();
  return warp_sums[wave] + incl - v;
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void dq_scan_chunks_kernel(T* data, uint64_t n, T* sums) {
  __shared__ T ws[kScanThreads / 64];
  __shared__ T total;
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanPer;
  T v[kScanPer];
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = base + k < n ? data[base + k] : (T)0;
    s += v[k];
  }
  T run = block_exclusive_scan<T>(s, ws, &total);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (base + k < n) data[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// one block: exclusive scan of the m chunk sums (in place), in rounds of kScanChunk with a carry
template <typename T>
__global__ __launch_bounds__(kScanThreads) void dq_scan_sums_kernel(T* sums, uint64_t m) {
  __shared__ T ws[kScanThreads / 64];
  __shared__ T total;
  T carry = 0;
  for (uint64_t r = 0; r < m; r += kScanChunk) {
    const uint64_t base = r + (uint64_t)threadIdx.x * kScanPer;
    T v[kScanPer];
    T s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = base + k < m ? sums[base + k] : (T)0;
      s += v[k];
    }
    T run = carry + block_exclusive_scan<T>(s, ws, &total);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      if (base + k < m) sums[base + k] = run;
      run += v[k];
    }
    carry += total;
    __syncthreads();  // ws / total are rewritten by the next round
  }
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void dq_scan_add_kernel(T* data, uint64_t n, const T* sums) {
  const T add = sums[blockIdx.x];
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanPer;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < n) data[base + k] += add;
}

// pieces[b] = work items of slice b's bucket (its count cut into kFreqAggPiece records), b < n
__global__ __launch_bounds__(kBlock) void dq_freq_pieces_kernel(const unsigned long long* __restrict__ counts,
                                                                uint64_t n, uint32_t* pieces) {
  for (uint64_t b = (uint64_t)blockIdx.x * kBlock + threadIdx.x; b <= n; b += (uint64_t)gridDim.x * kBlock)
    pieces[b] = b < n ? (uint32_t)((counts[b] + kFreqAggPiece - 1) / kFreqAggPiece) : 0u;
}

// Stage + level-1 partition fused: the rows of one batch become records written straight into
// their level-1 regions (top b1 bits of the table hash), so the staging is not written and read
// back in row order.  Tiles of kPartTile rows, grid-stride.  The sketch, the staged count and
// the long-key flag are kept as by dq_freq_stage_kernel.  Single-string keys (the common case)
// load their offsets, then their bytes, for all of a thread's rows at once.
// PACK (single string key only): the regions hold packed digit records (uint64_t, dq_keypack.h);
// a key that is not a digit string goes to the overflow list as a 16-B record (counted there and
// in `staged`), and a batch with more of them than the list holds raises `flag` (the host then
// rolls it back and stages the table's keys as 16-B records from then on).
// A pointer every lane holds alike, in scalar registers (a buffer descriptor built from a value
// the compiler cannot prove uniform is re-made per lane in a waterfall loop).
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// The validity bits of a tile of NT * PER rows starting at row r0 (a multiple of 32; m rows in
// the batch) as ONE dword per lane: row j of lane l of wave w is bit l & 31 of tile dword
// 2 NW j + 2 w + (l >> 5) (NW = NT / 64), which lane 2 j + (l >> 5) of the wave loads
// (stage_valid_mask).  0 for a column without a bitmap (never read then).
template <int NT, int PER>
__device__ __forceinline__ uint32_t tile_valid_word(const uint8_t* validity, int64_t r0, uint32_t m) {
  static_assert(2 * PER <= 64, "two lanes per row of the tile");
  if (validity == nullptr) return 0u;
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint8_t* vb = validity + (r0 >> 3);
  const uint32_t nbytes = (m + 7u) >> 3;
  // a 4-byte aligned bitmap (the usual case): the range covers the bitmap's last dword whole (it
  // lies in the page of the bitmap's last byte; the bits past the batch are never used)
  const bool al = ((uintptr_t)vb & 3u) == 0u;
  const __amdgpu_buffer_rsrc_t rs_v =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vb), 0, (int)(al ? (nbytes + 3u) & ~3u : nbytes), 0x00020000);
  const uint32_t dw = 2u * (NT / 64) * (l >> 1) + 2u * w + (l & 1u);
  uint32_t vword = 0u;
  if (l < 2u * PER) {
    if (al || 4u * dw + 4u <= nbytes) {
      vword = __builtin_amdgcn_raw_buffer_load_b32(rs_v, (int)(4u * dw), 0, 0);
    } else {  // an unaligned bitmap's last, partial dword: byte by byte (a range check is per dword)
      for (uint32_t k = 0; k < 4u; ++k)
        if (4u * dw + k < nbytes)
          vword |= (uint32_t)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rs_v, (int)(4u * dw + k), 0, 0) << (8u * k);
    }
  }
  return vword;
}

// The (begin, end) offsets of tile `tl`'s kStagePer rows of one utf8 column (row j of this thread
// = tl * kStageTile + j * kStageThreads + threadIdx.x): one 8-byte load of each row's offset pair
// through a descriptor of the tile's offsets (rows past the batch read 0).  The validity bits
// come as ONE dword per lane: row j of lane l of wave w is bit l & 31 of tile dword
// 16 j + 2 w + (l >> 5), which lane 2 j + (l >> 5) of the wave loads (stage_valid_mask).
__device__ __forceinline__ void stage_offsets(const DevColumn& c0, int64_t n_rows, int64_t tl,
                                              uint32_t (&pob)[kStagePer], uint32_t (&poe)[kStagePer],
                                              uint32_t& vword) {
  const int64_t r0 = tl * (int64_t)kStageTile;
  const int64_t left = n_rows - r0;
  const uint32_t m = (uint32_t)(left < (int64_t)kStageTile ? left : (int64_t)kStageTile);
  const uint32_t t = threadIdx.x;
  // (the validity dword first: its address arithmetic waits on nothing then)
  vword = tile_valid_word<kStageThreads, kStagePer>(uniform_ptr(c0.validity), r0, m);
  const __amdgpu_buffer_rsrc_t rs_off = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t*>(uniform_ptr(c0.offsets) + r0), 0, (int)(4u * (m + 1u)), 0x00020000);
#pragma unroll
  for (int j = 0; j < kStagePer; ++j) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_off, (int)(4u * ((uint32_t)j * kStageThreads + t)), 0, 0);
    pob[j] = v[0];
    poe[j] = v[1];
  }
}

// Key bytes through a buffer descriptor over the heap [0, heap_end).  A buffer load's range check
// is per dword of the load, counted from the load's own offset, so a 16-byte load reaching past
// heap_end would zero whole dwords -- key bytes included.  So every key is read as ONE unaligned
// 16-byte load at min(ob, heap_end - 16), always wholly in range: a key that starts within the
// heap's last 16 bytes lands s = ob - (heap_end - 16) bytes into the words (s + n <= 16), and is
// shifted down when it is processed (key_shr_bytes; rare, no memory access in the branch).  The
// kernels using it hand a batch whose whole heap is under 16 bytes back to the host's general
// path (no per-load branch for it).
__device__ __forceinline__ void key_load16(__amdgpu_buffer_rsrc_t rs_vals, uint32_t heap_end, uint32_t ob, uint32_t (&w)[4]) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_vals, (int)min(ob, heap_end - 16u), 0, 0);
  w[0] = v[0];
  w[1] = v[1];
  w[2] = v[2];
  w[3] = v[3];
}
// The byte position of the key in key_load16's words (0 unless it starts in the last 16 bytes;
// clamped to 15: only an empty key can start at heap_end itself).
__device__ __forceinline__ uint32_t key_shift(uint32_t ob, uint32_t heap_end) {
  const uint32_t s = ob > heap_end - 16u ? ob - (heap_end - 16u) : 0u;  // (heap_end >= 16)
  return s < 15u ? s : 15u;
}
// w >>= 8 s bits (128-bit, s in 1..15).
__device__ __forceinline__ void key_shr_bytes(uint32_t (&w)[4], uint32_t s) {
  const uint32_t q = s >> 2, r = 8u * (s & 3u);
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = q == 0 ? w[i] : q == 1 ? (i < 3 ? w[i + 1] : 0u) : q == 2 ? (i < 2 ? w[i + 2] : 0u) : (i < 1 ? w[3] : 0u);
  d[4] = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbit(d[i + 1], d[i], r);
}
// The fused stage's sizing sketch in min form (as the value scan's HLL, dq_scan_fast.hip): per
// register the minimum of s = bits 54..24 of the hash (in bits 30..0) with one unconditional
// ds_min -- no LDS read and wait per row -- turned into the rank nlz(s) when folded (an untouched
// register stays 0xFFFFFFFF; s = 0, rank >= 32, is taken as 32: the sketch only sizes the table).
__device__ __forceinline__ void stage_sketch(uint32_t* regs, uint64_t h) {
  const uint32_t s = __builtin_amdgcn_alignbit((uint32_t)(h >> 32), (uint32_t)h, 24) & 0x7FFFFFFFu;
  __hip_atomic_fetch_min(&regs[(uint32_t)(h >> kHllIdxShift)], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t stage_sketch_rank(uint32_t s) { return s ? (uint32_t)__builtin_clz(s) : 32u; }

// stage_pack's selectors for a key of n <= 15 bytes, word i: byte j of the word is the key's
// byte (v_perm selector 4 + j, from the first operand) if 4 i + j < n, else '0' (selector 0:
// byte 0 of the constant 0x30303030).
__host__ __device__ inline uint32_t stage_pack_sel(uint32_t n, int i) {
  uint32_t s = 0u;
  for (uint32_t j = 0; j < 4u; ++j)
    if (4u * (uint32_t)i + j < n) s |= (4u + j) << (8u * j);
  return s;
}

// kp_pack of a key given as its first 16 loaded bytes w (bytes past its length n <= 15
// arbitrary): the bytes past n become '0' with one v_perm per word (selectors by length from
// an LDS table), then kp_pack's digit test and nibble packing -- the same word kp_pack makes of
// the masked key, without the length masks' shifts and selects.
__device__ __forceinline__ bool stage_pack(const uint32_t (&w)[4], uint32_t n, uint4 sel, uint64_t* p) {
  const uint32_t y0 = __builtin_amdgcn_perm(w[0], 0x30303030u, sel.x), y1 = __builtin_amdgcn_perm(w[1], 0x30303030u, sel.y);
  const uint32_t y2 = __builtin_amdgcn_perm(w[2], 0x30303030u, sel.z), y3 = __builtin_amdgcn_perm(w[3], 0x30303030u, sel.w);
  if (kp_nondigit4(y0) | kp_nondigit4(y1) | kp_nondigit4(y2) | kp_nondigit4(y3)) return false;
  const uint32_t lo = kp_nib4(y0) | (kp_nib4(y1) << 16);
  const uint32_t hi = kp_nib4(y2) | (kp_nib4(y3) << 16) | (n << 28);
  *p = (uint64_t)lo | ((uint64_t)hi << 32);
  return true;
}

// The validity of row j of every lane of this wave, as a lane mask (from stage_offsets' vword).
__device__ __forceinline__ uint64_t stage_valid_mask(uint32_t vword, int j) {
  const uint32_t lo = __builtin_amdgcn_readlane(vword, 2 * j), hi = __builtin_amdgcn_readlane(vword, 2 * j + 1);
  return ((uint64_t)hi << 32) | lo;
}

#ifndef DQ_STAGE_WIN
#define DQ_STAGE_WIN 4
#endif
constexpr int kStageWin = DQ_STAGE_WIN < DQ_STAGE_PER ? DQ_STAGE_WIN : DQ_STAGE_PER;  // rows' key loads in flight

#ifndef DQ_STAGE_WOUT_UNROLL
#define DQ_STAGE_WOUT_UNROLL 2
#endif
#ifndef DQ_STAGEP_WAVES
#define DQ_STAGEP_WAVES 4
#endif
template <bool ONE_STRING, bool PACK>
__global__ __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(DQ_STAGEP_WAVES))) void dq_freq_stage_part_kernel(
    FreqKeySpec ks, const DevColumn* __restrict__ cols, int64_t n_rows, int b1,
    typename std::conditional<PACK, uint64_t, FreqRec>::type* __restrict__ out, uint64_t cap1,
    unsigned long long* fill1, FreqRec* ovf, unsigned long long* ovf_n, uint64_t ovf_cap, unsigned int* flag,
    uint32_t* hll, unsigned long long* long_key, unsigned long long* staged) {
  static_assert(ONE_STRING || !PACK, "packed records are staged from one string key column");
  using R = typename std::conditional<PACK, uint64_t, FreqRec>::type;
  __shared__ PartLdsT<(1 << kStageBinBits), R, (PACK ? kStageSubP : kStageSub16)> L;
  __shared__ uint32_t regs[kHllM];
  __shared__ uint4 psel[16];  // stage_pack's byte selectors by key length
  const uint32_t t = threadIdx.x;
  const uint32_t nb = 1u << b1;
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  if (PACK && t < 16u) psel[t] = make_uint4(stage_pack_sel(t, 0), stage_pack_sel(t, 1), stage_pack_sel(t, 2), stage_pack_sel(t, 3));
#ifdef DQ_STAGE_PROF
  if (t == 0 && blockIdx.x < 4096u) g_stage_blk[blockIdx.x][0] = wall_clock64();
#endif
  lds_barrier();
  const DevColumn& c0 = cols[ks.key_cols[0]];
  alignas(8) uint8_t scratch[kMaxLocalKey];
  const int64_t n_tiles = (n_rows + kStageTile - 1) / kStageTile;
  uint32_t n_side = 0;  // PACK: this thread's keys put on the overflow list (not digit strings)
  // ONE_STRING: the key bytes through one buffer descriptor (a utf8 column's offsets are int32, so
  // its heap is < 2 GiB); each tile's offsets through a descriptor of that tile's offsets (bounded,
  // so rows past the batch read 0), as (begin, end) pairs: one 8-byte load per row.
  const uint32_t heap_end = ONE_STRING ? __builtin_amdgcn_readfirstlane((uint32_t)uniform_ptr(c0.offsets)[n_rows]) : 0u;
  const uint8_t* vals = static_cast<const uint8_t*>(uniform_ptr(c0.values));
  const __amdgpu_buffer_rsrc_t rs_vals =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vals), 0, (int)heap_end, 0x00020000);
  if (ONE_STRING && heap_end < 16u) {  // (a heap under 16 bytes: key_load16's general path, as a long key)
    if (blockIdx.x == 0 && t == 0) atomicMax(long_key, 16ull);
    return;
  }
  const bool has_validity = uniform_ptr(c0.validity) != nullptr;
  uint32_t pob[kStagePer], poe[kStagePer], vword = 0u;
  // ONE_STRING: a tile's key words (kw), key lengths as bytes, 4 to a register (lens: n | s << 4
  // for a key of n <= 15 bytes at byte s of its loaded words -- key_shift; s + n <= 16, so the
  // codes below are never taken by a key; kLenNull = Histogram's NULL, "NullValue"; kLenLong = a
  // key over 15 bytes: the batch is rolled back) and its selected rows (sel)
  constexpr uint32_t kLenNull = 254u, kLenLong = 255u;
  uint32_t kw[kStagePer][4], lens[(kStagePer + 3) / 4], sel = 0u;
  auto tile_lens = [&](int64_t tl) {  // lens / sel of tile tl, from its offsets (pob / poe / vword)
    const int64_t r0 = tl * (int64_t)kStageTile;
    sel = 0u;
#pragma unroll
    for (int j = 0; j < (kStagePer + 3) / 4; ++j) lens[j] = 0u;
#pragma unroll
    for (int j = 0; j < kStagePer; ++j) {
      const int64_t row = r0 + j * kStageThreads + t;
      const uint32_t n = poe[j] - pob[j];
      const bool valid = !has_validity || ((stage_valid_mask(vword, j) >> (t & 63u)) & 1u);
      if (row < n_rows && (valid || ks.null_as_key)) sel |= 1u << j;
      const uint32_t nb8 = (row < n_rows && !valid) ? kLenNull : (n > 15u ? kLenLong : n | (key_shift(pob[j], heap_end) << 4));
      lens[j / 4] |= nb8 << (8 * (j % 4));
    }
  };
  // PACK: once the overflow list has filled up (a column of keys that are not digit strings) the
  // batch will be rolled back, so the workgroups stop: thread 0 reads `flag` while each tile's
  // room is reserved (abort_v) and the workgroup leaves at the next tile's top.
  __shared__ unsigned int abort_s;
  unsigned int abort_v = 0u;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    if constexpr (PACK) {
      if (tile != (int64_t)blockIdx.x) {
        if (t == 0) abort_s = abort_v;
        lds_barrier();
        if (abort_s) break;
      }
    }
    const int64_t row0 = tile * (int64_t)kStageTile;
    unsigned long long prof_t_ = 0;
    (void)prof_t_;
    DQ_PROF_MARK(true, 0);
    R rec[kStagePer];
    uint32_t bin[kStagePer];
    uint32_t too_long = 0u;
    if constexpr (ONE_STRING) {
      // The tile's offsets (and validity bits: one word per lane), then its keys 16 bytes each
      // from the key's first byte (key_load16) through a window of kStageWin rows in flight:
      // rows [0, kStageWin) now, row j + kStageWin as row j is processed.  (Deeper pipelines --
      // the next tile's offsets or keys loaded during this tile's split -- need more registers
      // than four waves per SIMD leave; at three waves a 6-wave workgroup runs alone on its CU.)
      stage_offsets(c0, n_rows, tile, pob, poe, vword);
      tile_lens(tile);
#pragma unroll
      for (int j = 0; j < kStageWin; ++j) key_load16(rs_vals, heap_end, pob[j], kw[j]);
#pragma unroll
      for (int j = 0; j < kStagePer; ++j) {
        if (j + kStageWin < kStagePer) key_load16(rs_vals, heap_end, pob[j + kStageWin], kw[j + kStageWin]);
        bin[j] = kPartNoBin;
        if (!((sel >> j) & 1u)) continue;
        uint32_t n = (lens[j / 4] >> (8 * (j % 4))) & 0xFFu;
        if (n == kLenLong) {  // (a key longer than 15 bytes: the host only tests > 15)
          too_long = 16u;
          continue;
        }
        if (n != kLenNull) {
          if (n > 15u) key_shr_bytes(kw[j], n >> 4);  // a key in the heap's last 16 bytes (rare)
          n &= 15u;
        }
        // the key bytes (NULL: Histogram's "NullValue"), masked to the length
        auto key_words = [&](uint64_t& k0, uint64_t& k1, uint32_t& len) {
          if (n == kLenNull) {
            len = 9;
            k0 = kNullK0;
            k1 = kNullK1;
          } else {
            const uint64_t lo = (uint64_t)kw[j][0] | ((uint64_t)kw[j][1] << 32);
            const uint64_t hi = (uint64_t)kw[j][2] | ((uint64_t)kw[j][3] << 32);
            len = n;
            k0 = n >= 8 ? lo : (lo & ((1ull << (8u * n)) - 1ull));
            k1 = n > 8 ? (hi & ((1ull << (8u * (n - 8u))) - 1ull)) : 0ull;
          }
        };
        uint64_t h;
        if constexpr (PACK) {
          // the digit test and packing straight from the loaded words (stage_pack); NULL packs
          // as kPackNull; anything else is checked against the "NullValue" string, then listed
          uint64_t p = kPackNull;
          bool packed = n == kLenNull || stage_pack(kw[j], n, psel[n], &p);
          uint64_t k0 = 0, k1 = 0;
          uint32_t len = 0;
          if (!packed) {
            key_words(k0, k1, len);
            packed = kp_pack_record(k0, k1, len, &p);
          }
          if (packed) {
            L.rec[j * kStageThreads + t] = p;  // (row order; part_tile sorts it)
            h = hash_record_packed(p);
          } else {  // not a digit key: a 16-B record on the overflow list
            h = hash_raw(k0, k1, len);
            stage_sketch(regs, h);
            FreqRec r;
            r.k0 = k0;
            r.k1 = k1 | ((unsigned long long)len << kRecLenShift);
            const unsigned long long k = atomicAdd(ovf_n, 1ull);
            if (k < ovf_cap) ovf[k] = r;
            else atomicOr(flag, 1u);
            ++n_side;
            continue;
          }
        } else {
          uint64_t k0, k1;
          uint32_t len;
          key_words(k0, k1, len);
          h = hash_inline(k0, k1, len);
          rec[j].k0 = k0;
          rec[j].k1 = k1 | ((unsigned long long)len << kRecLenShift);
        }
        bin[j] = (uint32_t)(h >> (64 - b1)) & (nb - 1u);
        stage_sketch(regs, h);
        // one row at a time: interleaving the twelve rows' packing and hashing would need more
        // registers than four waves per SIMD leave (the key words of the later rows are live)
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < kStagePer; ++i) {
        const int64_t row = row0 + i * kStageThreads + t;
        bin[i] = kPartNoBin;
        if (row >= n_rows) continue;
        Key k;
        bool tl;
        if (!make_key(ks, cols, row, k, scratch, tl)) {
          if (tl) too_long = max(too_long, (uint32_t)kMaxLocalKey + 1u);
          continue;
        }
        if (k.len > 15 || k.ptr != nullptr) {
          too_long = max(too_long, k.len > 15 ? k.len : 16u);
          continue;
        }
        if constexpr (!PACK) {
          rec[i].k0 = k.k0;
          rec[i].k1 = k.k1 | ((unsigned long long)k.len << kRecLenShift);
        }
        bin[i] = (uint32_t)(k.hash >> (64 - b1)) & (nb - 1u);
        stage_sketch(regs, k.hash);
      }
    }
    if (too_long) atomicMax(long_key, (unsigned long long)too_long);
#ifdef DQ_STAGE_PROF
    constexpr bool kProf = true;
#else
    constexpr bool kProf = false;
#endif
    // PACK: thread 0 reads `flag` as the tile's room is reserved (its wait is the atomics' wait);
    // the workgroup leaves at the next tile's top
    auto flag_read = [&]() {
      if constexpr (PACK)
        if (t == 0) abort_v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    part_tile<kStagePer, (1 << kStageBinBits), R, (PACK ? kStageSubP : kStageSub16), kProf, DQ_STAGE_WOUT_UNROLL,
              PACK, kStageThreads, decltype(flag_read)>(
        L, rec, bin, nb, 0, out, cap1, fill1, ovf, ovf_n, ovf_cap, flag, staged, nullptr, prof_t_, flag_read);
  }
  if (PACK && n_side) atomicAdd(staged, (unsigned long long)n_side);
#ifdef DQ_STAGE_PROF
  if (t == 0 && blockIdx.x < 4096u) g_stage_blk[blockIdx.x][1] = wall_clock64();
#endif
  lds_barrier();
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// The stage's first half on its own (round 5): every row of the batch becomes its record in ROW
// order -- out[row] -- with no split, so the kernel is a pure stream (the input read once, the
// records written with coalesced stores) that keeps the key loads of many workgroups in flight;
// the level-1 split runs next as dq_freq_part_kernel over the row array (level 1: records of
// 24 per thread in 6144-record LDS rounds).  Measured on one box (125M-row batches, C4): the
// fused stage + level-1 kernel 1.36-1.40 ms, its loads + packing + sketch alone 0.47 ms, with the
// row-order record stores 0.58 ms.  A row that stages nothing (NULL outside a Histogram, a key
// put on the overflow list, a key over 15 bytes) holds a hole: kPackEmpty / length kRecHole,
// which the split drops.  Sketch, long-key flag, overflow list and `staged` (the overflow list's
// share; the split counts the rest) are kept as the fused kernel keeps them.
template <bool ONE_STRING, bool PACK>
__global__ __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(DQ_STAGEP_WAVES))) void dq_freq_stage_rows_kernel(
    FreqKeySpec ks, const DevColumn* __restrict__ cols, int64_t n_rows,
    typename std::conditional<PACK, uint64_t, FreqRec>::type* __restrict__ out, FreqRec* ovf,
    unsigned long long* ovf_n, uint64_t ovf_cap, unsigned int* flag, uint32_t* hll, unsigned long long* long_key,
    unsigned long long* staged) {
  static_assert(ONE_STRING || !PACK, "packed records are staged from one string key column");
  __shared__ uint32_t regs[kHllM];
  __shared__ uint4 psel[16];  // stage_pack's byte selectors by key length
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  if (PACK && t < 16u) psel[t] = make_uint4(stage_pack_sel(t, 0), stage_pack_sel(t, 1), stage_pack_sel(t, 2), stage_pack_sel(t, 3));
  lds_barrier();
  const DevColumn& c0 = cols[ks.key_cols[0]];
  alignas(8) uint8_t scratch[kMaxLocalKey];
  const int64_t n_tiles = (n_rows + kStageTile - 1) / kStageTile;
  uint32_t n_side = 0;  // PACK: this thread's keys put on the overflow list (not digit strings)
  const uint32_t heap_end = ONE_STRING ? __builtin_amdgcn_readfirstlane((uint32_t)uniform_ptr(c0.offsets)[n_rows]) : 0u;
  const uint8_t* vals = static_cast<const uint8_t*>(uniform_ptr(c0.values));
  const __amdgpu_buffer_rsrc_t rs_vals =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vals), 0, (int)heap_end, 0x00020000);
  if (ONE_STRING && heap_end < 16u) {  // (a heap under 16 bytes: key_load16's general path, as a long key)
    if (blockIdx.x == 0 && t == 0) atomicMax(long_key, 16ull);
    return;
  }
  const bool has_validity = uniform_ptr(c0.validity) != nullptr;
  uint32_t pob[kStagePer], poe[kStagePer], vword = 0u;
  constexpr uint32_t kLenNull = 254u, kLenLong = 255u;
  uint32_t kw[kStagePer][4], lens[(kStagePer + 3) / 4], sel = 0u;
  using R = typename std::conditional<PACK, uint64_t, FreqRec>::type;
  auto hole = [&]() -> R {
    if constexpr (PACK) {
      return kPackEmpty;
    } else {
      FreqRec r;
      r.k0 = 0ull;
      r.k1 = (unsigned long long)kRecHole << kRecLenShift;
      return r;
    }
  };
  // PACK: once the overflow list has filled up (a column of keys that are not digit strings) the
  // batch will be rolled back, so a wave stops at its next tile once one of its lanes found the
  // list full (no flag read per tile: the atomic's own return says it)
  bool full = false;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    if constexpr (PACK)
      if (__ballot(full)) break;
    const int64_t row0 = tile * (int64_t)kStageTile;
    uint32_t too_long = 0u;
    if constexpr (ONE_STRING) {
      stage_offsets(c0, n_rows, tile, pob, poe, vword);
      sel = 0u;
#pragma unroll
      for (int j = 0; j < (kStagePer + 3) / 4; ++j) lens[j] = 0u;
#pragma unroll
      for (int j = 0; j < kStagePer; ++j) {
        const int64_t row = row0 + j * kStageThreads + t;
        const uint32_t n = poe[j] - pob[j];
        const bool valid = !has_validity || ((stage_valid_mask(vword, j) >> (t & 63u)) & 1u);
        if (row < n_rows && (valid || ks.null_as_key)) sel |= 1u << j;
        const uint32_t nb8 = (row < n_rows && !valid) ? kLenNull : (n > 15u ? kLenLong : n | (key_shift(pob[j], heap_end) << 4));
        lens[j / 4] |= nb8 << (8 * (j % 4));
      }
#pragma unroll
      for (int j = 0; j < kStageWin; ++j) key_load16(rs_vals, heap_end, pob[j], kw[j]);
#pragma unroll
      for (int j = 0; j < kStagePer; ++j) {
        if (j + kStageWin < kStagePer) key_load16(rs_vals, heap_end, pob[j + kStageWin], kw[j + kStageWin]);
        const int64_t row = row0 + j * kStageThreads + t;
        if (row >= n_rows) continue;
        R r = hole();
        if ((sel >> j) & 1u) {
          uint32_t n = (lens[j / 4] >> (8 * (j % 4))) & 0xFFu;
          if (n == kLenLong) {
            too_long = 16u;
          } else {
            if (n != kLenNull) {
              if (n > 15u) key_shr_bytes(kw[j], n >> 4);  // a key in the heap's last 16 bytes (rare)
              n &= 15u;
            }
            auto key_words = [&](uint64_t& k0, uint64_t& k1, uint32_t& len) {
              if (n == kLenNull) {
                len = 9;
                k0 = kNullK0;
                k1 = kNullK1;
              } else {
                const uint64_t lo = (uint64_t)kw[j][0] | ((uint64_t)kw[j][1] << 32);
                const uint64_t hi = (uint64_t)kw[j][2] | ((uint64_t)kw[j][3] << 32);
                len = n;
                k0 = n >= 8 ? lo : (lo & ((1ull << (8u * n)) - 1ull));
                k1 = n > 8 ? (hi & ((1ull << (8u * (n - 8u))) - 1ull)) : 0ull;
              }
            };
            if constexpr (PACK) {
              uint64_t p = kPackNull;
              bool packed = n == kLenNull || stage_pack(kw[j], n, psel[n], &p);
              uint64_t k0 = 0, k1 = 0;
              uint32_t len = 0;
              if (!packed) {
                key_words(k0, k1, len);
                packed = kp_pack_record(k0, k1, len, &p);
              }
              if (packed) {
                r = p;
                stage_sketch(regs, hash_record_packed(p));
              } else {  // not a digit key: a 16-B record on the overflow list, a hole in the rows
                stage_sketch(regs, hash_raw(k0, k1, len));
                FreqRec o;
                o.k0 = k0;
                o.k1 = k1 | ((unsigned long long)len << kRecLenShift);
                const unsigned long long k = atomicAdd(ovf_n, 1ull);
                if (k < ovf_cap) {
                  ovf[k] = o;
                } else {
                  atomicOr(flag, 1u);
                  full = true;
                }
                ++n_side;
              }
            } else {
              uint64_t k0, k1;
              uint32_t len;
              key_words(k0, k1, len);
              stage_sketch(regs, hash_inline(k0, k1, len));
              r.k0 = k0;
              r.k1 = k1 | ((unsigned long long)len << kRecLenShift);
            }
          }
        }
        out[row] = r;
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < kStagePer; ++i) {
        const int64_t row = row0 + i * kStageThreads + t;
        if (row >= n_rows) continue;
        R r = hole();
        Key k;
        bool tl;
        if (make_key(ks, cols, row, k, scratch, tl)) {
          if (k.len > 15 || k.ptr != nullptr) {
            too_long = max(too_long, k.len > 15 ? k.len : 16u);
          } else {
            if constexpr (!PACK) {
              r.k0 = k.k0;
              r.k1 = k.k1 | ((unsigned long long)k.len << kRecLenShift);
            }
            stage_sketch(regs, k.hash);
          }
        } else if (tl) {
          too_long = max(too_long, (uint32_t)kMaxLocalKey + 1u);
        }
        out[row] = r;
      }
    }
    if (too_long) atomicMax(long_key, (unsigned long long)too_long);
  }
  if (PACK && n_side) atomicAdd(staged, (unsigned long long)n_side);
  lds_barrier();
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// Copy regions (min(fill, cap) records each) to out[prefix[r] ..]: the partitioned staging
// laid out contiguously again for the sort path (rare: skew, or a table of few slices).
// (R = uint64_t: packed digit records, written out as 16-B records.)
template <typename R>
__global__ __launch_bounds__(kBlock) void dq_freq_compact_kernel(const R* __restrict__ in,
                                                                 const unsigned long long* __restrict__ fill,
                                                                 uint64_t cap, const unsigned long long* __restrict__ prefix,
                                                                 FreqRec* __restrict__ out) {
  const uint64_t r = blockIdx.y;
  const unsigned long long f = fill[r];
  const uint64_t have = f < cap ? f : cap;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < have; i += (uint64_t)gridDim.x * kBlock)
    out[prefix[r] + i] = rec_raw(in[r * cap + i]);
}

// Aggregate slice region b (records b * cap .. + min(fill[b], cap)) as its slice's owner.
// tr: see AggTrack (table_empty only).  512 threads: more waves per CU than three 256-thread
// slices' LDS images would give.
#ifndef DQ_AGG_THREADS
#define DQ_AGG_THREADS 512
#endif
constexpr int kAggRegionThreads = DQ_AGG_THREADS;
#ifndef DQ_AGG_WAVES
#define DQ_AGG_WAVES 4
#endif
__global__ __launch_bounds__(kAggRegionThreads) __attribute__((amdgpu_waves_per_eu(DQ_AGG_WAVES))) void dq_freq_agg_region_kernel(FreqTable T, const FreqRec* __restrict__ recs,
                                                                    const unsigned long long* __restrict__ fill,
                                                                    uint64_t cap, uint64_t n_slices, int table_empty,
                                                                    FreqRec* retry, unsigned long long* n_retry,
                                                                    unsigned long long* new_groups, AggTrack tr) {
  __shared__ AggLds L;
  const bool track = tr.hist != nullptr;
  if (track) {
    for (int i = threadIdx.x; i < kAggLdsHist; i += kAggRegionThreads) L.hist[i] = 0u;
    __syncthreads();
  }
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    const uint64_t r0 = b * cap;
    const unsigned long long f = fill[b];
    const uint64_t r1 = r0 + (f < cap ? f : cap);
    // the item's records are touched (one dword per 128-B line, one per thread) before the LDS
    // image is initialised, so their HBM latency overlaps the init and the barrier and the
    // item's loads then hit L2; one register, consumed after the item
    uint32_t touch = 0u;
    {
      const uint64_t i = r0 + (uint64_t)threadIdx.x * 8u;
      if (i < r1) touch = *reinterpret_cast<const uint32_t*>(recs + i);
    }
    if (r1 == r0) {
      if (tr.cmp.slots) {
        if (threadIdx.x == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        FreqSlot* slice = T.slots + (b << kFreqSliceLog);
        for (uint32_t s = threadIdx.x; s < (uint32_t)kFreqSliceSlots; s += kAggRegionThreads) slice[s] = FreqSlot{0ull, 0ull, 0ull, 0ull};
      }
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = 0u;
    } else {
      agg_item<kAggRegionThreads, true>(L, T, recs, r0, r1, b, true, table_empty, retry, n_retry, new_groups,
                                        track || tr.write_all || tr.cmp.slots ? &tr : nullptr);
    }
    asm volatile("" ::"v"(touch));
  }
  if (track) {
    __syncthreads();
    for (int i = threadIdx.x; i < kAggLdsHist; i += kAggRegionThreads)
      if (L.hist[i]) atomicAdd(&tr.hist[i], (unsigned long long)L.hist[i]);
  }
}

// The owner aggregation of slice regions of packed digit records (dq_keypack.h).  The LDS image
// holds one word per slot -- the packed key -- so a slot is claimed AND published by one CAS
// (no separate key publish, no busy state), and a record is counted with at most one CAS per
// probe plus one add.  The image is unpacked into the table's key bytes once per group, at
// write-out.  Same contract as dq_freq_agg_region_kernel (owner only; tr as there); a slice whose
// keys overflow the image returns all of its records to the retry list as 16-B records.
struct AggLdsP {
  unsigned long long K[kFreqSliceSlots];
  uint32_t C[kFreqSliceSlots];
  uint32_t wsum[4];
  int overflow;
  uint32_t fresh;
  uint32_t cmax;
  unsigned long long retry_base;
  unsigned long long cbase;
  uint32_t hist[kAggLdsHist];
};

// Count packed record p from LDS slot s on (probe `first` of its run); false if the image is full.
__device__ inline bool lds_count_packed(unsigned long long* K, uint32_t* C, uint64_t p, uint32_t s, uint32_t first = 0) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  for (uint32_t probe = first; probe < S; ++probe) {
    const unsigned long long c = atomicCAS(&K[s], kPackEmpty, (unsigned long long)p);
    if (c == kPackEmpty || c == p) {
      atomicAdd(&C[s], 1u);
      return true;
    }
    s = (s + 1) & (S - 1);
  }
  return false;
}


#ifndef DQ_AGGP_BATCH
#define DQ_AGGP_BATCH 4
#endif
constexpr int kAggPBatch = DQ_AGGP_BATCH;  // packed records per thread loaded together

#ifndef DQ_AGGP_WAVES
#define DQ_AGGP_WAVES 6  // (80 VGPRs, no spill; asking for 8 left the compiler at 84 VGPRs = 5 waves once
                         // the compacted write-out was added -- round 5's build reached 6 at 77)
#endif
#ifndef DQ_AGGP_THREADS
#define DQ_AGGP_THREADS 256
#endif
constexpr int kAggPThreads = DQ_AGGP_THREADS;
__global__ __launch_bounds__(kAggPThreads) __attribute__((amdgpu_waves_per_eu(DQ_AGGP_WAVES))) void dq_freq_agg_packed_kernel(
    FreqTable T, const uint64_t* __restrict__ recs, const unsigned long long* __restrict__ fill, uint64_t cap,
    uint64_t n_slices, int table_empty, FreqRec* retry, unsigned long long* n_retry, unsigned long long* new_groups,
    AggTrack tr) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kAggPThreads;
  __shared__ AggLdsP L;
  const bool track = tr.hist != nullptr;
  const bool compact = tr.cmp.slots != nullptr;  // (an empty table only)
  if (track) {
    for (int i = threadIdx.x; i < kAggLdsHist; i += NT) L.hist[i] = 0u;
    lds_barrier();
  }
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    const uint64_t r0 = b * cap;
    const unsigned long long f = fill[b];
    const uint64_t r1 = r0 + (f < cap ? f : cap);
    FreqSlot* slice = T.slots + (b << kFreqSliceLog);
    // touch the item's records (one dword per 128-B line) before the image is initialised, so
    // their HBM latency overlaps the init and the barrier (as dq_freq_agg_region_kernel)
    uint32_t touch = 0u;
    {
      const uint64_t i = r0 + (uint64_t)threadIdx.x * 16u;
      if (i < r1) touch = *reinterpret_cast<const uint32_t*>(recs + i);
    }
    if (r1 == r0) {
      if (compact) {
        if (threadIdx.x == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        for (uint32_t s = threadIdx.x; s < S; s += NT) slice[s] = FreqSlot{0ull, 0ull, 0ull, 0ull};
      }
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = 0u;
      asm volatile("" ::"v"(touch));
      continue;
    }
    for (uint32_t s = threadIdx.x; s < S; s += NT) {
      unsigned long long k = kPackEmpty;
      if (!table_empty) {
        const FreqSlot e = slice[s];
        const uint32_t len = (uint32_t)(e.ctrl & kLenMask);
        if (e.ctrl & kReady) {
          uint64_t p;
          k = !(e.ctrl & kHeapKey) && len <= 15 && kp_pack_record(e.k0, e.k1, len, &p) ? p : kPackForeign;
        }
      }
      L.K[s] = k;
      L.C[s] = 0u;
    }
    if (threadIdx.x == 0) {
      L.overflow = 0;
      L.fresh = 0u;
      L.cmax = 0u;
    }
    lds_barrier();
    uint64_t rb[kAggPBatch];
    for (uint64_t base = r0; base < r1; base += (uint64_t)NT * kAggPBatch) {
#pragma unroll
      for (int j = 0; j < kAggPBatch; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i < r1) rb[j] = recs[i];
      }
      // every record's first probe is issued before any result is looked at (independent LDS
      // round trips); at the table's ~0.4 load most records are counted there
      uint32_t sl[kAggPBatch];
      unsigned long long cv[kAggPBatch];
#pragma unroll
      for (int j = 0; j < kAggPBatch; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        sl[j] = (uint32_t)hash_record_packed(rb[j]) & (S - 1);
        cv[j] = i < r1 ? atomicCAS(&L.K[sl[j]], kPackEmpty, (unsigned long long)rb[j]) : 0ull;
      }
#pragma unroll
      for (int j = 0; j < kAggPBatch; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i >= r1) continue;
        if (cv[j] == kPackEmpty || cv[j] == rb[j]) atomicAdd(&L.C[sl[j]], 1u);
        else if (!lds_count_packed(L.K, L.C, rb[j], (sl[j] + 1) & (S - 1), 1)) L.overflow = 1;
      }
    }
    lds_barrier();
    // The slice is written as 16-byte halves, one per lane, so each store instruction covers a
    // contiguous 1 KiB (whole 128-byte lines): q = 2 * slot + half, half 0 = {ctrl, count},
    // half 1 = {k0, k1}.
    ulonglong2* halves = reinterpret_cast<ulonglong2*>(slice);
    if (L.overflow) {  // the slice is full: leave it untouched, hand the region's rows back
      if (threadIdx.x == 0) L.retry_base = atomicAdd(n_retry, (unsigned long long)(r1 - r0));
      lds_barrier();
      for (uint64_t i = r0 + threadIdx.x; i < r1; i += NT) retry[L.retry_base + (i - r0)] = rec_raw(recs[i]);
      if (compact) {
        if (threadIdx.x == 0) tr.cmp.num[b] = 0u;  // (the slice starts out empty)
      } else if (tr.write_all) {  // (the table was not cleared: the slice starts out empty)
        for (uint32_t q = threadIdx.x; q < 2 * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      }
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = 0xFFFFFFFFu;  // unknown: never skipped
    } else if (compact) {
      // Only the occupied slots are written (C4: ~0.37 of the slice), in slot order, at a place
      // reserved with one atomic per slice; the slice's occupancy bitmap (256 B) lets
      // dq_freq_expand_kernel rebuild the slot image exactly when a probing operation needs it.
      static_assert(S == 8u * NT, "eight slots per thread");
      const uint32_t t = threadIdx.x;
      const uint4 c0 = *reinterpret_cast<const uint4*>(&L.C[8u * t]);
      const uint4 c1 = *reinterpret_cast<const uint4*>(&L.C[8u * t + 4u]);
      const uint32_t cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      uint32_t occ = 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!cs[j]) continue;
        occ |= 1u << j;
        if (track || tr.smax) {
          atomicMax(&L.cmax, cs[j]);
          if (track) {
            if (cs[j] < (uint32_t)kAggLdsHist) atomicAdd(&L.hist[cs[j]], 1u);
            else if (cs[j] < (uint32_t)kFreqHist) atomicAdd(&tr.hist[cs[j]], 1ull);
            else {
              const unsigned long long i = atomicAdd(tr.n_big, 1ull);
              if (i < tr.big_cap) tr.big[i] = cs[j];
            }
          }
        }
      }
      uint32_t tot;
      const uint32_t k = block_prefix<NT>((uint32_t)__builtin_popcount(occ), L.wsum, &tot);
      tr.cmp.bits[(b << 8) + t] = (uint8_t)occ;
      if (t == 0) {
        const unsigned long long at = atomicAdd(tr.cmp.cursor, (unsigned long long)tot);
        L.cbase = at;
        tr.cmp.base[b] = at;
        tr.cmp.num[b] = tot;
        if (tot) atomicAdd(new_groups, (unsigned long long)tot);
      }
      lds_barrier();
      // each thread writes its own groups (~3 at C4's load), whole 32-B records at consecutive
      // positions: every store fills whole sectors, and the wave's stores fill whole lines
      FreqSlot* out = tr.cmp.slots + L.cbase + k;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!(occ & (1u << j))) continue;
        const uint64_t p = L.K[8u * t + (uint32_t)j];
        uint64_t k0, k1;
        uint32_t len;
        kp_unpack(p, &k0, &k1, &len);
        *out++ = FreqSlot{((unsigned long long)tag_of(hash_record_packed(p)) << 32) | kReady | len,
                          (unsigned long long)L.C[8u * t + (uint32_t)j], k0, k1};  // (re-read: registers)
      }
      if (tr.smax && t == 0) tr.smax[b] = L.cmax;
    } else {
      for (uint32_t q = threadIdx.x; q < 2 * S; q += NT) {
        const uint32_t s = q >> 1;
        const bool hi = (q & 1u) != 0u;
        const uint32_t c = L.C[s];
        bool is_new = false;
        if (!c) {
          // (an empty slot is ctrl = 0 and count = 0; its key half is never read)
          if (tr.write_all) halves[q] = ulonglong2{0ull, 0ull};
        } else {
          const bool existing = !table_empty && (slice[s].ctrl & kReady);
          const uint64_t p = L.K[s];
          if (!hi) {
            if (track || tr.smax) {
              atomicMax(&L.cmax, c);
              if (track) {
                if (c < (uint32_t)kAggLdsHist) {
                  atomicAdd(&L.hist[c], 1u);
                } else if (c < (uint32_t)kFreqHist) {
                  atomicAdd(&tr.hist[c], 1ull);
                } else {
                  const unsigned long long i = atomicAdd(tr.n_big, 1ull);
                  if (i < tr.big_cap) tr.big[i] = c;
                }
              }
            }
            if (existing) {
              slice[s].count += c;
            } else {
              const uint32_t len = p == kPackNull ? 9u : (uint32_t)(p >> 60);
              halves[q] = ulonglong2{((unsigned long long)tag_of(hash_record_packed(p)) << 32) | kReady | len,
                                     (unsigned long long)c};
              is_new = true;
            }
          } else if (!existing) {
            uint64_t k0, k1;
            uint32_t len;
            kp_unpack(p, &k0, &k1, &len);
            halves[q] = ulonglong2{k0, k1};
          }
        }
        const uint64_t nb = __ballot(is_new);  // one LDS add per wave, not one per new group
        if (nb && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(nb)) atomicAdd(&L.fresh, (uint32_t)__popcll(nb));
      }
      lds_barrier();
      if (threadIdx.x == 0 && L.fresh) atomicAdd(new_groups, (unsigned long long)L.fresh);
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = L.cmax;
    }
    lds_barrier();  // LDS is reused by the next slice
    asm volatile("" ::"v"(touch));
  }
  if (track) {
    lds_barrier();
    for (int i = threadIdx.x; i < kAggLdsHist; i += NT)
      if (L.hist[i]) atomicAdd(&tr.hist[i], (unsigned long long)L.hist[i]);
  }
}

// ---- Long and multi-column keys on the partition path (round 6).  The reference groups any key
// in one hash aggregate (GroupingAnalyzers.scala:67-71): isUnique / isPrimaryKey / hasUniqueness
// (Check.scala:140-230) on UUID-like ids or composite keys.  Such a key does not fit a 16-byte
// record, so the stage copies its bytes into the table's key heap once and stages a HashRec
// {table hash, heap reference}; the records travel the same two-level split as the other record
// forms, and each slice is aggregated in LDS by hash (dq_freq_agg_hashed_kernel), with every
// record of a hash group compared byte for byte against the group's first record, so the
// grouping is exact: a slice holding two different keys of one 64-bit hash (about 0.03 such
// pairs per 1e9 distinct keys) hands its records to the global inserts, which compare keys.

// Exact heap bytes the hashed stage appends for rows [0, n_rows): sum of 8-aligned key lengths.
// The encoded key length of `row` (make_key's encoding) in *n; false when the row is no key.
__device__ inline bool key_len_of(const FreqKeySpec& ks, const DevColumn* cols, int64_t row, uint32_t* n) {
  uint32_t m = 0;
  for (int i = 0; i < ks.n_keys; ++i) {
    const DevColumn& c = cols[ks.key_cols[i]];
    if (!col_valid(c, row)) {
      if (ks.n_keys == 1 && ks.null_as_key) {  // "NullValue" / the empty key
        *n = c.type == DQ_T_UTF8 ? 9u : 0u;
        return true;
      }
      return false;
    }
    if (c.type == DQ_T_UTF8) m += (uint32_t)(c.offsets[row + 1] - c.offsets[row]) + (ks.n_keys > 1 ? 4u : 0u);
    else m += (uint32_t)width_of(c.type);
  }
  *n = m;
  return true;
}

__global__ __launch_bounds__(kBlock) void dq_freq_key_bytes_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                   int64_t n_rows, unsigned long long* out) {
  unsigned long long local = 0;
  for (int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x; row < n_rows; row += (int64_t)gridDim.x * kBlock) {
    uint32_t n;
    if (key_len_of(ks, cols, row, &n)) local += ((unsigned long long)n + 7ull) & ~7ull;
  }
  for (int d = 32; d >= 1; d >>= 1) local += __shfl_xor(local, d, 64);
  if ((threadIdx.x & 63u) == 0 && local) atomicAdd(out, local);
}

// xxh64_any(p, len, seed) of a key held in registers: kw[i] = its bytes 8i .. 8i + 7 (little
// endian, zero past len), len <= 8 * MW.  The same stripes, words and tail as xxh64_any.
template <int MW>
__device__ inline uint64_t xxh64_words(const uint64_t (&kw)[MW], uint32_t len, uint64_t seed) {
  const uint32_t stripes = len >> 5, full = len >> 3;
  uint64_t h;
  if (stripes) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
#pragma unroll
    for (int st = 0; st < MW / 4; ++st) {
      if ((uint32_t)st < stripes) {
        v1 = xxh_round(v1, kw[4 * st]);
        v2 = xxh_round(v2, kw[4 * st + 1]);
        v3 = xxh_round(v3, kw[4 * st + 2]);
        v4 = xxh_round(v4, kw[4 * st + 3]);
      }
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h ^= xxh_round(0, v1); h = h * kP1 + kP4;
    h ^= xxh_round(0, v2); h = h * kP1 + kP4;
    h ^= xxh_round(0, v3); h = h * kP1 + kP4;
    h ^= xxh_round(0, v4); h = h * kP1 + kP4;
  } else {
    h = seed + kP5;
  }
  h += (uint64_t)len;
  uint64_t tail = 0ull;
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    if ((uint32_t)i >= 4u * stripes && (uint32_t)i < full) {
      h ^= xxh_round(0, kw[i]);
      h = rotl64(h, 27) * kP1 + kP4;
    }
    if ((uint32_t)i == full) tail = kw[i];
  }
  if (len & 7u) {
    h ^= tail * kP5;
    h = rotl64(h, 11) * kP1;
  }
  return xxh_avalanche(h);
}

// hash_long of a key held in registers (kw as for xxh64_words).
template <int MW>
__device__ inline uint64_t hash_long_words(const uint64_t (&kw)[MW], uint32_t len) {
  if constexpr (MW >= 5) {
    if (len == kUuidLen) {
      uint32_t w[9];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w[2 * i] = (uint32_t)kw[i];
        w[2 * i + 1] = (uint32_t)(kw[i] >> 32);
      }
      w[8] = (uint32_t)kw[4];
      uint64_t lo, hi;
      if (uuid_pack(w, &lo, &hi)) return hash_uuid(lo, hi);
    }
  }
  return xxh64_words<MW>(kw, len, 42);
}

// One row of the hashed stage the general way (make_key): its key bytes to heap + off, its
// record in *r; the heap bytes it used (0 when the row is no key).  Multi-column keys, NULLs
// and keys longer than the register path's 48 bytes.
__device__ __noinline__ uint32_t stage_hashed_row(const FreqKeySpec& ks, const DevColumn* cols, int64_t row,
                                                  const FreqTable& T, unsigned long long off, HashRec* r,
                                                  bool* tl) {
  alignas(8) uint8_t scratch[kMaxLocalKey];
  Key k;
  r->h = 0ull;
  r->ref = kHashHole;
  if (!make_key(ks, cols, row, k, scratch, *tl)) return 0u;
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(T.heap + off);
  if (k.ptr == nullptr) {  // an inline key (<= 16 bytes) in k0 / k1, zero padded
    if (k.len) dst[0] = k.k0;
    if (k.len > 8) dst[1] = k.k1;
  } else {
    for (uint32_t i = 0; i < k.len; i += 8) dst[i >> 3] = ld_partial(k.ptr + i, k.len - i < 8 ? k.len - i : 8);
  }
  r->h = k.hash;
  r->ref = (off << 24) | k.len;
  return (k.len + 7u) & ~7u;
}

// A multi-column key (make_key's encoding: fixed-width values' little-endian bytes, strings as
// a u32 length + their bytes) built in registers, kw[i] = bytes 8i .. 8i + 7, zero past *n.
// False when a column is NULL (no key) or the key is longer than 8 * MW bytes (*n = 0: the
// caller takes make_key).
template <int MW>
__device__ inline bool key_words(const FreqKeySpec& ks, const DevColumn* cols, int64_t row, uint64_t (&kw)[MW],
                                 uint32_t* n_out) {
  uint32_t n = 0;
#pragma unroll
  for (int i = 0; i < MW; ++i) kw[i] = 0ull;
  *n_out = 0u;
  // v's low nb (<= 8) bytes appended at byte n
  auto put = [&](uint64_t v, uint32_t nb) {
    if (nb < 8u) v &= (1ull << (8u * nb)) - 1ull;
    const uint32_t wi = n >> 3, sh = 8u * (n & 7u);
#pragma unroll
    for (int i = 0; i < MW; ++i) {
      if ((uint32_t)i == wi) kw[i] |= v << sh;
      if (sh && (uint32_t)i == wi + 1u) kw[i] |= v >> (64u - sh);
    }
    n += nb;
  };
  for (int c = 0; c < ks.n_keys; ++c) {
    const DevColumn& col = cols[ks.key_cols[c]];
    if (!col_valid(col, row)) return false;
    if (col.type == DQ_T_UTF8) {
      const int32_t b = col.offsets[row], e = col.offsets[row + 1];
      const uint32_t sl = (uint32_t)(e - b);
      if (n + 4u + sl > 8u * MW) return false;
      put(sl, 4u);
      const uint8_t* p = static_cast<const uint8_t*>(col.values) + b;
      for (uint32_t i = 0; i < sl; i += 8u) put(ld_partial(p + i, sl - i < 8u ? sl - i : 8u), sl - i < 8u ? sl - i : 8u);
    } else {
      const uint32_t w = (uint32_t)width_of(col.type);
      if (n + w > 8u * MW) return false;
      put(fixed_bits(col, row), w);
    }
  }
  *n_out = n;
  return true;
}

// One tile = kHashTile rows; wave w takes rows row0 + w * 64 * kHashPer + 64 j + lane (j <
// kHashPer), so the heap, like the records, is in row order: the rows' key lengths first (one
// wave prefix per j), a workgroup prefix over the waves, ONE heap reservation per tile (a
// reservation per wave put 15M atomics on one address per 1e9 rows: the stage ran at 0.5 TB/s),
// then each group of 64 rows copies its keys to consecutive heap bytes.  A single string key
// column's keys of 17..48 bytes (UUIDs) take the register path: kHashG rows' offsets, then
// their aligned words, loaded together; the key realigned in registers, hashed (xxh64_words)
// and stored from them.  Every other row takes stage_hashed_row.
constexpr int kHashPer = 16;
constexpr int kHashG = 2;      // rows whose words are in flight together
constexpr int kHashWords = 6;  // register path: keys of <= 48 bytes
constexpr uint32_t kHashTile = (uint32_t)kBlock * kHashPer;
template <bool ONE_STRING>
__global__ __launch_bounds__(kBlock) void dq_freq_stage_hashed_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                      int64_t n_rows, HashRec* __restrict__ out, FreqTable T,
                                                                      uint32_t* hll, unsigned long long* too_long,
                                                                      unsigned long long* staged,
                                                                      unsigned long long* max_len) {
  static_assert(kBlock / 64 <= 4, "four waves");
  __shared__ uint32_t regs[kHllM];
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long tile_base;
  for (uint32_t i = threadIdx.x; i < (uint32_t)kHllM; i += kBlock) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  __syncthreads();
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  constexpr bool one_string = ONE_STRING;  // (the host: ks.n_keys == 1 and a utf8 column)
  const DevColumn c0 = cols[ks.key_cols[0]];
  const uint8_t* bytes = static_cast<const uint8_t*>(c0.values);
  unsigned long long n_keys = 0;
  uint32_t longest = 0u;
  bool tl_any = false;
  const int64_t n_tiles = (n_rows + kHashTile - 1) / kHashTile;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t rw = tile * (int64_t)kHashTile + (int64_t)wave * 64 * kHashPer + lane;  // row of j = 0
    uint32_t off[kHashPer];  // heap offset of row j within the wave's run
    uint32_t run = 0u;
#pragma unroll
    for (int j = 0; j < kHashPer; ++j) {
      const int64_t row = rw + 64 * j;
      uint32_t n = 0u, m8 = 0u;
      if (row < n_rows && key_len_of(ks, cols, row, &n)) m8 = (n + 7u) & ~7u;
      uint32_t x = m8;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
      }
      off[j] = run + x - m8;
      run += __shfl(x, 63, 64);
    }
    if (lane == 0u) wsum[wave] = run;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      before += (uint32_t)w < wave ? wsum[w] : 0u;
      total += wsum[w];
    }
    if (t == 0) tile_base = total ? atomicAdd(T.heap_used, (unsigned long long)total) : 0ull;
    __syncthreads();
    const unsigned long long base = tile_base + before;
    const bool room = tile_base + total <= T.heap_cap;  // (the host sized the heap: never false)
    if (!room && t == 0) atomicOr(T.overflow, 2u);
#pragma unroll
    for (int g = 0; g < kHashPer; g += kHashG) {
      int32_t ob[kHashG], oe[kHashG];
      bool fast[kHashG];
#pragma unroll
      for (int q = 0; q < kHashG; ++q) {
        const int64_t row = rw + 64 * (g + q);
        ob[q] = oe[q] = 0;
        fast[q] = false;
        if (one_string && row < n_rows && col_valid(c0, row)) {
          ob[q] = c0.offsets[row];
          oe[q] = c0.offsets[row + 1];
          const uint32_t n = (uint32_t)(oe[q] - ob[q]);
          fast[q] = n > 16u && n <= 8u * kHashWords;
        }
      }
      uint64_t w[kHashG][kHashWords + 1];
#pragma unroll
      for (int q = 0; q < kHashG; ++q) {
        const uintptr_t a = (uintptr_t)(bytes + ob[q]);
        const uint64_t* src = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
        const uint32_t span = (uint32_t)(a & 7) + (uint32_t)(oe[q] - ob[q]);
#pragma unroll
        for (int i = 0; i <= kHashWords; ++i) w[q][i] = fast[q] && 8u * (uint32_t)i < span ? src[i] : 0ull;
      }
#pragma unroll
      for (int q = 0; q < kHashG; ++q) {
        const int j = g + q;
        const int64_t row = rw + 64 * j;
        if (row >= n_rows) continue;
        const unsigned long long at = base + off[j];
        HashRec r;
        uint64_t kwm[kHashWords];
        uint32_t nm = 0u;
        if (fast[q] && room) {
          const uint32_t n = (uint32_t)(oe[q] - ob[q]);
          const uint32_t sh = 8u * (uint32_t)(((uintptr_t)(bytes + ob[q])) & 7);
          uint64_t kw[kHashWords];
#pragma unroll
          for (int i = 0; i < kHashWords; ++i) {
            uint64_t v = sh ? (w[q][i] >> sh) | (w[q][i + 1] << (64u - sh)) : w[q][i];
            const int rem = (int)n - 8 * i;  // key bytes from word i on
            if (rem <= 0) v = 0ull;
            else if (rem < 8) v &= (1ull << (8 * rem)) - 1ull;
            kw[i] = v;
          }
          unsigned long long* dst = reinterpret_cast<unsigned long long*>(T.heap + at);
#pragma unroll
          for (int i = 0; i < kHashWords; ++i)
            if (8u * (uint32_t)i < n) dst[i] = kw[i];
          r.h = hash_long_words<kHashWords>(kw, n);
          r.ref = (at << 24) | n;
          longest = max(longest, n);
        } else if (!ONE_STRING && room && key_words<kHashWords>(ks, cols, row, kwm, &nm) && nm) {
          // a multi-column key in registers (make_key's bytes without its scratch copy)
          unsigned long long* dst = reinterpret_cast<unsigned long long*>(T.heap + at);
#pragma unroll
          for (int i = 0; i < kHashWords; ++i)
            if (8u * (uint32_t)i < nm) dst[i] = kwm[i];
          r.h = nm <= 16u ? hash_inline(kwm[0], kwm[1], nm) : hash_long_words<kHashWords>(kwm, nm);
          r.ref = (at << 24) | nm;
          longest = max(longest, nm);
        } else {
          bool tl = false;
          if (room) stage_hashed_row(ks, cols, row, T, at, &r, &tl);
          else { r.h = 0ull; r.ref = kHashHole; }
          tl_any |= tl;
          if (r.ref != kHashHole) longest = max(longest, (uint32_t)(r.ref & kLenMask));
        }
        if (r.ref != kHashHole) {
          stage_sketch(regs, r.h);
          ++n_keys;
        }
        out[row] = r;
      }
    }
    __syncthreads();  // (wsum and tile_base are rewritten by the next tile)
  }
  for (int d = 32; d >= 1; d >>= 1) n_keys += __shfl_xor(n_keys, d, 64);
  if (staged && lane == 0u && n_keys) atomicAdd(staged, n_keys);
  if (max_len && longest) atomicMax(max_len, (unsigned long long)longest);
  if (tl_any) atomicMax(too_long, (unsigned long long)kMaxLocalKey + 1ull);
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kBlock)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// The hashed stage of a multi-column key (round 6): dq_freq_stage_hashed_kernel<false>'s
// unrolled 16-row body held 251 VGPRs (two waves per SIMD) and ran 9.5 ms per 125M (int64, utf8)
// rows.  Here the same tile layout (heap and records in row order, one heap reservation per
// tile) with rolled loops: the rows' heap offsets wait in LDS between the length pass and the
// copy pass, so a thread holds one row's key at a time.
__global__ __launch_bounds__(kBlock) void dq_freq_stage_hashed_multi_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                            int64_t n_rows, HashRec* __restrict__ out,
                                                                            FreqTable T, uint32_t* hll,
                                                                            unsigned long long* too_long,
                                                                            unsigned long long* staged,
                                                                            unsigned long long* max_len) {
  static_assert(kBlock / 64 <= 4, "four waves");
  __shared__ uint32_t regs[kHllM];
  __shared__ uint32_t offs[kHashPer][kBlock];
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long tile_base;
  for (uint32_t i = threadIdx.x; i < (uint32_t)kHllM; i += kBlock) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  __syncthreads();
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  unsigned long long n_keys = 0;
  uint32_t longest = 0u;
  bool tl_any = false;
  const int64_t n_tiles = (n_rows + kHashTile - 1) / kHashTile;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t rw = tile * (int64_t)kHashTile + (int64_t)wave * 64 * kHashPer + lane;  // row of j = 0
    uint32_t run = 0u;
#pragma unroll 1
    for (int j = 0; j < kHashPer; ++j) {
      const int64_t row = rw + 64 * j;
      uint32_t n = 0u, m8 = 0u;
      if (row < n_rows && key_len_of(ks, cols, row, &n)) m8 = (n + 7u) & ~7u;
      uint32_t x = m8;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
      }
      offs[j][t] = run + x - m8;
      run += __shfl(x, 63, 64);
    }
    if (lane == 0u) wsum[wave] = run;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      before += (uint32_t)w < wave ? wsum[w] : 0u;
      total += wsum[w];
    }
    if (t == 0) tile_base = total ? atomicAdd(T.heap_used, (unsigned long long)total) : 0ull;
    __syncthreads();
    const unsigned long long base = tile_base + before;
    const bool room = tile_base + total <= T.heap_cap;  // (the host sized the heap: never false)
    if (!room && t == 0) atomicOr(T.overflow, 2u);
#pragma unroll 1
    for (int j = 0; j < kHashPer; ++j) {
      const int64_t row = rw + 64 * j;
      if (row >= n_rows) break;
      const unsigned long long at = base + offs[j][t];
      HashRec r;
      uint64_t kw[kHashWords];
      uint32_t nm = 0u;
      if (room && key_words<kHashWords>(ks, cols, row, kw, &nm) && nm) {
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(T.heap + at);
#pragma unroll
        for (int i = 0; i < kHashWords; ++i)
          if (8u * (uint32_t)i < nm) dst[i] = kw[i];
        r.h = nm <= 16u ? hash_inline(kw[0], kw[1], nm) : hash_long_words<kHashWords>(kw, nm);
        r.ref = (at << 24) | nm;
        longest = max(longest, nm);
      } else {
        bool tl = false;
        if (room) stage_hashed_row(ks, cols, row, T, at, &r, &tl);
        else { r.h = 0ull; r.ref = kHashHole; }
        tl_any |= tl;
        if (r.ref != kHashHole) longest = max(longest, (uint32_t)(r.ref & kLenMask));
      }
      if (r.ref != kHashHole) {
        stage_sketch(regs, r.h);
        ++n_keys;
      }
      out[row] = r;
    }
    __syncthreads();  // (offs, wsum and tile_base are rewritten by the next tile)
  }
  for (int d = 32; d >= 1; d >>= 1) n_keys += __shfl_xor(n_keys, d, 64);
  if (staged && lane == 0u && n_keys) atomicAdd(staged, n_keys);
  if (max_len && longest) atomicMax(max_len, (unsigned long long)longest);
  if (tl_any) atomicMax(too_long, (unsigned long long)kMaxLocalKey + 1ull);
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kBlock)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// The key of a hashed record, its bytes read from (and, when long, left in) T's heap.
__device__ inline Key hashed_key(const FreqTable& T, const FreqRec& r) {
  Key k;
  k.len = (uint32_t)(r.k1 & kLenMask);
  k.hash = r.k0;
  const uint8_t* p = T.heap + (r.k1 >> 24);
  k.k0 = k.k1 = 0ull;
  k.ptr = nullptr;
  if (k.len > 16) {
    k.ptr = p;
  } else {
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(p);
    if (k.len) k.k0 = w[0];
    if (k.len > 8) k.k1 = w[1];
  }
  return k;
}

// Two heap keys (8-byte aligned, zero padded) equal byte for byte.
__device__ inline bool heap_refs_equal(const uint8_t* heap, unsigned long long ra, unsigned long long rb) {
  if (ra == rb) return true;
  if ((ra & kLenMask) != (rb & kLenMask)) return false;
  const uint32_t words = (uint32_t)(((ra & kLenMask) + 7ull) >> 3);
  const unsigned long long* a = reinterpret_cast<const unsigned long long*>(heap + (ra >> 24));
  const unsigned long long* b = reinterpret_cast<const unsigned long long*>(heap + (rb >> 24));
  for (uint32_t i = 0; i < words; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// The owner aggregation of slice regions of hashed records into a FRESH table.  LDS image: the
// hash (0 kept as 1), the reference of the group's first record, the count.  A workgroup takes
// a region's records kAggHPer per thread at a time, all loaded together: they are counted by hash
// (one CAS per probe, the slot remembered), then -- after a barrier, when every group's first
// reference is in place -- each record that joined an existing hash group is compared with that
// group's first record byte for byte, kAggHCmp records' key words loaded together (round 6's first
// build compared word by word, one dependent heap read after another: 97 ms per 1e9 UUIDs).  A full image
// or a mismatch (two keys of one hash) hands the slice's records to the retry list; the caller
// inserts them globally.  Write-out as the packed aggregation: the slot image, or (tr.cmp) the
// occupied slots only; keys of <= 16 bytes inline, longer ones referring to their heap bytes.
constexpr int kAggHThreads = 256;
constexpr int kAggHPer = 16;    // records per thread per chunk
constexpr int kAggHCmp = 2;     // joined records compared together
constexpr int kAggHWords = 6;   // key words loaded unconditionally (keys of <= 48 bytes: one round)
static_assert(kAggHWords % 2 == 0, "key words in 16-byte pairs");
typedef unsigned long long u64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));  // (8-byte aligned pair)
struct AggLdsH {
  unsigned long long K[kFreqSliceSlots];
  unsigned long long R[kFreqSliceSlots];
  uint32_t C[kFreqSliceSlots];
  uint32_t wsum[4];
  int overflow;
  uint32_t fresh;
  uint32_t cmax;
  unsigned long long retry_base;
  unsigned long long cbase;
  uint32_t hist[kAggLdsHist];
};

__device__ inline uint32_t lds_find_hash(const unsigned long long* K, unsigned long long kk, uint32_t s) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  for (uint32_t probe = 0; probe < S; ++probe) {
    if (K[s] == kk) return s;
    s = (s + 1u) & (S - 1u);
  }
  return S;
}

__global__ __launch_bounds__(kAggHThreads) __attribute__((amdgpu_waves_per_eu(3))) void dq_freq_agg_hashed_kernel(FreqTable T, const HashRec* __restrict__ recs,
                                                                          const unsigned long long* __restrict__ fill,
                                                                          uint64_t cap, uint64_t n_slices, FreqRec* retry,
                                                                          unsigned long long* n_retry,
                                                                          unsigned long long* new_groups, AggTrack tr) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kAggHThreads;
  constexpr uint32_t kChunk = (uint32_t)kAggHPer * NT;  // records per round
  __shared__ AggLdsH L;
  const bool track = tr.hist != nullptr;
  const bool compact = tr.cmp.slots != nullptr;
  const uint32_t t = threadIdx.x;
  if (track) {
    for (int i = t; i < kAggLdsHist; i += NT) L.hist[i] = 0u;
    lds_barrier();
  }
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    const uint64_t r0 = b * cap;
    const unsigned long long f = fill[b];
    const uint64_t r1 = r0 + (f < cap ? f : cap);
    FreqSlot* slice = T.slots + (b << kFreqSliceLog);
    ulonglong2* halves = reinterpret_cast<ulonglong2*>(slice);
    if (r1 == r0) {
      if (compact) {
        if (t == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        for (uint32_t q = t; q < 2u * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      }
      if (tr.smax && t == 0) tr.smax[b] = 0u;
      continue;
    }
    for (uint32_t s = t; s < S; s += NT) {
      L.K[s] = 0ull;
      L.C[s] = 0u;
    }
    if (t == 0) {
      L.overflow = 0;
      L.cmax = 0u;
    }
    lds_barrier();
    for (uint64_t c0 = r0; c0 < r1; c0 += kChunk) {
      const uint64_t c1 = c0 + kChunk < r1 ? c0 + kChunk : r1;
      // the chunk's records all loaded together; each counted by hash (its slot remembered)
      HashRec rb[kAggHPer];
#pragma unroll
      for (int j = 0; j < kAggHPer; ++j) {
        const uint64_t idx = c0 + (uint64_t)j * NT + t;
        rb[j].h = 0ull;
        rb[j].ref = kHashHole;
        if (idx < c1) rb[j] = recs[idx];
      }
      uint32_t joined = 0u;
      uint32_t sl[kAggHPer];
#pragma unroll
      for (int j = 0; j < kAggHPer; ++j) {
        sl[j] = 0u;
        if (rb[j].ref == kHashHole) continue;
        const unsigned long long kk = rb[j].h ? rb[j].h : 1ull;
        uint32_t s = (uint32_t)rb[j].h & (S - 1u);
        uint32_t probe = 0;
        for (; probe < S; ++probe) {
          const unsigned long long c = atomicCAS(&L.K[s], 0ull, kk);
          if (c == 0ull) {
            L.R[s] = rb[j].ref;
            atomicAdd(&L.C[s], 1u);
            break;
          }
          if (c == kk) {
            atomicAdd(&L.C[s], 1u);
            joined |= 1u << j;
            sl[j] = s;
            break;
          }
          s = (s + 1u) & (S - 1u);
        }
        if (probe == S) L.overflow = 1;
      }
      lds_barrier();  // every group's first reference is in place
      if (!L.overflow && joined) {
        // each joined record compared with its group's first, kAggHCmp records' key words in
        // flight together (a key's words are loaded unconditionally, not word by word)
#pragma unroll
        for (int g = 0; g < kAggHPer; g += kAggHCmp) {
          if (!((joined >> g) & ((1u << kAggHCmp) - 1u))) continue;
          unsigned long long ra[kAggHCmp], wa[kAggHCmp][kAggHWords], wb[kAggHCmp][kAggHWords];
          bool todo[kAggHCmp];
#pragma unroll
          for (int q = 0; q < kAggHCmp; ++q) {
            const int j = g + q;
            todo[q] = false;
            ra[q] = 0ull;
            if (!((joined >> j) & 1u)) continue;
            ra[q] = L.R[sl[j]];
            const unsigned long long rr = rb[j].ref;
            todo[q] = ra[q] != rr;
            if ((ra[q] & kLenMask) != (rr & kLenMask)) {
              L.overflow = 2;  // (a length mismatch: two keys, one hash)
              todo[q] = false;
            }
          }
#pragma unroll
          for (int q = 0; q < kAggHCmp; ++q) {
            const int j = g + q;
            const uint32_t words = (uint32_t)(((ra[q] & kLenMask) + 7ull) >> 3);
            const unsigned long long* a = reinterpret_cast<const unsigned long long*>(T.heap + (ra[q] >> 24));
            const unsigned long long* b = reinterpret_cast<const unsigned long long*>(T.heap + (rb[j].ref >> 24));
            // 16-byte loads (a key's words in half the requests; heap keys are 8-byte aligned),
            // a last odd word alone: nothing past the key's padded bytes is read
#pragma unroll
            for (int w = 0; w < kAggHWords; w += 2) {
              wa[q][w] = wb[q][w] = wa[q][w + 1] = wb[q][w + 1] = 0ull;
              if (todo[q] && (uint32_t)w + 1u < words) {
                const u64x2_a8 x = *reinterpret_cast<const u64x2_a8*>(a + w);
                const u64x2_a8 y = *reinterpret_cast<const u64x2_a8*>(b + w);
                wa[q][w] = x.x;
                wa[q][w + 1] = x.y;
                wb[q][w] = y.x;
                wb[q][w + 1] = y.y;
              } else if (todo[q] && (uint32_t)w < words) {
                wa[q][w] = a[w];
                wb[q][w] = b[w];
              }
            }
          }
#pragma unroll
          for (int q = 0; q < kAggHCmp; ++q) {
            if (!todo[q]) continue;
            const int j = g + q;
            bool eq = true;
#pragma unroll
            for (int w = 0; w < kAggHWords; ++w) eq &= wa[q][w] == wb[q][w];
            if (eq && (ra[q] & kLenMask) > 8u * kAggHWords) eq = heap_refs_equal(T.heap, ra[q], rb[j].ref);  // (longer keys)
            if (!eq) L.overflow = 2;  // two keys, one hash (~never)
          }
        }
      }
      lds_barrier();
    }
    if (L.overflow) {  // hand the region's records back (inserted globally, keys compared)
      if (t == 0) L.retry_base = atomicAdd(n_retry, (unsigned long long)(r1 - r0));
      lds_barrier();
      for (uint64_t i = r0 + t; i < r1; i += NT) retry[L.retry_base + (i - r0)] = rec_raw(recs[i]);
      if (compact) {
        if (t == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        for (uint32_t q = t; q < 2u * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      }
      if (tr.smax && t == 0) tr.smax[b] = 0xFFFFFFFFu;
      lds_barrier();
      continue;
    }
    // the group of slot s as its two 16-byte halves
    auto half = [&](uint32_t s, bool hi) -> ulonglong2 {
      const unsigned long long ref = L.R[s];
      const uint32_t len = (uint32_t)(ref & kLenMask);
      const unsigned long long off = ref >> 24;
      if (!hi) {
        const unsigned long long ctrl = ((unsigned long long)tag_of(L.K[s]) << 32) | kReady |  // (tag_of(1) == tag_of(0))
                                        (len > 16u ? kHeapKey : 0ull) | len;
        return ulonglong2{ctrl, (unsigned long long)L.C[s]};
      }
      if (len > 16u) return ulonglong2{off, 0ull};
      const unsigned long long* w = reinterpret_cast<const unsigned long long*>(T.heap + off);
      return ulonglong2{len ? w[0] : 0ull, len > 8u ? w[1] : 0ull};
    };
    static_assert(S == 8u * NT, "eight slots per thread");
    const uint4 c0v = *reinterpret_cast<const uint4*>(&L.C[8u * t]);
    const uint4 c1v = *reinterpret_cast<const uint4*>(&L.C[8u * t + 4u]);
    const uint32_t cs[8] = {c0v.x, c0v.y, c0v.z, c0v.w, c1v.x, c1v.y, c1v.z, c1v.w};
    uint32_t occ = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!cs[j]) continue;
      occ |= 1u << j;
      if (track || tr.smax) {
        atomicMax(&L.cmax, cs[j]);
        if (track) {
          if (cs[j] < (uint32_t)kAggLdsHist) atomicAdd(&L.hist[cs[j]], 1u);
          else if (cs[j] < (uint32_t)kFreqHist) atomicAdd(&tr.hist[cs[j]], 1ull);
          else {
            const unsigned long long i = atomicAdd(tr.n_big, 1ull);
            if (i < tr.big_cap) tr.big[i] = cs[j];
          }
        }
      }
    }
    uint32_t tot;
    const uint32_t k = block_prefix<NT>((uint32_t)__builtin_popcount(occ), L.wsum, &tot);
    if (compact) {
      tr.cmp.bits[(b << 8) + t] = (uint8_t)occ;
      if (t == 0) {
        const unsigned long long at = atomicAdd(tr.cmp.cursor, (unsigned long long)tot);
        L.cbase = at;
        tr.cmp.base[b] = at;
        tr.cmp.num[b] = tot;
      }
      lds_barrier();
      ulonglong2* out = reinterpret_cast<ulonglong2*>(tr.cmp.slots + L.cbase + k);  // (as the packed kernel)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!(occ & (1u << j))) continue;
        *out++ = half(8u * t + (uint32_t)j, false);
        *out++ = half(8u * t + (uint32_t)j, true);
      }
    } else {
      for (uint32_t q = t; q < 2u * S; q += NT) {
        const uint32_t s = q >> 1;
        if (L.C[s]) halves[q] = half(s, (q & 1u) != 0u);
        else if (tr.write_all) halves[q] = ulonglong2{0ull, 0ull};
      }
    }
    if (t == 0) {
      if (tot) atomicAdd(new_groups, (unsigned long long)tot);
      if (tr.smax) tr.smax[b] = L.cmax;
    }
    lds_barrier();  // LDS is reused by the next slice
  }
  if (track) {
    lds_barrier();
    for (int i = t; i < kAggLdsHist; i += NT)
      if (L.hist[i]) atomicAdd(&tr.hist[i], (unsigned long long)L.hist[i]);
  }
}

// Hashed records into the GLOBAL table (T may hold groups; any slice count): the fall-back of
// the hashed path -- tables of fewer slices than level-1 regions, tables that already hold
// groups, and the records a slice aggregation handed back.  Each workgroup pre-aggregates its
// chunks of records in an LDS image by hash (as dq_freq_agg_hashed_kernel, joins compared byte
// for byte with the group's first record) and inserts each LDS group ONCE with its count when the
// image is half full and at the end, so a key repeated over many rows (few groups) costs one
// global insert per workgroup flush, not one per row.  A record whose hash group holds another
// key, or that finds the image full, is inserted on its own.
__global__ __launch_bounds__(kAggHThreads) void dq_freq_insert_hashed_kernel(FreqTable T, const FreqRec* __restrict__ recs,
                                                                             uint64_t n) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kAggHThreads;
  constexpr uint32_t kChunk = 64u * NT;
  __shared__ AggLdsH L;
  const uint32_t t = threadIdx.x;
  for (uint32_t s = t; s < S; s += NT) {
    L.K[s] = 0ull;
    L.C[s] = 0u;
  }
  if (t == 0) L.fresh = 0u;  // (groups in the image)
  lds_barrier();
  auto flush = [&]() {
    for (uint32_t s = t; s < S; s += NT) {
      const uint32_t c = L.C[s];
      if (c) {
        FreqRec r;
        r.k0 = L.K[s];  // (kk: a hash of 0 was kept as 1 -- the key's own hash is recomputed below)
        r.k1 = L.R[s];
        Key k = hashed_key(T, r);
        k.hash = k.len > 16 ? hash_long(k.ptr, k.len) : hash_inline(k.k0, k.k1, k.len);
        (void)global_insert<true, true>(T, k, (unsigned long long)c);
      }
      L.K[s] = 0ull;
      L.C[s] = 0u;
    }
    if (t == 0) L.fresh = 0u;
    lds_barrier();
  };
  for (uint64_t c0 = (uint64_t)blockIdx.x * kChunk; c0 < n; c0 += (uint64_t)gridDim.x * kChunk) {
    const uint64_t c1 = c0 + kChunk < n ? c0 + kChunk : n;
    unsigned long long joined = 0ull;
    for (uint32_t i = 0; i < 64u; ++i) {
      const uint64_t idx = c0 + (uint64_t)i * NT + t;
      if (idx >= c1) break;
      const FreqRec r = recs[idx];
      if (r.k1 == kHashHole) continue;
      const unsigned long long kk = r.k0 ? r.k0 : 1ull;
      uint32_t s = (uint32_t)r.k0 & (S - 1u);
      bool placed = false;
      for (uint32_t probe = 0; probe < S / 2u; ++probe) {  // (half the image: the flush keeps room)
        const unsigned long long c = atomicCAS(&L.K[s], 0ull, kk);
        if (c == 0ull) {
          L.R[s] = r.k1;
          atomicAdd(&L.C[s], 1u);
          atomicAdd(&L.fresh, 1u);
          placed = true;
          break;
        }
        if (c == kk) {
          atomicAdd(&L.C[s], 1u);
          joined |= 1ull << i;
          placed = true;
          break;
        }
        s = (s + 1u) & (S - 1u);
      }
      if (!placed) (void)global_insert<true, true>(T, hashed_key(T, r), 1ull);
    }
    lds_barrier();  // every group's first reference is in place
    while (joined) {
      const uint32_t i = (uint32_t)__builtin_ctzll(joined);
      joined &= joined - 1ull;
      const FreqRec r = recs[c0 + (uint64_t)i * NT + t];
      const unsigned long long kk = r.k0 ? r.k0 : 1ull;
      const uint32_t s = lds_find_hash(L.K, kk, (uint32_t)r.k0 & (S - 1u));
      if (!heap_refs_equal(T.heap, L.R[s], r.k1)) {  // two keys, one hash: this record on its own
        atomicSub(&L.C[s], 1u);
        (void)global_insert<true, true>(T, hashed_key(T, r), 1ull);
      }
    }
    lds_barrier();
    if (L.fresh > S / 4u) flush();
  }
  flush();
}

// ---- Canonical UUID keys on the partition path (round 6, dq_uuidpack.h).  A table whose keys
// are UUID text (isPrimaryKey's ids, Check.scala:140-230) stages each row as its 128-bit value
// (UuidRec), straight into its level-1 region; the level-2 split moves the same 16-byte records;
// the slice aggregation counts them by table hash in LDS and compares every record that joins a
// hash group with the group's first key IN LDS (two words), so the grouping is exact with no
// key-byte reads; and the write-out turns each GROUP's words back into its 36 text bytes in the
// key heap.  Against the hashed records of round 6's first build (every row's bytes copied into
// the heap, then two random heap reads per row in the aggregation) the path moves no key bytes
// but the input and the groups' text.
constexpr int kUuidPer = 8;    // rows per thread per stage tile
constexpr int kUuidWin = 2;    // rows whose key loads are in flight
constexpr uint32_t kUuidTile = (uint32_t)kStageThreads * kUuidPer;
constexpr uint32_t kUuidHeap = 40;  // heap bytes of a group's text (36, 8-byte aligned)

// The 36 bytes at ob as nine words (two 16-byte loads and one 4-byte load through the values'
// descriptor; bytes past the values read 0, so a shorter key near the end never faults).
__device__ __forceinline__ void uuid_load(__amdgpu_buffer_rsrc_t rs, uint32_t ob, uint32_t (&w)[9]) {
  const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)ob, 0, 0);
  const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(ob + 16u), 0, 0);
  w[0] = a[0];
  w[1] = a[1];
  w[2] = a[2];
  w[3] = a[3];
  w[4] = b[0];
  w[5] = b[1];
  w[6] = b[2];
  w[7] = b[3];
  w[8] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(ob + 32u), 0, 0);
}

// A group's text into the heap at off (five 8-byte stores: 36 bytes and 4 of zero padding).
__device__ __forceinline__ void uuid_store_text(uint8_t* heap, unsigned long long off, uint64_t lo, uint64_t hi) {
  uint32_t w[10];
  uuid_unpack(lo, hi, w);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(heap + off);
#pragma unroll
  for (int i = 0; i < 5; ++i) dst[i] = (unsigned long long)w[2 * i] | ((unsigned long long)w[2 * i + 1] << 32);
}

// Stage + level-1 split of one utf8 key column of canonical UUIDs (the host probed the batch;
// NULL rows stage nothing -- the table is not Histogram's NULL-as-key grouping).  A non-NULL key
// that is not a canonical UUID is counted in bad_keys and staged nothing: the host rolls the batch
// back and stages the table's keys as hashed records from then on.  Tiles of kUuidTile rows:
// the offsets as (begin, end) pairs, then each row's 36 bytes with kUuidWin rows in flight.
__global__ __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(DQ_STAGEP_WAVES))) void dq_freq_stage_uuid_kernel(
    FreqKeySpec ks, const DevColumn* __restrict__ cols, int64_t n_rows, int b1, UuidRec* __restrict__ out,
    uint64_t cap1, unsigned long long* fill1, FreqRec* ovf, unsigned long long* ovf_n, uint64_t ovf_cap,
    unsigned int* flag, uint32_t* hll, unsigned long long* bad_keys, unsigned long long* staged) {
  __shared__ PartLdsT<(1 << kStageBinBits), UuidRec, kPartSub> L;
  __shared__ uint32_t regs[kHllM];
  const uint32_t t = threadIdx.x;
  const uint32_t nb = 1u << b1;
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  lds_barrier();
  const DevColumn& c0 = cols[ks.key_cols[0]];
  const int32_t* offs = uniform_ptr(c0.offsets);
  const uint32_t heap_end = __builtin_amdgcn_readfirstlane((uint32_t)offs[n_rows]);
  const __amdgpu_buffer_rsrc_t rs_vals = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(static_cast<const uint8_t*>(uniform_ptr(c0.values))), 0, (int)heap_end, 0x00020000);
  const uint8_t* validity = uniform_ptr(c0.validity);
  const int64_t n_tiles = (n_rows + kUuidTile - 1) / kUuidTile;
  uint32_t n_bad = 0u;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t r0 = tile * (int64_t)kUuidTile;
    const int64_t left = n_rows - r0;
    const uint32_t m = (uint32_t)(left < (int64_t)kUuidTile ? left : (int64_t)kUuidTile);
    const uint32_t vword = tile_valid_word<kStageThreads, kUuidPer>(validity, r0, m);
    const __amdgpu_buffer_rsrc_t rs_off =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(offs + r0), 0, (int)(4u * (m + 1u)), 0x00020000);
    uint32_t pob[kUuidPer], len[kUuidPer];
#pragma unroll
    for (int j = 0; j < kUuidPer; ++j) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_off, (int)(4u * ((uint32_t)j * kStageThreads + t)), 0, 0);
      pob[j] = v[0];
      len[j] = v[1] - v[0];
    }
    UuidRec rec[kUuidPer];
    uint32_t bin[kUuidPer];
    uint32_t kw[kUuidWin][9];
#pragma unroll
    for (int j = 0; j < kUuidWin; ++j) uuid_load(rs_vals, pob[j], kw[j]);
#pragma unroll
    for (int j = 0; j < kUuidPer; ++j) {
      uint32_t w[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) w[i] = kw[j % kUuidWin][i];
      if (j + kUuidWin < kUuidPer) uuid_load(rs_vals, pob[j + kUuidWin], kw[j % kUuidWin]);
      bin[j] = kPartNoBin;
      rec[j].lo = rec[j].hi = 0ull;
      const uint32_t i = (uint32_t)j * kStageThreads + t;
      const bool valid = validity == nullptr || ((stage_valid_mask(vword, j) >> (t & 63u)) & 1u);
      if (i >= m || !valid) continue;
      uint64_t lo, hi;
      if (len[j] != kUuidLen || !uuid_pack(w, &lo, &hi)) {
        ++n_bad;
        continue;
      }
      rec[j].lo = lo;
      rec[j].hi = hi;
      const uint64_t h = hash_uuid(lo, hi);
      bin[j] = (uint32_t)(h >> (64 - b1)) & (nb - 1u);
      stage_sketch(regs, h);
    }
    part_tile<kUuidPer, (1 << kStageBinBits), UuidRec, kPartSub, false, DQ_STAGE_WOUT_UNROLL, false, kStageThreads>(
        L, rec, bin, nb, 0, out, cap1, fill1, ovf, ovf_n, ovf_cap, flag, staged);
  }
  for (int d = 32; d >= 1; d >>= 1) n_bad += __shfl_xor(n_bad, d, 64);
  if ((t & 63u) == 0u && n_bad) atomicAdd(bad_keys, (unsigned long long)n_bad);
  lds_barrier();
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// Stage + level-1 split of 16-byte keys as Raw16Rec (round 6): STRING -- one utf8 column whose
// non-NULL keys are all 16 bytes (one 16-byte load per row; any other length is counted in
// bad_keys and the host rolls the batch back to hashed records); otherwise two 8-byte fixed-width
// columns, the record being their value bits (make_key's encoding), a NULL in either dropping the
// row.  The tile layout, the split and the sketch are the UUID stage's.
template <bool STRING>
__global__ __launch_bounds__(kStageThreads) __attribute__((amdgpu_waves_per_eu(DQ_STAGEP_WAVES))) void dq_freq_stage_raw16_kernel(
    FreqKeySpec ks, const DevColumn* __restrict__ cols, int64_t n_rows, int b1, Raw16Rec* __restrict__ out,
    uint64_t cap1, unsigned long long* fill1, FreqRec* ovf, unsigned long long* ovf_n, uint64_t ovf_cap,
    unsigned int* flag, uint32_t* hll, unsigned long long* bad_keys, unsigned long long* staged) {
  __shared__ PartLdsT<(1 << kStageBinBits), Raw16Rec, kPartSub> L;
  __shared__ uint32_t regs[kHllM];
  const uint32_t t = threadIdx.x;
  const uint32_t nb = 1u << b1;
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads) regs[i] = 0xFFFFFFFFu;  // (stage_sketch)
  lds_barrier();
  const DevColumn& c0 = cols[ks.key_cols[0]];
  const DevColumn& c1 = cols[ks.key_cols[STRING ? 0 : 1]];
  const int32_t* offs = STRING ? uniform_ptr(c0.offsets) : nullptr;
  const uint32_t heap_end = STRING ? __builtin_amdgcn_readfirstlane((uint32_t)offs[n_rows]) : 0u;
  const __amdgpu_buffer_rsrc_t rs_vals = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(static_cast<const uint8_t*>(uniform_ptr(c0.values))), 0, (int)heap_end, 0x00020000);
  const uint8_t* validity0 = uniform_ptr(c0.validity);
  const uint8_t* validity1 = STRING ? nullptr : uniform_ptr(c1.validity);
  const unsigned long long* v0 = static_cast<const unsigned long long*>(uniform_ptr(c0.values));
  const unsigned long long* v1 = static_cast<const unsigned long long*>(uniform_ptr(c1.values));
  const int64_t n_tiles = (n_rows + kUuidTile - 1) / kUuidTile;
  uint32_t n_bad = 0u;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t r0 = tile * (int64_t)kUuidTile;
    const int64_t left = n_rows - r0;
    const uint32_t m = (uint32_t)(left < (int64_t)kUuidTile ? left : (int64_t)kUuidTile);
    const uint32_t vword0 = tile_valid_word<kStageThreads, kUuidPer>(validity0, r0, m);
    const uint32_t vword1 = STRING ? 0u : tile_valid_word<kStageThreads, kUuidPer>(validity1, r0, m);
    Raw16Rec rec[kUuidPer];
    uint32_t bin[kUuidPer];
    if constexpr (STRING) {
      const __amdgpu_buffer_rsrc_t rs_off =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(offs + r0), 0, (int)(4u * (m + 1u)), 0x00020000);
      uint32_t pob[kUuidPer], len[kUuidPer];
#pragma unroll
      for (int j = 0; j < kUuidPer; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_off, (int)(4u * ((uint32_t)j * kStageThreads + t)), 0, 0);
        pob[j] = v[0];
        len[j] = v[1] - v[0];
      }
#pragma unroll
      for (int j = 0; j < kUuidPer; ++j) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs_vals, (int)pob[j], 0, 0);
        rec[j].lo = (unsigned long long)w[0] | ((unsigned long long)w[1] << 32);
        rec[j].hi = (unsigned long long)w[2] | ((unsigned long long)w[3] << 32);
        bin[j] = len[j];  // (the length, until the row is checked below)
      }
    } else {
#pragma unroll
      for (int j = 0; j < kUuidPer; ++j) {
        const int64_t row = r0 + (int64_t)j * kStageThreads + t;
        rec[j].lo = rec[j].hi = 0ull;
        if (row < n_rows) {
          rec[j].lo = v0[row];
          rec[j].hi = v1[row];
        }
        bin[j] = 16u;
      }
    }
#pragma unroll
    for (int j = 0; j < kUuidPer; ++j) {
      const uint32_t i = (uint32_t)j * kStageThreads + t;
      const bool valid = (validity0 == nullptr || ((stage_valid_mask(vword0, j) >> (t & 63u)) & 1u)) &&
                         (STRING || validity1 == nullptr || ((stage_valid_mask(vword1, j) >> (t & 63u)) & 1u));
      const uint32_t n = bin[j];
      bin[j] = kPartNoBin;
      if (i >= m || !valid) continue;
      if (n != 16u) {
        ++n_bad;
        continue;
      }
      const uint64_t h = hash_inline(rec[j].lo, rec[j].hi, 16u);
      bin[j] = (uint32_t)(h >> (64 - b1)) & (nb - 1u);
      stage_sketch(regs, h);
    }
    part_tile<kUuidPer, (1 << kStageBinBits), Raw16Rec, kPartSub, false, DQ_STAGE_WOUT_UNROLL, false, kStageThreads>(
        L, rec, bin, nb, 0, out, cap1, fill1, ovf, ovf_n, ovf_cap, flag, staged);
  }
  for (int d = 32; d >= 1; d >>= 1) n_bad += __shfl_xor(n_bad, d, 64);
  if ((t & 63u) == 0u && n_bad) atomicAdd(bad_keys, (unsigned long long)n_bad);
  lds_barrier();
  for (uint32_t i = t; i < (uint32_t)kHllM; i += kStageThreads)
    if (regs[i] != 0xFFFFFFFFu) atomicMax(&hll[i], stage_sketch_rank(regs[i]));
}

// The owner aggregation of slice regions of UUID records into a FRESH table.  LDS image: the
// table hash (0 kept as 1; the claimed mark), the group's key words and its count.  A chunk of
// kAggUPer records per thread is counted by hash (one CAS per probe; the claimer stores its key
// words), then, after one barrier, every record that joined an existing hash group is compared
// with the group's words in LDS.  A full image, two keys of one hash (a slice holding two UUIDs of
// one 64-bit hash: ~never) or no heap room hands the slice's records to the retry list (their
// bits; the host converts and inserts them globally).  Write-out: each thread's groups (it owns
// eight consecutive slots) as whole 32-byte slots at one reserved place per slice (tr.cmp) or in
// the slot image, and their text as 40 consecutive heap bytes each at one heap reservation per
// slice.
constexpr int kAggUThreads = 512;  // (the 58 KB image allows two workgroups per CU: 4 waves per SIMD)
constexpr int kAggUPer = 4;  // (<= 128 VGPRs: two workgroups per CU)
struct AggLdsU {
  unsigned long long K[kFreqSliceSlots];
  ulonglong2 KW[kFreqSliceSlots];  // the group's key words {w0, w1}: one 16-byte LDS access
  uint32_t C[kFreqSliceSlots];
  uint32_t wsum[8];
  int overflow;
  uint32_t cmax;
  unsigned long long retry_base;
  unsigned long long cbase;
  unsigned long long hbase;
  uint32_t hist[kAggLdsHist];
};

// The record's two key words and its table hash (UuidRec: the UUID's 128 bits; FreqRec: the
// inline key bytes with the length in k1's top byte -- the same words make the same key).
__device__ inline uint64_t agg_w0(const UuidRec& r) { return r.lo; }
__device__ inline uint64_t agg_w1(const UuidRec& r) { return r.hi; }
__device__ inline uint64_t agg_w0(const FreqRec& r) { return r.k0; }
__device__ inline uint64_t agg_w1(const FreqRec& r) { return r.k1; }
__device__ inline uint64_t agg_w0(const Raw16Rec& r) { return r.lo; }
__device__ inline uint64_t agg_w1(const Raw16Rec& r) { return r.hi; }
__device__ inline uint64_t agg_hash(uint64_t w0, uint64_t w1, const Raw16Rec*) { return hash_inline(w0, w1, 16u); }
__device__ inline uint64_t agg_hash(uint64_t w0, uint64_t w1, const UuidRec*) { return hash_uuid(w0, w1); }
__device__ inline uint64_t agg_hash(uint64_t w0, uint64_t w1, const FreqRec*) {
  const uint32_t len = (uint32_t)(w1 >> kRecLenShift);
  return hash_inline(w0, w1 & ((1ull << kRecLenShift) - 1ull), len);
}

// R = UuidRec: canonical UUID records (text into the heap at write-out); R = FreqRec: 16-byte
// records of keys of <= 15 bytes (round 6: the same hash-CAS + LDS compare in place of
// dq_freq_agg_region_kernel's two-word publish protocol, for fresh tables).
template <typename R>
__global__ __launch_bounds__(kAggUThreads) __attribute__((amdgpu_waves_per_eu(4))) void dq_freq_agg_keys_kernel(
    FreqTable T, const R* __restrict__ recs, const unsigned long long* __restrict__ fill, uint64_t cap,
    uint64_t n_slices, FreqRec* retry, unsigned long long* n_retry, unsigned long long* new_groups, AggTrack tr) {
  constexpr bool kUuid = std::is_same<R, UuidRec>::value;
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kAggUThreads;
  constexpr uint32_t kChunk = (uint32_t)kAggUPer * NT;
  static_assert(S == 4u * NT, "four slots per thread");
  __shared__ AggLdsU L;
  const bool track = tr.hist != nullptr;
  const bool compact = tr.cmp.slots != nullptr;
  const uint32_t t = threadIdx.x;
  if (track) {
    for (int i = t; i < kAggLdsHist; i += NT) L.hist[i] = 0u;
    lds_barrier();
  }
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    const uint64_t r0 = b * cap;
    const unsigned long long f = fill[b];
    const uint64_t r1 = r0 + (f < cap ? f : cap);
    ulonglong2* halves = reinterpret_cast<ulonglong2*>(T.slots + (b << kFreqSliceLog));
    if (r1 == r0) {
      if (compact) {
        if (t == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        for (uint32_t q = t; q < 2u * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      }
      if (tr.smax && t == 0) tr.smax[b] = 0u;
      continue;
    }
    for (uint32_t s = t; s < S; s += NT) {
      L.K[s] = 0ull;
      L.C[s] = 0u;
    }
    if (t == 0) {
      L.overflow = 0;
      L.cmax = 0u;
    }
    lds_barrier();
    for (uint64_t c0 = r0; c0 < r1; c0 += kChunk) {
      R rb[kAggUPer];
      uint32_t sl[kAggUPer];
#pragma unroll
      for (int j = 0; j < kAggUPer; ++j) {
        const uint64_t idx = c0 + (uint64_t)j * NT + t;
        if (idx < r1) rb[j] = recs[idx];
      }
      // every record's first probe is issued before any result is looked at (independent LDS
      // round trips, as dq_freq_agg_packed_kernel); at the table's ~0.4 load most records are
      // counted there
      uint32_t joined = 0u;
      unsigned long long kk[kAggUPer], cv[kAggUPer];
#pragma unroll
      for (int j = 0; j < kAggUPer; ++j) {
        const bool in = c0 + (uint64_t)j * NT + t < r1;
        const uint64_t h = agg_hash(agg_w0(rb[j]), agg_w1(rb[j]), (const R*)nullptr);
        kk[j] = h ? h : 1ull;
        sl[j] = (uint32_t)h & (S - 1u);
        cv[j] = in ? atomicCAS(&L.K[sl[j]], 0ull, kk[j]) : ~0ull;
      }
#pragma unroll
      for (int j = 0; j < kAggUPer; ++j) {
        if (c0 + (uint64_t)j * NT + t >= r1) continue;
        uint32_t s = sl[j];
        unsigned long long c = cv[j];
        uint32_t probe = 0;
        while (true) {
          if (c == 0ull) {
            L.KW[s] = ulonglong2{agg_w0(rb[j]), agg_w1(rb[j])};
            atomicAdd(&L.C[s], 1u);
            break;
          }
          if (c == kk[j]) {
            atomicAdd(&L.C[s], 1u);
            joined |= 1u << j;
            sl[j] = s;
            break;
          }
          if (++probe == S) {
            L.overflow = 1;
            break;
          }
          s = (s + 1u) & (S - 1u);
          c = atomicCAS(&L.K[s], 0ull, kk[j]);
        }
      }
      lds_barrier();  // every group's first key words are in place (later claims touch other slots)
#pragma unroll
      for (int j = 0; j < kAggUPer; ++j)
        if ((joined >> j) & 1u) {
          const ulonglong2 w = L.KW[sl[j]];
          if (w.x != agg_w0(rb[j]) || w.y != agg_w1(rb[j])) L.overflow = 2;
        }
    }
    lds_barrier();
    // this thread's eight slots: occupancy, the slice's group count, one heap reservation
    const uint4 cv = *reinterpret_cast<const uint4*>(&L.C[4u * t]);
    const uint32_t cs[4] = {cv.x, cv.y, cv.z, cv.w};
    uint32_t occ = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) occ |= (cs[j] ? 1u : 0u) << j;
    uint32_t tot;
    const uint32_t k = block_prefix<NT>((uint32_t)__builtin_popcount(occ), L.wsum, &tot);
    if (t == 0 && !L.overflow) {
      // the slice's heap text (UUIDs) and compacted slots, both reserved before one barrier (a
      // slice that then hands its records back leaves an unused range: readers go by base / num)
      unsigned long long hb = 0ull, at = 0ull;
      const unsigned long long need = (unsigned long long)tot * kUuidHeap;
      if (kUuid) hb = atomicAdd(T.heap_used, need);
      if (compact) at = atomicAdd(tr.cmp.cursor, (unsigned long long)tot);
      if (kUuid && hb + need > T.heap_cap) L.overflow = 3;  // (the host sized the heap from the sketch; it clamps heap_used)
      L.hbase = hb;
      L.cbase = at;
      if (compact) {
        tr.cmp.base[b] = at;
        tr.cmp.num[b] = L.overflow ? 0u : tot;
      }
    }
    lds_barrier();
    if (L.overflow) {  // hand the region's records back (their bits: the host converts, then inserts globally)
      if (t == 0) L.retry_base = atomicAdd(n_retry, (unsigned long long)(r1 - r0));
      lds_barrier();
      for (uint64_t i = r0 + t; i < r1; i += NT) retry[L.retry_base + (i - r0)] = rec_raw(recs[i]);
      if (compact) {
        if (t == 0) tr.cmp.num[b] = 0u;
      } else if (tr.write_all) {
        for (uint32_t q = t; q < 2u * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      }
      if (tr.smax && t == 0) tr.smax[b] = 0xFFFFFFFFu;
      lds_barrier();
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!cs[j] || !(track || tr.smax)) continue;
      atomicMax(&L.cmax, cs[j]);
      if (track) {
        if (cs[j] < (uint32_t)kAggLdsHist) atomicAdd(&L.hist[cs[j]], 1u);
        else if (cs[j] < (uint32_t)kFreqHist) atomicAdd(&tr.hist[cs[j]], 1ull);
        else {
          const unsigned long long i = atomicAdd(tr.n_big, 1ull);
          if (i < tr.big_cap) tr.big[i] = cs[j];
        }
      }
    }
    if (compact) {
      const uint32_t pair = occ | ((uint32_t)__shfl_down((int)occ, 1, 64) << 4);  // (byte t / 2: slots 4t .. 4t + 7)
      if (!(t & 1u)) tr.cmp.bits[(b << 8) + (t >> 1)] = (uint8_t)pair;
    }
    unsigned long long hoff = L.hbase + (unsigned long long)k * kUuidHeap;
    FreqSlot* out = compact ? tr.cmp.slots + L.cbase + k : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t s = 4u * t + (uint32_t)j;
      if (!cs[j]) {
        if (!compact && tr.write_all) {
          halves[2u * s] = ulonglong2{0ull, 0ull};
          halves[2u * s + 1u] = ulonglong2{0ull, 0ull};
        }
        continue;
      }
      const ulonglong2 kw = L.KW[s];
      const uint64_t w0 = kw.x, w1 = kw.y;
      unsigned long long ctrl, k0, k1;
      if constexpr (kUuid) {
        uuid_store_text(T.heap, hoff, w0, w1);
        ctrl = ((unsigned long long)tag_of(hash_uuid(w0, w1)) << 32) | kReady | kHeapKey | kUuidLen;
        k0 = hoff;
        k1 = 0ull;
        hoff += kUuidHeap;
      } else if constexpr (std::is_same<R, Raw16Rec>::value) {  // (a 16-byte key, inline)
        ctrl = ((unsigned long long)tag_of(agg_hash(w0, w1, (const R*)nullptr)) << 32) | kReady | 16ull;
        k0 = w0;
        k1 = w1;
      } else {
        ctrl = ((unsigned long long)tag_of(agg_hash(w0, w1, (const R*)nullptr)) << 32) | kReady | (w1 >> kRecLenShift);
        k0 = w0;
        k1 = w1 & ((1ull << kRecLenShift) - 1ull);
      }
      if (compact) {
        *out++ = FreqSlot{ctrl, (unsigned long long)cs[j], k0, k1};
      } else {
        halves[2u * s] = ulonglong2{ctrl, (unsigned long long)cs[j]};
        halves[2u * s + 1u] = ulonglong2{k0, k1};
      }
    }
    lds_barrier();  // LDS is reused by the next slice (every cmax update is in)
    if (t == 0) {  // (thread 0 resets L.cmax only at the next slice's start, after this read)
      if (tot) atomicAdd(new_groups, (unsigned long long)tot);
      if (tr.smax) tr.smax[b] = L.cmax;
    }
  }
  if (track) {
    lds_barrier();
    for (int i = t; i < kAggLdsHist; i += NT)
      if (L.hist[i]) atomicAdd(&tr.hist[i], (unsigned long long)L.hist[i]);
  }
}

// A list of UUID records' bits (FreqRec {lo, hi}: the retry / overflow lists of the UUID path)
// turned in place into hashed records {table hash, heap reference}: each key's text written to
// the heap (one reservation per wave), so dq_freq_insert_hashed_kernel can insert them.  The host
// reserved the room; a record that finds none raises the heap-full bit.
template <bool UUID>
__global__ __launch_bounds__(kBlock) void dq_freq_uuid_to_hashed_kernel(FreqTable T, FreqRec* recs, uint64_t n) {
  constexpr unsigned long long kBytes = UUID ? kUuidHeap : 16ull;  // (a Raw16Rec's key: 16 bytes)
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kBlock; i0 < n; i0 += (uint64_t)gridDim.x * kBlock) {
    const uint64_t i = i0 + threadIdx.x;
    const bool act = i < n;
    const uint64_t ball = __ballot(act);
    if (!ball) continue;
    const uint32_t first = (uint32_t)__builtin_ctzll(ball);
    unsigned long long base = 0ull;
    if (lane == first) base = atomicAdd(T.heap_used, (unsigned long long)__popcll(ball) * kBytes);
    base = __shfl(base, (int)first, 64);
    if (!act) continue;
    const FreqRec r = recs[i];
    const unsigned long long off = base + (unsigned long long)__popcll(ball & ((1ull << lane) - 1ull)) * kBytes;
    if (off + kBytes > T.heap_cap) {
      atomicOr(T.overflow, 2u);
      continue;
    }
    FreqRec o;
    if constexpr (UUID) {
      uuid_store_text(T.heap, off, r.k0, r.k1);
      o.k0 = hash_uuid(r.k0, r.k1);
      o.k1 = (off << 24) | kUuidLen;
    } else {
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(T.heap + off);
      dst[0] = r.k0;
      dst[1] = r.k1;
      o.k0 = hash_inline(r.k0, r.k1, 16u);
      o.k1 = (off << 24) | 16ull;
    }
    recs[i] = o;
  }
}

// Whether a single-utf8-key staging holds canonical UUIDs: out[0] counts the sampled non-NULL keys
// (kPackProbe scattered rows, as dq_freq_pack_probe_kernel) that are not, out[1] those that are.
__global__ __launch_bounds__(kBlock) void dq_freq_uuid_probe_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                    int64_t n_rows, unsigned long long* out) {
  const DevColumn& c = cols[ks.key_cols[0]];
  constexpr int64_t kProbe = 16384;  // (as kPackProbe)
  const int64_t samples = n_rows < kProbe ? n_rows : kProbe;
  uint32_t bad = 0u, good = 0u;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < samples; i += (int64_t)gridDim.x * kBlock) {
    const int64_t row = samples == n_rows ? i : (int64_t)(((uint64_t)i * 11400714819323198485ull) % (uint64_t)n_rows);
    if (c.validity != nullptr && !((c.validity[row >> 3] >> (row & 7)) & 1u)) continue;
    const uint8_t* v = static_cast<const uint8_t*>(c.values) + c.offsets[row];
    const uint32_t n = (uint32_t)(c.offsets[row + 1] - c.offsets[row]);
    uint64_t lo, hi;
    if (uuid_pack_bytes(v, n, &lo, &hi)) ++good;
    else ++bad;
  }
  if (bad) atomicAdd(&out[0], (unsigned long long)bad);
  if (good) atomicAdd(&out[1], (unsigned long long)good);
}

// The slot image of a compacted table (AggTrack::cmp) rebuilt in T: slice b's groups, stored in
// slot order from cmp.base[b], go back to the slots its occupancy bitmap names; every other slot
// is written empty (T is not cleared first).  One workgroup per slice, whole 1 KiB stores.
__global__ __launch_bounds__(kAggPThreads) void dq_freq_expand_kernel(FreqTable T, FreqCompact cmp, uint64_t n_slices) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kAggPThreads;
  __shared__ uint16_t pos[kFreqSliceSlots];  // slot -> its group's index in the slice, 0xFFFF empty
  __shared__ uint32_t wsum[4];
  static_assert(S == 8u * NT, "eight slots per thread");
  const uint32_t t = threadIdx.x;
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    ulonglong2* halves = reinterpret_cast<ulonglong2*>(T.slots + (b << kFreqSliceLog));
    const uint32_t n = cmp.num[b];
    if (n == 0u) {
      for (uint32_t q = t; q < 2u * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      continue;
    }
    const uint32_t occ = cmp.bits[(b << 8) + t];
    uint32_t tot;
    uint32_t k = block_prefix<NT>((uint32_t)__builtin_popcount(occ), wsum, &tot);
#pragma unroll
    for (int j = 0; j < 8; ++j) pos[8u * t + (uint32_t)j] = (occ & (1u << j)) ? (uint16_t)(k++) : (uint16_t)0xFFFFu;
    lds_barrier();
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(cmp.slots + cmp.base[b]);
    for (uint32_t q = t; q < 2u * S; q += NT) {
      const uint32_t g = pos[q >> 1];
      halves[q] = g == 0xFFFFu ? ulonglong2{0ull, 0ull} : src[2u * g + (q & 1u)];
    }
    lds_barrier();  // (pos and wsum are rewritten by the next slice)
  }
}

// dq_freq_export_slices_kernel over a compacted table: slice b's groups are the cmp.num[b]
// records from cmp.base[b]; slices whose largest count (smax) is below min_count are skipped.
__global__ __launch_bounds__(kBlock) void dq_freq_export_compact_kernel(FreqCompact cmp, uint64_t n_slices,
                                                                        unsigned long long min_count,
                                                                        const uint32_t* __restrict__ smax, FreqOut out) {
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    if (smax && (unsigned long long)smax[b] < min_count) continue;
    const FreqSlot* g = cmp.slots + cmp.base[b];
    const uint32_t n = cmp.num[b];
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
      const FreqSlot e = g[i];
      if (e.count >= min_count) {
        const unsigned long long j = atomicAdd(out.n, 1ull);
        if (j < out.cap) {
          out.ctrl[j] = e.ctrl;
          out.count[j] = e.count;
          out.k0[j] = e.k0;
          out.k1[j] = e.k1;
        }
      }
    }
  }
}

// Table growth: move every group of `old_slots` into the (empty, larger) table T.  All keys
// are distinct, so a slot is claimed with its final ctrl word and nobody compares keys.
__global__ __launch_bounds__(kBlock) void dq_freq_rehash_kernel(const FreqSlot* __restrict__ old_slots,
                                                                uint64_t old_n, FreqTable T) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < old_n; i += (uint64_t)gridDim.x * kBlock) {
    const FreqSlot e = old_slots[i];
    if (!(e.ctrl & kReady)) continue;
    const uint32_t len = (uint32_t)(e.ctrl & kLenMask);
    const uint64_t h = (e.ctrl & kHeapKey) ? hash_long(T.heap + e.k0, len) : hash_inline(e.k0, e.k1, len);
    uint64_t it = 0;
    for (; it < kFreqSliceSlots; ++it) {
      const uint64_t slot = probe_slot(T, h, it);
      if (atomicCAS(&T.slots[slot].ctrl, 0ull, e.ctrl) == 0ull) {
        T.slots[slot].count = e.count;
        T.slots[slot].k0 = e.k0;
        T.slots[slot].k1 = e.k1;
        break;
      }
    }
    if (it == kFreqSliceSlots) atomicOr(T.overflow, 1u);
  }
}

static unsigned slot_blocks(const FreqTable& T) {
  const uint64_t n = T.mask + 1;
  uint64_t blocks = (n + kBlock * 16 - 1) / (kBlock * 16);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  return (unsigned)blocks;
}

hipError_t launch_freq_stage(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, FreqRec* d_out,
                             unsigned long long* d_cursor, uint32_t* d_hll,
                             unsigned long long* d_long_key, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + kBlock * 16 - 1) / (kBlock * 16);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(dq_freq_stage_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols, n_rows, d_out,
                     d_cursor, d_hll, d_long_key);
  return hipGetLastError();
}

hipError_t launch_freq_split(const FreqRec* d_in, uint64_t n, const unsigned long long* d_in_off, uint64_t n_regions,
                             uint64_t max_region, int bits, int b2, unsigned long long* d_count, FreqRec* d_out,
                             const unsigned long long* d_region_start, unsigned long long* d_cursor, hipStream_t stream) {
  if (bits < 0 || bits > 2 * kPartMaxBinBits || b2 < 0 || bits - b2 > kPartMaxBinBits || b2 > kPartMaxBinBits)
    return hipErrorInvalidValue;
  dim3 grid;
  if (d_in_off) {
    if (n_regions == 0 || n_regions > 65535) return hipErrorInvalidValue;
    if (max_region == 0) return hipSuccess;
    grid = dim3((unsigned)((max_region + kPartTile - 1) / kPartTile), (unsigned)n_regions);
  } else {
    if (n == 0) return hipSuccess;
    grid = dim3((unsigned)((n + kPartTile - 1) / kPartTile));
  }
  hipLaunchKernelGGL(dq_freq_split_kernel, grid, dim3(kPartThreads), 0, stream, d_in, n, d_in_off, bits, b2, d_count,
                     d_out, d_region_start, d_cursor);
  return hipGetLastError();
}

template <typename T>
static hipError_t exclusive_scan(T* d_data, uint64_t n, T* d_sums, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t chunks = (n + kScanChunk - 1) / kScanChunk;
  hipLaunchKernelGGL(dq_scan_chunks_kernel<T>, dim3((unsigned)chunks), dim3(kScanThreads), 0, stream, d_data, n, d_sums);
  if (chunks > 1) {
    hipLaunchKernelGGL(dq_scan_sums_kernel<T>, dim3(1), dim3(kScanThreads), 0, stream, d_sums, chunks);
    hipLaunchKernelGGL(dq_scan_add_kernel<T>, dim3((unsigned)chunks), dim3(kScanThreads), 0, stream, d_data, n,
                       static_cast<const T*>(d_sums));
  }
  return hipGetLastError();
}
hipError_t scan_exclusive_u64(unsigned long long* d_data, uint64_t n, unsigned long long* d_sums, hipStream_t stream) {
  return exclusive_scan<unsigned long long>(d_data, n, d_sums, stream);
}
hipError_t scan_exclusive_u32(uint32_t* d_data, uint64_t n, uint32_t* d_sums, hipStream_t stream) {
  return exclusive_scan<uint32_t>(d_data, n, d_sums, stream);
}

hipError_t launch_freq_pieces(const unsigned long long* d_counts, uint64_t n, uint32_t* d_pieces, hipStream_t stream) {
  uint64_t blocks = (n + 1 + kBlock - 1) / kBlock;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(dq_freq_pieces_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, d_counts, n, d_pieces);
  return hipGetLastError();
}

hipError_t launch_freq_agg(const FreqTable& T, const FreqRec* d_recs, const uint64_t* d_off,
                           const uint32_t* d_piece_start, uint64_t n_buckets, uint64_t max_items, int table_empty,
                           FreqRec* d_retry, unsigned long long* d_n_retry, unsigned long long* d_new_groups,
                           hipStream_t stream) {
  uint64_t blocks = max_items < 65536 ? max_items : 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_agg_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_recs, d_off,
                     d_piece_start, n_buckets, table_empty, d_retry, d_n_retry, d_new_groups);
  return hipGetLastError();
}

hipError_t launch_freq_part(const void* d_in, uint64_t in_n, const unsigned long long* d_in_fill, uint64_t in_cap,
                            uint64_t n_in_regions, int id_bits, int bin_bits, void* d_out, uint64_t out_cap,
                            unsigned long long* d_out_fill, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                            uint64_t ovf_cap, unsigned int* d_flag, int rec_kind, hipStream_t stream,
                            unsigned long long* d_staged) {
  if (bin_bits < 0 || bin_bits > kPartMaxBinBits || id_bits < bin_bits || id_bits > 32) return hipErrorInvalidValue;
  const bool packed = rec_kind == kRecPacked;
  const uint64_t tile = packed ? kPartTileP : kPartTile;  // (the kernel's records per workgroup)
  dim3 grid;
  if (d_in_fill) {
    if (n_in_regions == 0 || n_in_regions > 65535) return hipErrorInvalidValue;
    grid = dim3((unsigned)((in_cap + tile - 1) / tile), (unsigned)n_in_regions);
  } else {
    if (in_n == 0) return hipSuccess;
    grid = dim3((unsigned)((in_n + tile - 1) / tile));
  }
  if (packed && bin_bits <= kStageBinBits)
    hipLaunchKernelGGL((dq_freq_part_kernel<uint64_t, (1 << kStageBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const uint64_t*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<uint64_t*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (packed)
    hipLaunchKernelGGL((dq_freq_part_kernel<uint64_t, (1 << kPartMaxBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const uint64_t*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<uint64_t*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (bin_bits <= kStageBinBits && rec_kind == kRecHashed)  // (512 bins: a smaller LDS image, 2 workgroups per CU)
    hipLaunchKernelGGL((dq_freq_part_kernel<HashRec, (1 << kStageBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const HashRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<HashRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (bin_bits <= kStageBinBits && rec_kind == kRecUuid)
    hipLaunchKernelGGL((dq_freq_part_kernel<UuidRec, (1 << kStageBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const UuidRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<UuidRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (bin_bits <= kStageBinBits && rec_kind == kRecRaw16)
    hipLaunchKernelGGL((dq_freq_part_kernel<Raw16Rec, (1 << kStageBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const Raw16Rec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<Raw16Rec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (rec_kind == kRecRaw16)
    hipLaunchKernelGGL((dq_freq_part_kernel<Raw16Rec, (1 << kPartMaxBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const Raw16Rec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<Raw16Rec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (bin_bits <= kStageBinBits && rec_kind == kRecFree)
    hipLaunchKernelGGL((dq_freq_part_kernel<FreqRec, (1 << kStageBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const FreqRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<FreqRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (rec_kind == kRecHashed)
    hipLaunchKernelGGL((dq_freq_part_kernel<HashRec, (1 << kPartMaxBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const HashRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<HashRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else if (rec_kind == kRecUuid)
    hipLaunchKernelGGL((dq_freq_part_kernel<UuidRec, (1 << kPartMaxBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const UuidRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<UuidRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  else
    hipLaunchKernelGGL((dq_freq_part_kernel<FreqRec, (1 << kPartMaxBinBits)>), grid, dim3(kPartThreads), 0, stream,
                       static_cast<const FreqRec*>(d_in), in_n, d_in_fill, in_cap, id_bits, bin_bits,
                       static_cast<FreqRec*>(d_out), out_cap, d_out_fill, d_ovf, d_ovf_n, ovf_cap, d_flag, d_staged);
  return hipGetLastError();
}

// Whether a single-utf8-key staging should pack its keys (dq_keypack.h): a strided sample of
// the batch's rows (kPackProbe of them) is checked, and out[0] counts the sampled non-NULL keys
// that do not pack (longer than 15 bytes or not a digit string).  A batch whose keys mostly do
// not pack would fill the packed stage's overflow list and be staged twice.
constexpr int kPackProbe = 16384;
__global__ __launch_bounds__(kBlock) void dq_freq_pack_probe_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                    int64_t n_rows, unsigned long long* out,
                                                                    unsigned long long* n_long) {
  const DevColumn& c = cols[ks.key_cols[0]];
  const int64_t samples = n_rows < kPackProbe ? n_rows : kPackProbe;
  uint32_t bad = 0u, longer = 0u;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < samples; i += (int64_t)gridDim.x * kBlock) {
    // scattered rows (a multiplicative hash of i), not a fixed stride: a periodic key pattern
    // would alias with a stride
    const int64_t row = samples == n_rows ? i : (int64_t)(((uint64_t)i * 11400714819323198485ull) % (uint64_t)n_rows);
    if (c.validity != nullptr && !((c.validity[row >> 3] >> (row & 7)) & 1u)) continue;
    const uint8_t* v = static_cast<const uint8_t*>(c.values) + c.offsets[row];
    const uint32_t n = (uint32_t)(c.offsets[row + 1] - c.offsets[row]);
    if (n > 15u) {
      ++bad;
      ++longer;
      continue;
    }
    uint64_t k0 = 0ull, k1 = 0ull, p;
    for (uint32_t b = 0; b < n; ++b) {
      const uint64_t x = (uint64_t)v[b];
      if (b < 8u) k0 |= x << (8u * b);
      else k1 |= x << (8u * (b - 8u));
    }
    if (!kp_pack_record(k0, k1, n, &p)) ++bad;
  }
  if (bad) atomicAdd(out, (unsigned long long)bad);
  if (longer && n_long) atomicAdd(n_long, (unsigned long long)longer);
}

hipError_t launch_freq_pack_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                  hipStream_t stream, unsigned long long* d_long) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_freq_pack_probe_kernel, dim3((kPackProbe + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, ks,
                     d_cols, n_rows, d_out, d_long);
  return hipGetLastError();
}

// The rollback image of a region staging, taken on the device before the batch's kernels: the
// level-1 fills, the sizing sketch and the overflow count, and the batch's longest-key counter
// cleared -- one launch instead of three copies and a memset per batch.
__global__ __launch_bounds__(kBlock) void dq_freq_stage_save_kernel(const unsigned long long* __restrict__ fill,
                                                                    unsigned long long* __restrict__ fill_save, uint32_t n_fill,
                                                                    const uint32_t* __restrict__ sketch,
                                                                    uint32_t* __restrict__ sketch_save,
                                                                    const unsigned long long* __restrict__ ovf_n,
                                                                    unsigned long long* __restrict__ ovf_save,
                                                                    unsigned long long* __restrict__ long_key) {
  for (uint32_t i = threadIdx.x; i < n_fill; i += kBlock) fill_save[i] = fill[i];
  for (uint32_t i = threadIdx.x; i < (uint32_t)kHllM; i += kBlock) sketch_save[i] = sketch[i];
  if (threadIdx.x == 0) {
    *ovf_save = *ovf_n;
    *long_key = 0ull;
  }
}

hipError_t launch_freq_stage_save(const unsigned long long* d_fill, unsigned long long* d_fill_save, uint32_t n_fill,
                                  const uint32_t* d_sketch, uint32_t* d_sketch_save, const unsigned long long* d_ovf_n,
                                  unsigned long long* d_ovf_save, unsigned long long* d_long_key, hipStream_t stream) {
  hipLaunchKernelGGL(dq_freq_stage_save_kernel, dim3(1), dim3(kBlock), 0, stream, d_fill, d_fill_save, n_fill, d_sketch,
                     d_sketch_save, d_ovf_n, d_ovf_save, d_long_key);
  return hipGetLastError();
}

hipError_t launch_freq_stage_part(const FreqKeySpec& ks, bool one_string, bool packed, const DevColumn* d_cols,
                                  int64_t n_rows, int b1, void* d_out,
                                  uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                                  uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll, unsigned long long* d_long_key,
                                  unsigned long long* d_staged, hipStream_t stream, void* d_rows) {
  if (n_rows <= 0) return hipSuccess;
  if (b1 < 1 || b1 > kStageBinBits || (packed && !one_string)) return hipErrorInvalidValue;
  const int64_t tiles = (n_rows + kStageTile - 1) / kStageTile;
  int dev = 0, cus = 256, per_cu = 2;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (d_rows) {  // row-order staging, then the level-1 split over the rows (dq_freq_stage_rows_kernel)
    if (packed)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_rows_kernel<true, true>, kStageThreads, 0);
    else if (one_string)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_rows_kernel<true, false>, kStageThreads, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_rows_kernel<false, false>, kStageThreads, 0);
    const int64_t resident = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
    const int64_t blocks = tiles < resident ? tiles : resident;
    if (packed)
      hipLaunchKernelGGL((dq_freq_stage_rows_kernel<true, true>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                         d_cols, n_rows, static_cast<uint64_t*>(d_rows), d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll,
                         d_long_key, d_staged);
    else if (one_string)
      hipLaunchKernelGGL((dq_freq_stage_rows_kernel<true, false>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                         d_cols, n_rows, static_cast<FreqRec*>(d_rows), d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll,
                         d_long_key, d_staged);
    else
      hipLaunchKernelGGL((dq_freq_stage_rows_kernel<false, false>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                         d_cols, n_rows, static_cast<FreqRec*>(d_rows), d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll,
                         d_long_key, d_staged);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_freq_part(d_rows, (uint64_t)n_rows, nullptr, 0, 0, b1, b1, d_out, cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap,
                            d_flag, packed, stream, d_staged);
  }
  // one resident round of workgroups (grid-stride over the tiles)
  if (packed)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_part_kernel<true, true>, kStageThreads, 0);
  else if (one_string)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_part_kernel<true, false>, kStageThreads, 0);
  else
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_part_kernel<false, false>, kStageThreads, 0);
  const int64_t resident = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  const int64_t blocks = tiles < resident ? tiles : resident;
#ifdef DQ_STAGE_PROF
  {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stage_prof), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
  }
#endif
  if (packed)
    hipLaunchKernelGGL((dq_freq_stage_part_kernel<true, true>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                       d_cols, n_rows, b1, static_cast<uint64_t*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag,
                       d_hll, d_long_key, d_staged);
  else if (one_string)
    hipLaunchKernelGGL((dq_freq_stage_part_kernel<true, false>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                       d_cols, n_rows, b1, static_cast<FreqRec*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag,
                       d_hll, d_long_key, d_staged);
  else
    hipLaunchKernelGGL((dq_freq_stage_part_kernel<false, false>), dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks,
                       d_cols, n_rows, b1, static_cast<FreqRec*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag,
                       d_hll, d_long_key, d_staged);
#ifdef DQ_STAGE_PROF
  {
    unsigned long long z[8];
    (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_stage_prof), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    const double tiles_d = (double)tiles;
    {
      std::vector<unsigned long long> bt((size_t)std::min<int64_t>(blocks, 4096) * 2);
      (void)hipMemcpyFromSymbol(bt.data(), HIP_SYMBOL(g_stage_blk), bt.size() * sizeof(unsigned long long), 0,
                                hipMemcpyDeviceToHost);
      unsigned long long lo = ~0ull, hi = 0, sum = 0;
      for (size_t b = 0; b < bt.size() / 2; ++b) {
        lo = std::min(lo, bt[2 * b]);
        hi = std::max(hi, bt[2 * b + 1]);
        sum += bt[2 * b + 1] - bt[2 * b];
      }
      std::fprintf(stderr, "[stage_prof] workgroups: span %.1f us, mean life %.1f us, mean concurrency %.1f\n",
                   (hi - lo) / 100.0, sum / 100.0 / (double)(bt.size() / 2), (double)sum / (double)(hi - lo));
    }
    std::fprintf(stderr, "[stage_prof] rows %lld tiles %lld blocks %lld ns/tile (100 MHz wall clock): own-loads+compute %.0f "
                 "wait-others %.0f rank %.0f scan %.0f reserve %.0f lds-scatter %.0f write %.0f\n",
                 (long long)n_rows, (long long)tiles, (long long)blocks, 10 * z[0] / tiles_d, 10 * z[1] / tiles_d,
                 10 * z[2] / tiles_d, 10 * z[3] / tiles_d, 10 * z[4] / tiles_d, 10 * z[5] / tiles_d, 10 * z[6] / tiles_d);
  }
#endif
  return hipGetLastError();
}

hipError_t launch_freq_compact(const void* d_in, bool packed, const unsigned long long* d_fill, uint64_t cap,
                               uint64_t n_regions, const unsigned long long* d_prefix, FreqRec* d_out, hipStream_t stream) {
  if (n_regions == 0) return hipSuccess;
  if (n_regions > 65535) return hipErrorInvalidValue;
  uint64_t bx = (cap + kBlock * 8 - 1) / (kBlock * 8);
  if (bx > 64) bx = 64;
  if (bx < 1) bx = 1;
  if (packed)
    hipLaunchKernelGGL(dq_freq_compact_kernel<uint64_t>, dim3((unsigned)bx, (unsigned)n_regions), dim3(kBlock), 0, stream,
                       static_cast<const uint64_t*>(d_in), d_fill, cap, d_prefix, d_out);
  else
    hipLaunchKernelGGL(dq_freq_compact_kernel<FreqRec>, dim3((unsigned)bx, (unsigned)n_regions), dim3(kBlock), 0, stream,
                       static_cast<const FreqRec*>(d_in), d_fill, cap, d_prefix, d_out);
  return hipGetLastError();
}

// 16-byte records into a fresh table take dq_freq_agg_keys_kernel<FreqRec> (round 6);
// DQ_FREQ_AGG16=0 keeps dq_freq_agg_region_kernel (A/B knob).
static const bool g_agg_keys_free = [] {
  const char* e = std::getenv("DQ_FREQ_AGG16");
  return e == nullptr || e[0] != '0';
}();

hipError_t launch_freq_agg_region(const FreqTable& T, const void* d_recs, int rec_kind, const unsigned long long* d_fill,
                                  uint64_t cap, uint64_t n_slices, int table_empty, FreqRec* d_retry,
                                  unsigned long long* d_n_retry, unsigned long long* d_new_groups,
                                  unsigned long long* d_hist, unsigned long long* d_big, unsigned long long* d_n_big,
                                  unsigned long long big_cap, uint32_t* d_smax, int write_all, hipStream_t stream,
                                  const FreqCompact* compact) {
  uint64_t blocks = n_slices < 65536 ? n_slices : 65536;
  if (blocks < 1) blocks = 1;
  if (!table_empty && (d_hist || d_smax || write_all)) return hipErrorInvalidValue;
  const bool packed = rec_kind == kRecPacked;
  if (compact && !table_empty) return hipErrorInvalidValue;
  if ((rec_kind == kRecHashed || rec_kind == kRecUuid || rec_kind == kRecRaw16) && !table_empty)
    return hipErrorInvalidValue;  // (fresh tables only)
  AggTrack tr{d_hist, d_big, d_n_big, big_cap, d_smax, write_all, compact ? *compact : FreqCompact{}};
  if (rec_kind == kRecUuid)
    hipLaunchKernelGGL(dq_freq_agg_keys_kernel<UuidRec>, dim3((unsigned)blocks), dim3(kAggUThreads), 0, stream, T,
                       static_cast<const UuidRec*>(d_recs), d_fill, cap, n_slices, d_retry, d_n_retry, d_new_groups, tr);
  else if (rec_kind == kRecRaw16)
    hipLaunchKernelGGL(dq_freq_agg_keys_kernel<Raw16Rec>, dim3((unsigned)blocks), dim3(kAggUThreads), 0, stream, T,
                       static_cast<const Raw16Rec*>(d_recs), d_fill, cap, n_slices, d_retry, d_n_retry, d_new_groups, tr);
  else if (rec_kind == kRecFree && table_empty && g_agg_keys_free)
    hipLaunchKernelGGL(dq_freq_agg_keys_kernel<FreqRec>, dim3((unsigned)blocks), dim3(kAggUThreads), 0, stream, T,
                       static_cast<const FreqRec*>(d_recs), d_fill, cap, n_slices, d_retry, d_n_retry, d_new_groups, tr);
  else if (rec_kind == kRecHashed)
    hipLaunchKernelGGL(dq_freq_agg_hashed_kernel, dim3((unsigned)blocks), dim3(kAggHThreads), 0, stream, T,
                       static_cast<const HashRec*>(d_recs), d_fill, cap, n_slices, d_retry, d_n_retry, d_new_groups, tr);
  else if (packed)
    hipLaunchKernelGGL(dq_freq_agg_packed_kernel, dim3((unsigned)blocks), dim3(kAggPThreads), 0, stream, T,
                       static_cast<const uint64_t*>(d_recs), d_fill, cap, n_slices, table_empty, d_retry, d_n_retry,
                       d_new_groups, tr);
  else
    hipLaunchKernelGGL(dq_freq_agg_region_kernel, dim3((unsigned)blocks), dim3(kAggRegionThreads), 0, stream, T,
                       static_cast<const FreqRec*>(d_recs), d_fill, cap, n_slices, table_empty, d_retry, d_n_retry,
                       d_new_groups, tr);
  return hipGetLastError();
}

hipError_t launch_freq_stage_uuid(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, int b1, void* d_out,
                                  uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                                  uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll, unsigned long long* d_bad,
                                  unsigned long long* d_staged, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  if (b1 < 1 || b1 > kStageBinBits) return hipErrorInvalidValue;
  const int64_t tiles = (n_rows + kUuidTile - 1) / kUuidTile;
  int dev = 0, cus = 256, per_cu = 2;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_uuid_kernel, kStageThreads, 0);
  const int64_t resident = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  const int64_t blocks = tiles < resident ? tiles : resident;  // (one resident round, grid-stride over the tiles)
  hipLaunchKernelGGL(dq_freq_stage_uuid_kernel, dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks, d_cols, n_rows,
                     b1, static_cast<UuidRec*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll, d_bad,
                     d_staged);
  return hipGetLastError();
}

hipError_t launch_freq_uuid_to_hashed(const FreqTable& T, FreqRec* d_recs, uint64_t n, hipStream_t stream, int rec_kind) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 65536) blocks = 65536;
  if (rec_kind == kRecRaw16)
    hipLaunchKernelGGL(dq_freq_uuid_to_hashed_kernel<false>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_recs, n);
  else
    hipLaunchKernelGGL(dq_freq_uuid_to_hashed_kernel<true>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_recs, n);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void dq_freq_len_probe_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                   int64_t n_rows, unsigned long long* out) {
  constexpr int64_t kProbe = 16384;  // (as kPackProbe)
  const int64_t samples = n_rows < kProbe ? n_rows : kProbe;
  uint32_t longer = 0u;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < samples; i += (int64_t)gridDim.x * kBlock) {
    const int64_t row = samples == n_rows ? i : (int64_t)(((uint64_t)i * 11400714819323198485ull) % (uint64_t)n_rows);
    uint32_t n;
    if (key_len_of(ks, cols, row, &n) && n > 15u) ++longer;
  }
  if (longer) atomicAdd(out, (unsigned long long)longer);
}

hipError_t launch_freq_len_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                 hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_freq_len_probe_kernel, dim3((16384 + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, ks, d_cols,
                     n_rows, d_out);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void dq_freq_len16_probe_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                     int64_t n_rows, unsigned long long* out) {
  const DevColumn& c = cols[ks.key_cols[0]];
  constexpr int64_t kProbe = 16384;  // (as kPackProbe)
  const int64_t samples = n_rows < kProbe ? n_rows : kProbe;
  uint32_t other = 0u;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < samples; i += (int64_t)gridDim.x * kBlock) {
    const int64_t row = samples == n_rows ? i : (int64_t)(((uint64_t)i * 11400714819323198485ull) % (uint64_t)n_rows);
    if (c.validity != nullptr && !((c.validity[row >> 3] >> (row & 7)) & 1u)) continue;
    if (c.offsets[row + 1] - c.offsets[row] != 16) ++other;
  }
  if (other) atomicAdd(out, (unsigned long long)other);
}

hipError_t launch_freq_len16_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                   unsigned long long* d_out, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_freq_len16_probe_kernel, dim3((16384 + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, ks, d_cols,
                     n_rows, d_out);
  return hipGetLastError();
}

hipError_t launch_freq_stage_raw16(const FreqKeySpec& ks, bool one_string, const DevColumn* d_cols, int64_t n_rows,
                                   int b1, void* d_out, uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf,
                                   unsigned long long* d_ovf_n, uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll,
                                   unsigned long long* d_bad, unsigned long long* d_staged, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  if (b1 < 1 || b1 > kStageBinBits || (!one_string && ks.n_keys != 2)) return hipErrorInvalidValue;
  const int64_t tiles = (n_rows + kUuidTile - 1) / kUuidTile;
  int dev = 0, cus = 256, per_cu = 2;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (one_string)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_raw16_kernel<true>, kStageThreads, 0);
  else
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dq_freq_stage_raw16_kernel<false>, kStageThreads, 0);
  const int64_t resident = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  const int64_t blocks = tiles < resident ? tiles : resident;
  if (one_string)
    hipLaunchKernelGGL(dq_freq_stage_raw16_kernel<true>, dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks, d_cols,
                       n_rows, b1, static_cast<Raw16Rec*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll,
                       d_bad, d_staged);
  else
    hipLaunchKernelGGL(dq_freq_stage_raw16_kernel<false>, dim3((unsigned)blocks), dim3(kStageThreads), 0, stream, ks, d_cols,
                       n_rows, b1, static_cast<Raw16Rec*>(d_out), cap1, d_fill1, d_ovf, d_ovf_n, ovf_cap, d_flag, d_hll,
                       d_bad, d_staged);
  return hipGetLastError();
}

hipError_t launch_freq_uuid_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                  hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_freq_uuid_probe_kernel, dim3((16384 + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, ks, d_cols,
                     n_rows, d_out);
  return hipGetLastError();
}

hipError_t launch_freq_expand(const FreqTable& T, const FreqCompact& cmp, hipStream_t stream) {
  const uint64_t n_slices = (T.mask + 1) >> kFreqSliceLog;
  uint64_t blocks = n_slices < 65536 ? n_slices : 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_expand_kernel, dim3((unsigned)blocks), dim3(kAggPThreads), 0, stream, T, cmp, n_slices);
  return hipGetLastError();
}

// The heap bytes of exported groups (ctrl / k0 as launch_freq_export writes them) gathered to
// dst at off[i] (heap keys only): a top-N export of a table whose heap holds every row's key (the
// hashed path) moves its few keys, not the whole heap.
__global__ __launch_bounds__(kBlock) void dq_freq_gather_keys_kernel(const uint8_t* __restrict__ heap,
                                                                     const unsigned long long* __restrict__ ctrl,
                                                                     const unsigned long long* __restrict__ k0,
                                                                     const unsigned long long* __restrict__ off,
                                                                     uint64_t n, uint8_t* __restrict__ dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const unsigned long long c = ctrl[i];
    if (!(c & kHeapKey)) continue;
    const uint32_t words = (uint32_t)(((c & kLenMask) + 7ull) >> 3);
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(heap + k0[i]);
    unsigned long long* d = reinterpret_cast<unsigned long long*>(dst + off[i]);
    for (uint32_t w = 0; w < words; ++w) d[w] = src[w];
  }
}

hipError_t launch_freq_gather_keys(const uint8_t* d_heap, const unsigned long long* d_ctrl, const unsigned long long* d_k0,
                                   const unsigned long long* d_off, uint64_t n, uint8_t* d_dst, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_freq_gather_keys_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, d_heap, d_ctrl, d_k0,
                     d_off, n, d_dst);
  return hipGetLastError();
}

hipError_t launch_freq_key_bytes(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                 unsigned long long* d_out, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + kBlock * 8 - 1) / (kBlock * 8);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_freq_key_bytes_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols, n_rows, d_out);
  return hipGetLastError();
}

// Multi-column keys take dq_freq_stage_hashed_multi_kernel; DQ_FREQ_HSTAGE=unrolled the round's
// first (unrolled) body (A/B knob).
static const bool g_hstage_unrolled = [] {
  const char* e = std::getenv("DQ_FREQ_HSTAGE");
  return e != nullptr && std::strcmp(e, "unrolled") == 0;
}();

hipError_t launch_freq_stage_hashed(const FreqKeySpec& ks, bool one_string, const DevColumn* d_cols, int64_t n_rows, HashRec* d_out,
                                    const FreqTable& T, uint32_t* d_hll, unsigned long long* d_too_long,
                                    unsigned long long* d_staged, unsigned long long* d_max_len, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + kHashTile - 1) / kHashTile;
  if (blocks > 8192) blocks = 8192;
  if (one_string)
    hipLaunchKernelGGL(dq_freq_stage_hashed_kernel<true>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols,
                       n_rows, d_out, T, d_hll, d_too_long, d_staged, d_max_len);
  else if (g_hstage_unrolled)
    hipLaunchKernelGGL(dq_freq_stage_hashed_kernel<false>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols,
                       n_rows, d_out, T, d_hll, d_too_long, d_staged, d_max_len);
  else
    hipLaunchKernelGGL(dq_freq_stage_hashed_multi_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols,
                       n_rows, d_out, T, d_hll, d_too_long, d_staged, d_max_len);
  return hipGetLastError();
}

hipError_t launch_freq_insert_hashed(const FreqTable& T, const FreqRec* d_recs, uint64_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t chunk = 64ull * kAggHThreads;
  uint64_t blocks = (n + chunk - 1) / chunk;
  if (blocks > 2ull * (uint64_t)cus) blocks = 2ull * (uint64_t)cus;  // (each workgroup flushes its image once at the end)
  hipLaunchKernelGGL(dq_freq_insert_hashed_kernel, dim3((unsigned)blocks), dim3(kAggHThreads), 0, stream, T, d_recs, n);
  return hipGetLastError();
}

hipError_t launch_freq_export_compact(const FreqCompact& cmp, uint64_t n_slices, unsigned long long min_count,
                                      const FreqOut& out, const uint32_t* d_smax, hipStream_t stream) {
  uint64_t blocks = n_slices < 16384 ? n_slices : 16384;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_export_compact_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, cmp, n_slices,
                     min_count, d_smax, out);
  return hipGetLastError();
}

hipError_t launch_freq_rehash(const FreqSlot* d_old, uint64_t old_n, const FreqTable& T, hipStream_t stream) {
  uint64_t blocks = (old_n + kBlock * 8 - 1) / (kBlock * 8);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_rehash_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, d_old, old_n, T);
  return hipGetLastError();
}

// Bytes of long (> 16 B) single-string keys in a batch: the key heap is grown to fit first.
__global__ __launch_bounds__(kBlock) void dq_freq_heap_need_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                   int64_t n_rows, unsigned long long* need,
                                                                   unsigned long long* max_len) {
  unsigned long long local = 0;
  unsigned int longest = 0;
  for (int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x; row < n_rows; row += (int64_t)gridDim.x * kBlock) {
    uint32_t n = 0;
    bool any_null = false;
    for (int i = 0; i < ks.n_keys; ++i) {
      const DevColumn& c = cols[ks.key_cols[i]];
      if (!col_valid(c, row)) {
        any_null = true;
        continue;
      }
      if (c.type == DQ_T_UTF8) n += (uint32_t)(c.offsets[row + 1] - c.offsets[row]) + (ks.n_keys > 1 ? 4u : 0u);
      else n += (uint32_t)width_of(c.type);
    }
    if (any_null && !(ks.null_as_key && ks.n_keys == 1)) n = 0;
    if (any_null && ks.null_as_key && ks.n_keys == 1 && cols[ks.key_cols[0]].type == DQ_T_UTF8) n = 9;  // "NullValue"
    if (n > 16) local += (n + 7u) & ~7u;
    longest = n > longest ? n : longest;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    local += __shfl_down(local, d, 64);
    const unsigned int o = __shfl_down(longest, d, 64);
    longest = o > longest ? o : longest;
  }
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(need, local);
  if ((threadIdx.x & 63) == 0 && longest) atomicMax(max_len, (unsigned long long)longest);
}

hipError_t launch_freq_insert(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                              const FreqTable& T, hipStream_t stream, int max_blocks) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + 4095) / 4096;
  if (blocks > max_blocks) blocks = max_blocks;
  hipLaunchKernelGGL(dq_freq_insert_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols,
                     n_rows, T);
  return hipGetLastError();
}

hipError_t launch_freq_hist(const FreqTable& T, unsigned long long* d_hist, unsigned long long* d_big,
                            unsigned long long* d_nbig, unsigned long long big_cap, hipStream_t stream) {
  const uint64_t n = T.mask + 1;
  uint64_t blocks = (n + kBlock * 16 - 1) / (kBlock * 16);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_hist_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_hist, d_big,
                     d_nbig, big_cap);
  return hipGetLastError();
}

hipError_t launch_freq_export(const FreqTable& T, unsigned long long min_count, const FreqOut& out,
                              hipStream_t stream, const uint32_t* d_smax) {
  if (d_smax && min_count > 0) {
    const uint64_t n_slices = (T.mask + 1) >> kFreqSliceLog;
    const uint64_t blocks = n_slices < 16384 ? n_slices : 16384;
    hipLaunchKernelGGL(dq_freq_export_slices_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, min_count,
                       d_smax, out);
    return hipGetLastError();
  }
  const uint64_t n = T.mask + 1;
  uint64_t blocks = (n + kBlock * 16 - 1) / (kBlock * 16);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dq_freq_export_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, min_count, out);
  return hipGetLastError();
}

// Diagnostics: the table hash and the packed word (or ~0) of n inline keys (tests compare them
// with a host restatement: every path must place a key with this one function).
__global__ __launch_bounds__(kBlock) void dq_freq_hash_kernel(const uint64_t* __restrict__ k0, const uint64_t* __restrict__ k1,
                                                              const uint32_t* __restrict__ len, int64_t n, uint64_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    uint64_t p;
    const uint64_t h = hash_inline(k0[i], k1[i], len[i]);
    const bool pk = kp_pack_record(k0[i], k1[i], len[i], &p);
    // (a packed record must hash like its key: a disagreement shows up as a wrong hash)
    out[2 * i] = pk && hash_record_packed(p) != h ? ~h : h;
    out[2 * i + 1] = pk ? p : ~0ull;
  }
}

hipError_t launch_freq_hash(const uint64_t* d_k0, const uint64_t* d_k1, const uint32_t* d_len, int64_t n, uint64_t* d_out,
                            hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_freq_hash_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, d_k0, d_k1, d_len, n, d_out);
  return hipGetLastError();
}

hipError_t launch_freq_lookup(const FreqTable& T, const uint8_t* d_key, uint32_t len, unsigned long long* d_out,
                              hipStream_t stream, const FreqCompact* cmp) {
  hipLaunchKernelGGL(dq_freq_lookup_kernel, dim3(1), dim3(64), 0, stream, T, d_key, len, d_out,
                     cmp ? *cmp : FreqCompact{});
  return hipGetLastError();
}

uint64_t freq_flat_chunks(uint64_t slots) { return (slots + kFlatChunk - 1) / kFlatChunk; }

hipError_t launch_freq_flat_count(const FreqTable& T, unsigned long long* d_chunk_n, uint64_t n_chunks,
                                  unsigned long long* d_sums, hipStream_t stream) {
  if (n_chunks == 0 || n_chunks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dq_flat_count_kernel, dim3((unsigned)n_chunks), dim3(kBlock), 0, stream, T, d_chunk_n, n_chunks);
  return exclusive_scan<unsigned long long>(d_chunk_n, n_chunks + 1, d_sums, stream);
}

hipError_t launch_freq_flat_fill(const FreqTable& T, const unsigned long long* d_chunk_base, uint64_t n_chunks, uint64_t n,
                                 unsigned long long* d_ctrl, unsigned long long* d_count, unsigned long long* d_k0,
                                 unsigned long long* d_k1, unsigned long long* d_offs, unsigned long long* d_sums,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(dq_flat_fill_kernel, dim3((unsigned)n_chunks), dim3(kBlock), 0, stream, T, d_chunk_base, n, d_ctrl,
                     d_count, d_k0, d_k1, d_offs);
  return exclusive_scan<unsigned long long>(d_offs, n + 1, d_sums, stream);
}

hipError_t launch_freq_flat_keys(const FreqTable& T, const unsigned long long* d_ctrl, const unsigned long long* d_k0,
                                 const unsigned long long* d_k1, const unsigned long long* d_offs, uint64_t n,
                                 uint8_t* d_out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(dq_flat_keys_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_ctrl, d_k0, d_k1, d_offs,
                     n, d_out);
  return hipGetLastError();
}

hipError_t launch_freq_import_flat(const FreqTable& T, const long long* d_counts, const long long* d_offs,
                                   const uint8_t* d_bytes, uint64_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock * 4 - 1) / (kBlock * 4);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(dq_freq_import_flat_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, d_counts, d_offs,
                     d_bytes, n);
  return hipGetLastError();
}

hipError_t launch_freq_import(const FreqTable& T, const FreqIn& in, hipStream_t stream) {
  if (in.n == 0) return hipSuccess;
  uint64_t blocks = (in.n + kBlock * 4 - 1) / (kBlock * 4);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(dq_freq_import_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, T, in);
  return hipGetLastError();
}

hipError_t launch_freq_heap_need(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                 unsigned long long* d_need, unsigned long long* d_max_len, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + kBlock * 16 - 1) / (kBlock * 16);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_freq_heap_need_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, ks, d_cols,
                     n_rows, d_need, d_max_len);
  return hipGetLastError();
}


// =============================================================================================
// Key-hash exchange and table merges (round 4): FrequenciesAndNumRows.sum as an outer join of
// two key sets (GroupingAnalyzers.scala:128-148) and the groupBy's hash exchange (:67-72).
//
// Sender: dq_freq_partition writes each owner's groups as a part = [packed records, 16 B:
// {packed key word, count} for keys that pack (dq_keypack.h)] [general records, 32 B: FreqSlot
// with READY clear, k0 of a long key = offset in the part's key bytes], each section in the
// order of the sender's slice chunks (2^chunk_log slices per chunk, chunk_log = 0 unless parts x
// chunks would be too many counters).  A slice is a range of the top hash bits, so a receiver
// whose table has no more slice bits than the sender finds the records of each of its slices
// contiguous in every part -- no sort, no per-group atomics.
//
// Receiver (dq_freq_import_parts / dq_freq_merge): every record stream ("run": a part's packed
// section, its general section, or a whole source table's slot array) is
//   1. sketched (HLL p = 9 of the record hashes) to size the table,
//   2. cut at the receiver's slice boundaries (dq_import_bounds_kernel: start / end per (run,
//      slice), one streaming pass; a run found out of order is flagged and imported group by
//      group instead),
//   3. merged by ONE workgroup per receiver slice (dq_import_merge_kernel): the slice is loaded
//      into an LDS image (or starts empty), every run's records of that slice are counted in with
//      their weights, and the slice is written back whole -- the slice-owner aggregation of the
//      partition path, with weighted records.
// Records whose keys do not fit the LDS image (longer than 15 bytes) and runs out of slice order
// take dq_import_global_kernel (global_insert, per group); a slice whose keys overflow the image
// is left untouched and listed, the table grows, and its records are inserted group by group.
// =============================================================================================

// A group's hash, packed word and class: 0 = its key packs (a packed wire record), 1 = general.
__device__ inline uint64_t slot_key_hash(const FreqTable& T, const FreqSlot& e, uint32_t len, uint64_t* packed,
                                         int* kind) {
  *kind = 1;
  if (e.ctrl & kHeapKey) return hash_long(T.heap + e.k0, len);
  uint64_t p;
  if (kp_pack_record(e.k0, e.k1, len, &p)) {
    *packed = p;
    *kind = 0;
    return hash_record_packed(p);
  }
  return hash_raw(e.k0, e.k1, len);
}

constexpr int kWireThreads = 256;
constexpr int kWireMaxParts = 4096;

// Counts per (part, kind, chunk) -- cnt[(2 p + kind) * n_chunks + chunk] -- and long-key bytes per
// part.  One chunk per workgroup iteration (LDS counters, written out whole).
__global__ __launch_bounds__(kWireThreads) void dq_wire_count_kernel(FreqTable T, int n_parts, int chunk_log,
                                                                     uint64_t n_chunks, unsigned long long* cnt,
                                                                     unsigned long long* kbytes) {
  __shared__ uint32_t c_l[2 * kWireMaxParts];
  const uint32_t np2 = 2u * (uint32_t)n_parts;
  for (uint32_t i = threadIdx.x; i < np2; i += kWireThreads) c_l[i] = 0u;
  __syncthreads();
  const uint64_t per = (uint64_t)kFreqSliceSlots << chunk_log;
  for (uint64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    for (uint64_t s = c * per + threadIdx.x; s < (c + 1) * per; s += kWireThreads) {
      const FreqSlot e = T.slots[s];  // launch boundary: every insert is visible
      if (!(e.ctrl & kReady)) continue;
      const uint32_t len = (uint32_t)(e.ctrl & kLenMask);
      uint64_t pk;
      int kind;
      const uint64_t h = slot_key_hash(T, e, len, &pk, &kind);
      const uint32_t o = freq_owner(h, (uint32_t)n_parts);
      atomicAdd(&c_l[2 * o + kind], 1u);
      if (e.ctrl & kHeapKey) atomicAdd(&kbytes[o], ((unsigned long long)len + 7ull) & ~7ull);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < np2; i += kWireThreads) {
      cnt[(uint64_t)i * n_chunks + c] = c_l[i];
      c_l[i] = 0u;
    }
    __syncthreads();
  }
}

// out[i] = scanned[i * stride] for i <= n (section starts of the scanned counts).
__global__ void dq_gather_strided_kernel(const unsigned long long* __restrict__ scanned, uint64_t stride, uint64_t n,
                                         unsigned long long* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = scanned[i * stride];
}

// sec[4 p ..]: {byte offset of part p in out, first packed index, first general index, packed
// records of p}; pos = the exclusive scan of dq_wire_count_kernel's counts.
__global__ __launch_bounds__(kWireThreads) void dq_wire_scatter_kernel(FreqTable T, int n_parts, int chunk_log,
                                                                       uint64_t n_chunks,
                                                                       const unsigned long long* __restrict__ pos,
                                                                       const unsigned long long* __restrict__ sec,
                                                                       const unsigned long long* __restrict__ key_base,
                                                                       unsigned long long* key_cursor, uint8_t* out,
                                                                       uint8_t* keys) {
  __shared__ uint32_t c_l[2 * kWireMaxParts];
  const uint32_t np2 = 2u * (uint32_t)n_parts;
  for (uint32_t i = threadIdx.x; i < np2; i += kWireThreads) c_l[i] = 0u;
  __syncthreads();
  const uint64_t per = (uint64_t)kFreqSliceSlots << chunk_log;
  for (uint64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    for (uint64_t s = c * per + threadIdx.x; s < (c + 1) * per; s += kWireThreads) {
      FreqSlot e = T.slots[s];
      if (!(e.ctrl & kReady)) continue;
      const uint32_t len = (uint32_t)(e.ctrl & kLenMask);
      uint64_t pk = 0;
      int kind;
      const uint64_t h = slot_key_hash(T, e, len, &pk, &kind);
      const uint32_t o = freq_owner(h, (uint32_t)n_parts);
      const uint32_t k = 2u * o + (uint32_t)kind;
      const unsigned long long idx = pos[(uint64_t)k * n_chunks + c] + atomicAdd(&c_l[k], 1u);
      const unsigned long long* q = sec + 4 * o;
      if (kind == 0) {
        WirePacked w;
        w.key = pk;
        w.count = e.count;
        *reinterpret_cast<WirePacked*>(out + q[0] + 16ull * (idx - q[1])) = w;
      } else {
        if (e.ctrl & kHeapKey) {
          const unsigned long long bytes = ((unsigned long long)len + 7ull) & ~7ull;
          const unsigned long long off = atomicAdd(&key_cursor[o], bytes);  // within part o's key bytes
          const uint64_t* src = reinterpret_cast<const uint64_t*>(T.heap + e.k0);
          uint64_t* dst = reinterpret_cast<uint64_t*>(keys + key_base[o] + off);
          for (unsigned long long w = 0; w < bytes / 8; ++w) dst[w] = src[w];
          e.k0 = off;
        }
        e.ctrl &= ~kReady;  // wire form: READY is a table-internal flag
        *reinterpret_cast<FreqSlot*>(out + q[0] + 16ull * q[3] + 32ull * (idx - q[2])) = e;
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < np2; i += kWireThreads) c_l[i] = 0u;
    __syncthreads();
  }
}

// ---- receiver (ImportRun: dq_internal.h)
// One record of a run, decoded: present (a group), its weight, hash, and -- when it fits the LDS
// image (a key of <= 15 bytes) -- its key as k0 / k1 (length in k1's top byte) or packed word.
struct ImpRec {
  uint64_t k0, k1, p, hash;  // k1: the key's bytes 8..15 (the LDS image adds the length byte)
  unsigned long long count;
  uint32_t len;
  bool present, lds_ok, heap;
};

template <bool PACKED>
__device__ inline void imp_load(const ImportRun& R, uint64_t i, ImpRec& r) {
  if (R.kind == 0) {
    const WirePacked w = static_cast<const WirePacked*>(R.recs)[i];
    r.p = w.key;
    r.count = w.count;
    r.present = true;
    r.lds_ok = true;
    r.heap = false;
    r.hash = hash_record_packed(w.key);
    if constexpr (!PACKED) {
      uint64_t k0, k1;
      uint32_t len;
      kp_unpack(w.key, &k0, &k1, &len);
      r.k0 = k0;
      r.k1 = k1;
      r.len = len;
    }
    return;
  }
  const FreqSlot e = static_cast<const FreqSlot*>(R.recs)[i];
  r.present = R.kind == 1 || (e.ctrl & kReady);
  r.count = e.count;
  r.len = (uint32_t)(e.ctrl & kLenMask);
  r.heap = (e.ctrl & kHeapKey) != 0;
  r.lds_ok = !r.heap && r.len <= 15;
  r.k0 = e.k0;
  r.k1 = e.k1;
  r.p = 0;
  if (!r.present) return;
  r.hash = r.heap ? hash_long(R.heap + e.k0, r.len) : hash_inline(e.k0, e.k1, r.len);
}

__device__ inline uint64_t dst_slice(uint64_t h, int rb) { return rb ? (h >> (64 - rb)) : 0ull; }

// The record range of run R for receiver slice r (rb slice bits): kind 2 from the source table's
// geometry, wire runs from the bounds pass.
__device__ inline void imp_range(const ImportRun& R, int run, uint64_t r, int rb, const uint32_t* start,
                                 const uint32_t* end, uint64_t n_slices, uint64_t* b, uint64_t* e) {
  if (R.kind == 2) {
    if (rb <= R.src_bits) {
      const int sh = R.src_bits - rb + kFreqSliceLog;
      *b = r << sh;
      *e = (r + 1) << sh;
    } else {
      const uint64_t sl = r >> (rb - R.src_bits);
      *b = sl << kFreqSliceLog;
      *e = (sl + 1) << kFreqSliceLog;
    }
    return;
  }
  const uint64_t q = R.bits < rb ? r >> (rb - R.bits) : r;  // (coarser bounds: the enclosing range)
  *b = start[(uint64_t)run * n_slices + q];
  *e = end[(uint64_t)run * n_slices + q];
}

// HLL p = 9 of every present record's hash (table sizing).
__global__ __launch_bounds__(kBlock) void dq_import_sketch_kernel(const ImportRun* __restrict__ runs, uint32_t* hll) {
  __shared__ uint32_t regs[kHllM];
  for (int i = threadIdx.x; i < kHllM; i += kBlock) regs[i] = 0u;
  __syncthreads();
  const ImportRun R = runs[blockIdx.y];
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < R.n; i += (uint64_t)gridDim.x * kBlock) {
    ImpRec r;
    imp_load<false>(R, i, r);
    if (r.present) sketch_update(regs, r.hash);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHllM; i += kBlock)
    if (regs[i]) atomicMax(&hll[i], regs[i]);
}

// Slice boundaries of each wire run (blockIdx.y) at its R.bits slice bits: start[run][r] /
// end[run][r] (both 0 for a slice the run does not hold); unsorted[run] = 1 if the run is not in
// order at those bits -- then drop[run] = the fewest top bits to drop for it to be in order (the
// largest depth, below R.bits, at which two adjacent records' slices first differ the wrong way).
// rerun: only the runs whose bits were lowered (R.bits < rb) are cut again.
__global__ __launch_bounds__(kBlock) void dq_import_bounds_kernel(const ImportRun* __restrict__ runs, int rb,
                                                                  uint64_t n_slices, uint32_t* start, uint32_t* end,
                                                                  unsigned int* unsorted, unsigned int* drop, int rerun) {
  const int run = blockIdx.y;
  const ImportRun R = runs[run];
  if (R.kind == 2 || (rerun && R.bits >= rb)) return;
  const int g = R.bits;
  uint32_t* st = start + (uint64_t)run * n_slices;
  uint32_t* en = end + (uint64_t)run * n_slices;
  unsigned int worst = 0u;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < R.n; i += (uint64_t)gridDim.x * kBlock) {
    ImpRec r, q;
    imp_load<true>(R, i, r);
    const uint64_t si = dst_slice(r.hash, g);
    if (i == 0) {
      st[si] = 0u;
    } else {
      imp_load<true>(R, i - 1, q);
      const uint64_t sp = dst_slice(q.hash, g);
      if (sp != si) {
        if (sp > si) {  // equal top bits: clz of the difference within the g-bit slice number
          const unsigned int same = (unsigned int)(__clzll((long long)(sp ^ si)) - (64 - g));
          worst = max(worst, (unsigned int)g - same);
        }
        st[si] = (uint32_t)i;
        en[sp] = (uint32_t)i;
      }
    }
    if (i + 1 == R.n) en[si] = (uint32_t)R.n;
  }
  if (worst) {
    unsorted[run] = 1u;
    atomicMax(&drop[run], worst);
  }
}

// The LDS image of a receiver slice: PACKED -- one word per slot (the packed key, kPackEmpty or
// kPackForeign); general -- K0 / K1 as the partition path's 16-byte records (kLdsEmpty / kLdsBusy
// / kLdsForeign in K1).  Counts are 64-bit (merged groups carry their weights).
constexpr int kMergeLdsRuns = 64;  // runs whose slice bounds are staged in LDS (more: read per run)
constexpr int kFlatRuns = kImportFlatRuns;  // packed runs merged as one index space (more: run by run)
template <bool PACKED>
struct MergeLds;
template <>
struct MergeLds<true> {
  unsigned long long K[kFreqSliceSlots];
  uint32_t C[kFreqSliceSlots];  // (32-bit: a weight or sum that does not fit fails the slice, see merge_add)
  int overflow;
  uint32_t fresh;
  unsigned long long cmax;
  uint32_t hist[kAggLdsHist];
  unsigned long long rb[kMergeLdsRuns], re[kMergeLdsRuns];  // the slice's record range per run
  uint32_t pe[kFlatRuns];             // (flat path) records of the slice in runs 0..k, inclusive
  unsigned long long fb[kFlatRuns];   // (flat path) address of flat index 0 in run k's records
};
template <>
struct MergeLds<false> {
  unsigned long long K0[kFreqSliceSlots], K1[kFreqSliceSlots];
  unsigned long long C[kFreqSliceSlots];
  int overflow;
  uint32_t fresh;
  unsigned long long cmax;
  uint32_t hist[kAggLdsHist];
  unsigned long long rb[kMergeLdsRuns], re[kMergeLdsRuns];  // the slice's record range per run
};

// Adds weight w to a 32-bit LDS count; false if w or the sum does not fit 32 bits (the slice then
// takes the overflow path: left untouched and its records inserted group by group, 64-bit).
__device__ inline bool merge_add(uint32_t* C, uint32_t s, unsigned long long w) {
  const uint32_t old = atomicAdd(&C[s], (uint32_t)w);
  return (w >> 32) == 0ull && (uint32_t)(old + (uint32_t)w) >= old;
}

// Counts packed key p with weight w into the image, probing from slot s.
__device__ inline bool merge_count_at(MergeLds<true>& L, uint64_t p, unsigned long long w, uint32_t s) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  for (uint32_t probe = 0; probe < S; ++probe) {
    const unsigned long long c = atomicCAS(&L.K[s], kPackEmpty, (unsigned long long)p);
    if (c == kPackEmpty || c == p) return merge_add(L.C, s, w);
    s = (s + 1) & (S - 1);
  }
  return false;
}

__device__ inline bool merge_count(MergeLds<true>& L, const ImpRec& r) {
  return merge_count_at(L, r.p, r.count, (uint32_t)r.hash & (uint32_t)(kFreqSliceSlots - 1));
}

__device__ inline bool merge_count(MergeLds<false>& L, const ImpRec& r) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  const unsigned long long k1 = r.k1 | ((unsigned long long)r.len << kRecLenShift);
  uint32_t s = (uint32_t)r.hash & (S - 1);
  bool done = false;
  for (uint32_t probe = 0; probe < S && !done;) {  // (the publish stays inside the iteration: see lds_count)
    const unsigned long long c = atomicCAS(&L.K1[s], kLdsEmpty, kLdsBusy);
    if (c == kLdsEmpty) {
      L.K0[s] = r.k0;
      __threadfence_block();
      atomicExch(&L.K1[s], k1);
      atomicAdd(&L.C[s], r.count);
      done = true;
    } else if (c == kLdsBusy) {
      // being published by another lane: look again
    } else if (c == k1 && __hip_atomic_load(&L.K0[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == r.k0) {
      atomicAdd(&L.C[s], r.count);
      done = true;
    } else {
      s = (s + 1) & (S - 1);
      ++probe;
    }
  }
  return done;
}

constexpr int kMergeThreads = 256;
#ifndef DQ_IMP_BATCH
#define DQ_IMP_BATCH 4
#endif
constexpr int kImpBatch = DQ_IMP_BATCH;  // records per thread in flight in the import merge

// One workgroup per receiver slice (grid-stride): the slice's LDS image, every run's records of
// the slice counted in with their weights, the slice written back whole.  ovf_list gets the
// slices whose keys did not fit the image (left untouched; zero-filled when write_all).
#ifndef DQ_IMP_WAVES
#define DQ_IMP_WAVES 5
#endif
// FLAT (PACKED only): every run is a packed wire run, at most kFlatRuns of them, none skipped.
template <bool PACKED, bool FLAT>
__global__ __launch_bounds__(kMergeThreads) __attribute__((amdgpu_waves_per_eu(FLAT ? DQ_IMP_WAVES : 1))) void dq_import_merge_kernel(
    FreqTable T, const ImportRun* __restrict__ runs, int n_runs, const uint32_t* __restrict__ start,
    const uint32_t* __restrict__ end, uint64_t n_slices, int table_empty, AggTrack tr, uint32_t* ovf_list,
    unsigned long long* n_ovf, unsigned long long* ovf_recs, unsigned long long* new_groups) {
  constexpr uint32_t S = (uint32_t)kFreqSliceSlots;
  constexpr int NT = kMergeThreads;
  __shared__ MergeLds<PACKED> L;
  const int rb = T.bucket_bits;
  const bool track = tr.hist != nullptr;
  if (track) {
    for (int i = threadIdx.x; i < kAggLdsHist; i += NT) L.hist[i] = 0u;
    lds_barrier();
  }
  static_assert(PACKED || !FLAT, "the flat merge takes packed runs");
  // thread t < n_runs keeps run t's descriptor and fetches its range of the NEXT slice while this
  // one is merged (the bounds' load latency is off the slice's critical path)
  const int my_run = (int)threadIdx.x < n_runs && threadIdx.x < (uint32_t)kMergeLdsRuns ? (int)threadIdx.x : -1;
  ImportRun myR{};
  if (my_run >= 0) myR = runs[my_run];
  uint64_t nx0 = 0, nx1 = 0;
  if (my_run >= 0 && blockIdx.x < n_slices) imp_range(myR, my_run, blockIdx.x, rb, start, end, n_slices, &nx0, &nx1);
  for (uint64_t b = blockIdx.x; b < n_slices; b += gridDim.x) {
    FreqSlot* slice = T.slots + (b << kFreqSliceLog);
    for (uint32_t s = threadIdx.x; s < S; s += NT) {
      bool have = false;
      uint64_t k0 = 0, k1 = 0;
      uint32_t len = 0;
      bool fits = false;
      if (!table_empty) {
        const FreqSlot e = slice[s];
        have = (e.ctrl & kReady) != 0;
        len = (uint32_t)(e.ctrl & kLenMask);
        fits = have && !(e.ctrl & kHeapKey) && len <= 15;
        k0 = e.k0;
        k1 = e.k1;
      }
      if constexpr (PACKED) {
        uint64_t p;
        L.K[s] = !have ? kPackEmpty : (fits && kp_pack_record(k0, k1, len, &p) ? p : kPackForeign);
      } else {
        L.K0[s] = k0;
        L.K1[s] = !have ? kLdsEmpty : (fits ? (k1 | ((unsigned long long)len << kRecLenShift)) : kLdsForeign);
      }
      L.C[s] = 0ull;
    }
    if (threadIdx.x == 0) {
      L.overflow = 0;
      L.fresh = 0u;
      L.cmax = 0ull;
    }
    if (my_run >= 0) {
      L.rb[my_run] = nx0;
      L.re[my_run] = nx1;
      if (b + gridDim.x < n_slices) imp_range(myR, my_run, b + gridDim.x, rb, start, end, n_slices, &nx0, &nx1);
    }
    lds_barrier();
    uint32_t mine = 0;  // this thread's records of the slice (an overflowed slice's key bound)
    if constexpr (FLAT) {
      {
        // every run is a packed wire run: the slice's records of all runs as ONE index space f,
        // kImpBatch per thread loaded together (a run holds only ~1/n_runs of a slice's records,
        // so per-run batches would leave most threads idle per load latency).  Run k holds
        // f in [pe[k-1], pe[k]); its record f sits at fb[k] + 16 f.
        if (threadIdx.x < 64u) {  // wave 0: inclusive scan of the per-run counts
          const int lane = (int)threadIdx.x;
          const uint32_t v = lane < n_runs ? (uint32_t)(L.re[lane] - L.rb[lane]) : 0u;
          uint32_t incl = v;
#pragma unroll
          for (int d = 1; d < kFlatRuns; d <<= 1) {
            const uint32_t u = __shfl_up(incl, (unsigned)d, 64);
            if (lane >= d) incl += u;
          }
          if (lane < kFlatRuns) {
            L.pe[lane] = lane < n_runs ? incl : 0xFFFFFFFFu;
            if (lane < n_runs)
              L.fb[lane] = reinterpret_cast<unsigned long long>(myR.recs) +
                           16ull * (L.rb[lane] - (unsigned long long)(incl - v));
          }
        }
        lds_barrier();
        uint32_t pe[kFlatRuns - 1];
#pragma unroll
        for (int k = 0; k < kFlatRuns - 1; ++k) pe[k] = L.pe[k];
        const uint32_t total = L.pe[n_runs - 1];
        for (uint32_t f0 = threadIdx.x; f0 < total; f0 += (uint32_t)kImpBatch * NT) {
          unsigned long long key[kImpBatch], cnt[kImpBatch];
#pragma unroll
          for (int j = 0; j < kImpBatch; ++j) {
            const uint32_t f = f0 + (uint32_t)j * NT;
            key[j] = kPackEmpty;
            cnt[j] = 0ull;
            if (f < total) {
              uint32_t r = 0;
#pragma unroll
              for (int k = 0; k < kFlatRuns - 1; ++k) r += pe[k] <= f ? 1u : 0u;
              const WirePacked w = *reinterpret_cast<const WirePacked*>(L.fb[r] + 16ull * f);
              key[j] = w.key;
              cnt[j] = w.count;
            }
          }
          // every record's first probe is issued before any result is looked at
          uint32_t sl[kImpBatch];
          unsigned long long cv[kImpBatch];
#pragma unroll
          for (int j = 0; j < kImpBatch; ++j) {
            const uint64_t h = hash_record_packed(key[j]);
            if (key[j] != kPackEmpty && dst_slice(h, rb) != b) key[j] = kPackEmpty;
            sl[j] = (uint32_t)h & (S - 1);
            cv[j] = key[j] != kPackEmpty ? atomicCAS(&L.K[sl[j]], kPackEmpty, key[j]) : 0ull;
          }
#pragma unroll
          for (int j = 0; j < kImpBatch; ++j) {
            if (key[j] == kPackEmpty) continue;
            ++mine;
            if (cv[j] == kPackEmpty || cv[j] == key[j]) {
              if (!merge_add(L.C, sl[j], cnt[j])) L.overflow = 1;
            } else if (!merge_count_at(L, key[j], cnt[j], (sl[j] + 1) & (S - 1))) L.overflow = 1;
          }
        }
      }
    }
    for (int run = 0; run < (FLAT ? 0 : n_runs); ++run) {
      const ImportRun R = runs[run];
      if (R.skip) continue;
      uint64_t i0, i1;
      if (run < kMergeLdsRuns) {
        i0 = L.rb[run];
        i1 = L.re[run];
      } else {
        imp_range(R, run, b, rb, start, end, n_slices, &i0, &i1);
      }
      // kImpBatch records per thread loaded together, then counted (one load latency per batch)
      for (uint64_t i = i0 + threadIdx.x; i < i1; i += (uint64_t)kImpBatch * NT) {
        ImpRec r[kImpBatch];
#pragma unroll
        for (int j = 0; j < kImpBatch; ++j) {
          r[j].present = false;
          if (i + (uint64_t)j * NT < i1) imp_load<PACKED>(R, i + (uint64_t)j * NT, r[j]);
        }
#pragma unroll
        for (int j = 0; j < kImpBatch; ++j) {
          if (!r[j].present || !r[j].lds_ok || dst_slice(r[j].hash, rb) != b) continue;
          ++mine;
          if (!merge_count(L, r[j])) L.overflow = 1;
        }
      }
    }
    lds_barrier();
    ulonglong2* halves = reinterpret_cast<ulonglong2*>(slice);
    if (L.overflow) {
      if (threadIdx.x == 0) ovf_list[atomicAdd(n_ovf, 1ull)] = (uint32_t)b;
      if (mine) atomicAdd(ovf_recs, (unsigned long long)mine);
      if (tr.write_all)
        for (uint32_t q = threadIdx.x; q < 2 * S; q += NT) halves[q] = ulonglong2{0ull, 0ull};
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = 0xFFFFFFFFu;
    } else {
      for (uint32_t q = threadIdx.x; q < 2 * S; q += NT) {
        const uint32_t s = q >> 1;
        const bool hi = (q & 1u) != 0u;
        const unsigned long long c = L.C[s];
        bool is_new = false;
        if (!c) {
          if (tr.write_all) halves[q] = ulonglong2{0ull, 0ull};
        } else {
          const bool existing = !table_empty && (slice[s].ctrl & kReady);
          uint64_t k0, k1, h;
          uint32_t len;
          if constexpr (PACKED) {
            kp_unpack(L.K[s], &k0, &k1, &len);
            h = hash_record_packed(L.K[s]);
          } else {
            const unsigned long long kk1 = L.K1[s];
            k0 = L.K0[s];
            k1 = kk1 & kRecKeyMask;
            len = (uint32_t)(kk1 >> kRecLenShift);
            h = hash_inline(k0, k1, len);
          }
          if (!hi) {
            if (track || tr.smax) {
              atomicMax(&L.cmax, c);
              if (track) {
                if (c < (unsigned long long)kAggLdsHist) {
                  atomicAdd(&L.hist[c], 1u);
                } else if (c < (unsigned long long)kFreqHist) {
                  atomicAdd(&tr.hist[c], 1ull);
                } else {
                  const unsigned long long i = atomicAdd(tr.n_big, 1ull);
                  if (i < tr.big_cap) tr.big[i] = c;
                }
              }
            }
            if (existing) {
              slice[s].count += c;
            } else {
              halves[q] = ulonglong2{((unsigned long long)tag_of(h) << 32) | kReady | len, c};
              is_new = true;
            }
          } else if (!existing) {
            halves[q] = ulonglong2{k0, k1};
          }
        }
        const uint64_t nb = __ballot(is_new);
        if (nb && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(nb)) atomicAdd(&L.fresh, (uint32_t)__popcll(nb));
      }
      lds_barrier();
      if (threadIdx.x == 0 && L.fresh) atomicAdd(new_groups, (unsigned long long)L.fresh);
      if (tr.smax && threadIdx.x == 0) tr.smax[b] = L.cmax > 0xFFFFFFFEull ? 0xFFFFFFFFu : (uint32_t)L.cmax;
    }
    lds_barrier();
  }
  if (track) {
    lds_barrier();
    for (int i = threadIdx.x; i < kAggLdsHist; i += NT)
      if (L.hist[i]) atomicAdd(&tr.hist[i], (unsigned long long)L.hist[i]);
  }
}

// Group-by-group inserts (global_insert with the group's weight), blockIdx.y = run:
//  mode 0: every present record of runs marked skip (out of slice order);
//  mode 1: the records the LDS image cannot hold (keys longer than 15 bytes) of the other runs;
//  mode 2: the records of the listed overflowed slices (ovf_list, rb_old = the slice bits they
//          were cut with) that fit the image -- after the table has grown.
__global__ __launch_bounds__(kBlock) void dq_import_global_kernel(FreqTable T, const ImportRun* __restrict__ runs,
                                                                  int mode, int rb_old, const uint32_t* __restrict__ start,
                                                                  const uint32_t* __restrict__ end, uint64_t n_slices_old,
                                                                  const uint32_t* __restrict__ ovf_list, uint64_t n_ovf) {
  const int run = blockIdx.y;
  const ImportRun R = runs[run];
  if (mode == 0 ? !R.skip : R.skip) return;
  auto one = [&](uint64_t i, bool filter, uint64_t sl) -> bool {
    ImpRec r;
    imp_load<false>(R, i, r);
    if (!r.present) return true;
    if (mode == 1 && r.lds_ok) return true;
    if (mode == 2 && (!r.lds_ok || dst_slice(r.hash, rb_old) != sl)) return true;
    (void)filter;
    Key k;
    k.k0 = r.k0;
    k.k1 = r.k1;
    k.len = r.len;
    k.ptr = r.heap ? R.heap + r.k0 : nullptr;
    if (r.heap) k.k0 = k.k1 = 0;
    k.hash = r.hash;
    return global_insert(T, k, r.count);
  };
  if (mode != 2) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < R.n; i += (uint64_t)gridDim.x * kBlock)
      if (!one(i, false, 0)) return;
    return;
  }
  for (uint64_t o = blockIdx.x; o < n_ovf; o += gridDim.x) {
    const uint64_t sl = ovf_list[o];
    uint64_t i0, i1;
    imp_range(R, run, sl, rb_old, start, end, n_slices_old, &i0, &i1);
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += kBlock)
      if (!one(i, true, sl)) return;
  }
}

static unsigned grid_for(uint64_t n, uint64_t per, unsigned cap) {
  uint64_t b = (n + per - 1) / per;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (unsigned)b;
}

hipError_t launch_wire_count(const FreqTable& T, int n_parts, int chunk_log, uint64_t n_chunks, unsigned long long* d_cnt,
                             unsigned long long* d_kbytes, hipStream_t stream) {
  if (n_parts < 1 || n_parts > kWireMaxParts) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dq_wire_count_kernel, dim3(grid_for(n_chunks, 1, 65536)), dim3(kWireThreads), 0, stream, T, n_parts,
                     chunk_log, n_chunks, d_cnt, d_kbytes);
  return hipGetLastError();
}

hipError_t launch_gather_strided(const unsigned long long* d_scanned, uint64_t stride, uint64_t n, unsigned long long* d_out,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(dq_gather_strided_kernel, dim3(grid_for(n + 1, 256, 1024)), dim3(256), 0, stream, d_scanned, stride, n,
                     d_out);
  return hipGetLastError();
}

hipError_t launch_wire_scatter(const FreqTable& T, int n_parts, int chunk_log, uint64_t n_chunks,
                               const unsigned long long* d_pos, const unsigned long long* d_sec,
                               const unsigned long long* d_key_base, unsigned long long* d_key_cursor, uint8_t* d_out,
                               uint8_t* d_keys, hipStream_t stream) {
  if (n_parts < 1 || n_parts > kWireMaxParts) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dq_wire_scatter_kernel, dim3(grid_for(n_chunks, 1, 65536)), dim3(kWireThreads), 0, stream, T, n_parts,
                     chunk_log, n_chunks, d_pos, d_sec, d_key_base, d_key_cursor, d_out, d_keys);
  return hipGetLastError();
}

hipError_t launch_import_sketch(const ImportRun* d_runs, int n_runs, uint64_t max_n, uint32_t* d_hll, hipStream_t stream) {
  if (n_runs < 1 || n_runs > 65535 || max_n == 0) return hipSuccess;
  hipLaunchKernelGGL(dq_import_sketch_kernel, dim3(grid_for(max_n, kBlock * 8, 2048), (unsigned)n_runs), dim3(kBlock), 0,
                     stream, d_runs, d_hll);
  return hipGetLastError();
}

hipError_t launch_import_bounds(const ImportRun* d_runs, int n_runs, uint64_t max_n, int rb, uint64_t n_slices,
                                uint32_t* d_start, uint32_t* d_end, unsigned int* d_unsorted, unsigned int* d_drop,
                                int rerun, hipStream_t stream) {
  if (n_runs < 1 || n_runs > 65535 || max_n == 0) return hipSuccess;
  hipLaunchKernelGGL(dq_import_bounds_kernel, dim3(grid_for(max_n, kBlock * 8, 2048), (unsigned)n_runs), dim3(kBlock), 0,
                     stream, d_runs, rb, n_slices, d_start, d_end, d_unsorted, d_drop, rerun);
  return hipGetLastError();
}

hipError_t launch_import_merge(const FreqTable& T, bool packed, bool flat, const ImportRun* d_runs, int n_runs, const uint32_t* d_start,
                               const uint32_t* d_end, int table_empty, unsigned long long* d_hist, unsigned long long* d_big,
                               unsigned long long* d_n_big, unsigned long long big_cap, uint32_t* d_smax, int write_all,
                               uint32_t* d_ovf_list, unsigned long long* d_n_ovf, unsigned long long* d_ovf_recs,
                               unsigned long long* d_new_groups, hipStream_t stream) {
  const uint64_t n_slices = (T.mask + 1) >> kFreqSliceLog;
  if (!table_empty && (d_hist || d_smax || write_all)) return hipErrorInvalidValue;
  AggTrack tr{d_hist, d_big, d_n_big, big_cap, d_smax, write_all};
  const unsigned blocks = grid_for(n_slices, 1, 65536);
  if (packed && flat)
    hipLaunchKernelGGL((dq_import_merge_kernel<true, true>), dim3(blocks), dim3(kMergeThreads), 0, stream, T, d_runs, n_runs,
                       d_start, d_end, n_slices, table_empty, tr, d_ovf_list, d_n_ovf, d_ovf_recs, d_new_groups);
  else if (packed)
    hipLaunchKernelGGL((dq_import_merge_kernel<true, false>), dim3(blocks), dim3(kMergeThreads), 0, stream, T, d_runs, n_runs,
                       d_start, d_end, n_slices, table_empty, tr, d_ovf_list, d_n_ovf, d_ovf_recs, d_new_groups);
  else
    hipLaunchKernelGGL((dq_import_merge_kernel<false, false>), dim3(blocks), dim3(kMergeThreads), 0, stream, T, d_runs, n_runs, d_start,
                       d_end, n_slices, table_empty, tr, d_ovf_list, d_n_ovf, d_ovf_recs, d_new_groups);
  return hipGetLastError();
}

hipError_t launch_import_global(const FreqTable& T, const ImportRun* d_runs, int n_runs, uint64_t max_n, int mode, int rb_old,
                                const uint32_t* d_start, const uint32_t* d_end, uint64_t n_slices_old,
                                const uint32_t* d_ovf_list, uint64_t n_ovf, hipStream_t stream) {
  if (n_runs < 1 || n_runs > 65535) return hipSuccess;
  const unsigned gx = mode == 2 ? grid_for(n_ovf, 1, 4096) : grid_for(max_n, kBlock * 4, 4096);
  hipLaunchKernelGGL(dq_import_global_kernel, dim3(gx, (unsigned)n_runs), dim3(kBlock), 0, stream, T, d_runs, mode, rb_old,
                     d_start, d_end, n_slices_old, d_ovf_list, n_ovf);
  return hipGetLastError();
}


// =============================================================================================
// Few groups (round 4): the profiler's low-cardinality histograms (ColumnProfiler.scala:564-606:
// columns with at most 120 distinct values) and any grouping hinted to have at most
// kFreqFewGroups groups (dq_freq_expect_groups).  One key column; every workgroup counts its
// contiguous rows in an LDS table of kSmallSlots keys (each row: one probe, one LDS add), keys
// loaded as the fused stage loads them (offset pairs one iteration ahead, one unaligned 16-byte
// load per string), then writes its groups -- not into the global table (every workgroup would
// hit the same few slots with device atomics) but to its own staging list; one small merge kernel
// sums the lists and inserts each group once.  A key longer than 15 bytes, or more keys than the
// LDS table holds, raises `bad` and the host takes the general insert path instead.
// =============================================================================================
constexpr int kSmallSlots = 1024;
// Rows per thread per step: 4 (70 VGPRs, 7 waves per SIMD) measured 4.64 ms for C5's 20-column
// launch against 5.13 with 8 (109 VGPRs, 4 waves); 2 / 3 / 6 rows and 256 threads per block were
// within 0.1 ms of 4, 1024 threads 5.96 (profiles/r05_c5_small_per_ab.txt)
#ifndef DQ_SMALL_PER
#define DQ_SMALL_PER 4
#endif
#ifndef DQ_SMALL_THREADS
#define DQ_SMALL_THREADS 512
#endif
constexpr int kSmallThreads = DQ_SMALL_THREADS;
constexpr int kSmallPer = DQ_SMALL_PER;  // rows per thread per iteration

// Counts in kSmallCopies copies per slot, a lane adding to copy (lane & 3): with ~100 keys most
// of a wave's 64 rows fall on a few slots, and LDS atomics of one instruction to ONE address are
// serialised (C5 round 5: 0.49 of the LDS-active cycles in bank conflicts); the copies of a slot
// are adjacent words, so lanes of one key hit four banks.
#ifndef DQ_SMALL_COPIES
#define DQ_SMALL_COPIES 4
#endif
constexpr int kSmallCopies = DQ_SMALL_COPIES;
static_assert(kSmallCopies == 1 || kSmallCopies == 2 || kSmallCopies == 4, "the write-out reads the copies as one load");
struct SmallLds {
  unsigned long long K0[kSmallSlots], K1[kSmallSlots];  // K1 = key bytes 8..14 | length << 56
  alignas(16) uint32_t C[kSmallSlots * kSmallCopies];
  uint32_t n_used;
};

__device__ inline bool small_count(SmallLds& L, uint64_t k0, uint64_t k1l) {
  uint32_t s = lds_hash(k0, k1l, 0) & (kSmallSlots - 1);
  const uint32_t cp = threadIdx.x & (kSmallCopies - 1);
  // the common case once the few keys are in: the key in its first slot (both words read in
  // one LDS round trip; volatile keeps K1's read before K0's -- a wave's LDS reads execute in
  // order and a slot's K0 is written before its K1 is published -- so a matching K1 comes with
  // its own K0, never an older word)
  {
    const unsigned long long c1 = *reinterpret_cast<volatile unsigned long long*>(&L.K1[s]);
    const unsigned long long c0 = *reinterpret_cast<volatile unsigned long long*>(&L.K0[s]);
    if (c1 == k1l && c0 == k0) {
      atomicAdd(&L.C[s * kSmallCopies + cp], 1u);
      return true;
    }
  }
  bool done = false;
  for (uint32_t probe = 0; probe < (uint32_t)kSmallSlots && !done;) {  // (publish inside the iteration)
    const unsigned long long c = __hip_atomic_load(&L.K1[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (c == k1l && __hip_atomic_load(&L.K0[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == k0) {
      atomicAdd(&L.C[s * kSmallCopies + cp], 1u);
      done = true;
    } else if (c == kLdsEmpty) {
      if (atomicCAS(&L.K1[s], kLdsEmpty, kLdsBusy) == kLdsEmpty) {
        L.K0[s] = k0;
        __threadfence_block();
        atomicExch(&L.K1[s], k1l);
        atomicAdd(&L.C[s * kSmallCopies + cp], 1u);
        done = true;
      }
    } else if (c == kLdsBusy) {
      // being published: look again
    } else {
      s = (s + 1) & (kSmallSlots - 1);
      ++probe;
    }
  }
  return done;
}

// out_k0 / out_k1 / out_c: kSmallSlots entries per workgroup, out_n[block] of them used.
template <bool STRING>
__global__ __launch_bounds__(kSmallThreads) void dq_freq_small_kernel(FreqKeySpec ks, const DevColumn* __restrict__ cols,
                                                                      int64_t n_rows, unsigned long long* out_k0,
                                                                      unsigned long long* out_k1, uint32_t* out_c,
                                                                      uint32_t* out_n, unsigned int* bad) {
  __shared__ SmallLds L;
  const uint32_t t = threadIdx.x;
  {  // a launch over several columns (dq_profile_few_strings): blockIdx.y picks the column and
     // its lists (gridDim.y = 1 otherwise)
    const uint64_t y = blockIdx.y;
    cols += y;
    out_k0 += y * gridDim.x * kSmallSlots;
    out_k1 += y * gridDim.x * kSmallSlots;
    out_c += y * gridDim.x * kSmallSlots;
    out_n += y * gridDim.x;
    bad += y;
  }
  for (uint32_t i = t; i < (uint32_t)kSmallSlots; i += kSmallThreads) L.K1[i] = kLdsEmpty;
  for (uint32_t i = t; i < (uint32_t)(kSmallSlots * kSmallCopies); i += kSmallThreads) L.C[i] = 0u;
  if (t == 0) L.n_used = 0u;
  __syncthreads();
  const DevColumn& c0 = cols[ks.key_cols[0]];
  const bool null_key = ks.null_as_key != 0;
  const uint8_t* validity = uniform_ptr(c0.validity);
  const int64_t per = (((n_rows + gridDim.x - 1) / gridDim.x) + 63) & ~(int64_t)63;
  const int64_t r0 = min((int64_t)blockIdx.x * per, n_rows);
  const int64_t r1 = min(r0 + per, n_rows);
  bool fail = false;
  constexpr int64_t step = (int64_t)kSmallThreads * kSmallPer;
  if constexpr (STRING) {
    const int32_t* offs = uniform_ptr(c0.offsets);
    const uint32_t heap_end = __builtin_amdgcn_readfirstlane((uint32_t)offs[n_rows]);
    const uint8_t* vals = static_cast<const uint8_t*>(uniform_ptr(c0.values));
    const __amdgpu_buffer_rsrc_t rs_vals =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vals), 0, (int)heap_end, 0x00020000);
    if (heap_end < 16u) {  // (key_load16: the general path groups a heap under 16 bytes)
      if (t == 0) atomicOr(bad, 1u);
      return;
    }
    uint32_t ob[kSmallPer], oe[kSmallPer], vword = 0u;
    auto load_offs = [&](int64_t base) {  // the offsets (and validity bits) of the step at base
      const int64_t left = r1 - base;
      const uint32_t m = (uint32_t)(left < step ? left : step);
      vword = tile_valid_word<kSmallThreads, kSmallPer>(validity, base, m);
      const __amdgpu_buffer_rsrc_t rs_off = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(offs + base), 0, (int)(4u * (m + 1u)), 0x00020000);
#pragma unroll
      for (int j = 0; j < kSmallPer; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_off, (int)(4u * ((uint32_t)j * kSmallThreads + t)), 0, 0);
        ob[j] = v[0];
        oe[j] = v[1];
      }
    };
    if (r0 < r1) load_offs(r0);
    for (int64_t base = r0; base < r1 && !fail; base += step) {
      uint32_t lens[(kSmallPer + 3) / 4] = {};
      uint32_t kw[kSmallPer][4];
      uint32_t sel = 0u, nul = 0u;
#pragma unroll
      for (int j = 0; j < kSmallPer; ++j) {  // (lens byte: as the fused stage's, 255 = too long)
        const int64_t row = base + (int64_t)j * kSmallThreads + t;
        const uint32_t n = oe[j] - ob[j];
        lens[j / 4] |= (n > 15u ? 255u : n | (key_shift(ob[j], heap_end) << 4)) << (8 * (j % 4));
        const bool valid = validity == nullptr || ((stage_valid_mask(vword, j) >> (t & 63u)) & 1u);
        if (row < r1 && (valid || null_key)) sel |= 1u << j;
        if (row < r1 && !valid) nul |= 1u << j;
        key_load16(rs_vals, heap_end, ob[j], kw[j]);
      }
      if (base + step < r1) load_offs(base + step);
#pragma unroll
      for (int j = 0; j < kSmallPer; ++j) {
        if (!((sel >> j) & 1u)) continue;
        uint64_t k0, k1;
        uint32_t n;
        if ((nul >> j) & 1u) {
          n = 9;
          k0 = kNullK0;
          k1 = kNullK1;
        } else {
          n = (lens[j / 4] >> (8 * (j % 4))) & 0xFFu;
          if (n == 255u) {
            fail = true;
            continue;
          }
          if (n > 15u) key_shr_bytes(kw[j], n >> 4);
          n &= 15u;
          const uint64_t lo = (uint64_t)kw[j][0] | ((uint64_t)kw[j][1] << 32);
          const uint64_t hi = (uint64_t)kw[j][2] | ((uint64_t)kw[j][3] << 32);
          k0 = n >= 8 ? lo : (lo & ((1ull << (8u * n)) - 1ull));
          k1 = n > 8 ? (hi & ((1ull << (8u * (n - 8u))) - 1ull)) : 0ull;
        }
        if (!small_count(L, k0, k1 | ((unsigned long long)n << kRecLenShift))) fail = true;
      }
    }
  } else {
    const int w = width_of(c0.type);
    for (int64_t base = r0; base < r1 && !fail; base += step) {
      uint64_t v[kSmallPer];
      uint32_t sel = 0u, nul = 0u;
#pragma unroll
      for (int j = 0; j < kSmallPer; ++j) {
        const int64_t row = base + (int64_t)j * kSmallThreads + t;
        v[j] = 0;
        if (row >= r1) continue;
        const bool valid = validity == nullptr || ((validity[row >> 3] >> (row & 7)) & 1u);
        if (valid || null_key) sel |= 1u << j;
        if (!valid) nul |= 1u << j;
        else v[j] = fixed_bits(c0, row);
      }
#pragma unroll
      for (int j = 0; j < kSmallPer; ++j) {
        if (!((sel >> j) & 1u)) continue;
        uint64_t k0 = v[j];
        uint32_t n = (uint32_t)w;
        if ((nul >> j) & 1u) {  // Histogram NULL of a non-string column: the empty key
          k0 = 0;
          n = 0;
        } else if (null_key) {  // Histogram groups cast-to-string values: every NaN is "NaN"
          if (c0.type == DQ_T_FLOAT64 && (k0 & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) k0 = 0x7ff8000000000000ull;
          if (c0.type == DQ_T_FLOAT32 && (k0 & 0x7fffffffull) > 0x7f800000ull) k0 = 0x7fc00000ull;
        }
        if (!small_count(L, k0, (unsigned long long)n << kRecLenShift)) fail = true;
      }
    }
  }
  if (fail) atomicOr(bad, 1u);
  __syncthreads();
  // this workgroup's groups, compacted into its staging list
  for (uint32_t i = t; i < (uint32_t)kSmallSlots; i += kSmallThreads) {
    uint32_t c = 0u;
#pragma unroll
    for (int k = 0; k < kSmallCopies; ++k) c += L.C[i * kSmallCopies + k];
    const bool used = c != 0u;
    const uint64_t m = __ballot(used);
    uint32_t at = 0;
    if (m) {
      const uint32_t lane = t & 63u;
      uint32_t base_w = 0;
      if (lane == (uint32_t)__builtin_ctzll(m)) base_w = atomicAdd(&L.n_used, (uint32_t)__popcll(m));
      base_w = __shfl(base_w, __builtin_ctzll(m), 64);
      at = base_w + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    if (used) {
      const uint64_t o = (uint64_t)blockIdx.x * kSmallSlots + at;
      out_k0[o] = L.K0[i];
      out_k1[o] = L.K1[i];
      out_c[o] = c;
    }
  }
  __syncthreads();
  if (t == 0) out_n[blockIdx.x] = L.n_used;
}

// Sums the workgroups' staging lists into one LDS table (K0 / K1 / C, kSmallSlots keys; one
// workgroup): thread t merges the lists of blocks t, t + kSmallThreads, ..., 8 entries at a time
// with their loads issued together (one list per thread: the lists' loads all in flight at once).
// Returns (to every thread) whether more keys than the table holds arrived.
__device__ bool small_merge_lists(unsigned long long* K0, unsigned long long* K1, unsigned long long* C,
                                  const unsigned long long* __restrict__ in_k0, const unsigned long long* __restrict__ in_k1,
                                  const uint32_t* __restrict__ in_c, const uint32_t* __restrict__ in_n, int n_blocks,
                                  unsigned int* any_fail) {
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < (uint32_t)kSmallSlots; i += kSmallThreads) {
    K1[i] = kLdsEmpty;
    C[i] = 0ull;
  }
  if (t == 0) *any_fail = 0u;
  __syncthreads();
  bool fail = false;
  constexpr int U = 8;
  for (int b = (int)t; b < n_blocks; b += kSmallThreads) {
    const uint32_t n = in_n[b];
    for (uint32_t i0 = 0; i0 < n; i0 += U) {
      unsigned long long k0[U], k1[U];
      uint32_t cnt[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const uint64_t o = (uint64_t)b * kSmallSlots + i0 + j;
        const bool in = i0 + j < n;
        k0[j] = in ? in_k0[o] : 0ull;
        k1[j] = in ? in_k1[o] : 0ull;
        cnt[j] = in ? in_c[o] : 0u;
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (i0 + j >= n) continue;
        uint32_t s = lds_hash(k0[j], k1[j], 0) & (kSmallSlots - 1);
        bool done = false;
        {  // the key already in its first slot (as small_count: K1's read ordered before K0's)
          const unsigned long long c1 = *reinterpret_cast<volatile unsigned long long*>(&K1[s]);
          const unsigned long long c0 = *reinterpret_cast<volatile unsigned long long*>(&K0[s]);
          if (c1 == k1[j] && c0 == k0[j]) {
            atomicAdd(&C[s], (unsigned long long)cnt[j]);
            done = true;
          }
        }
        for (uint32_t probe = 0; probe < (uint32_t)kSmallSlots && !done;) {
          const unsigned long long c = atomicCAS(&K1[s], kLdsEmpty, kLdsBusy);
          if (c == kLdsEmpty) {
            K0[s] = k0[j];
            __threadfence_block();
            atomicExch(&K1[s], k1[j]);
            atomicAdd(&C[s], (unsigned long long)cnt[j]);
            done = true;
          } else if (c == kLdsBusy) {
          } else if (c == k1[j] && __hip_atomic_load(&K0[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == k0[j]) {
            atomicAdd(&C[s], (unsigned long long)cnt[j]);
            done = true;
          } else {
            s = (s + 1) & (kSmallSlots - 1);
            ++probe;
          }
        }
        if (!done) fail = true;
      }
    }
  }
  if (fail) *any_fail = 1u;
  __syncthreads();
  return *any_fail != 0u;
}

// Sums the workgroups' staging lists and inserts each group into the table once (global_insert:
// the table may already hold groups).
__global__ __launch_bounds__(kSmallThreads) void dq_freq_small_merge_kernel(const unsigned long long* __restrict__ in_k0,
                                                                            const unsigned long long* __restrict__ in_k1,
                                                                            const uint32_t* __restrict__ in_c,
                                                                            const uint32_t* __restrict__ in_n, int n_blocks,
                                                                            FreqTable T, unsigned int* bad) {
  __shared__ unsigned long long K0[kSmallSlots], K1[kSmallSlots];
  __shared__ unsigned long long C[kSmallSlots];
  __shared__ unsigned int any_fail;
  const uint32_t t = threadIdx.x;
  if (*bad) return;  // (the counting kernel failed: the host takes the general path)
  if (small_merge_lists(K0, K1, C, in_k0, in_k1, in_c, in_n, n_blocks, &any_fail)) {
    // more keys than the image holds: nothing is inserted, the host regroups
    if (t == 0) atomicOr(bad, 1u);
    return;
  }
  for (uint32_t i = t; i < (uint32_t)kSmallSlots; i += kSmallThreads) {
    if (!C[i]) continue;
    Key k;
    k.k0 = K0[i];
    k.k1 = K1[i] & kRecKeyMask;
    k.len = (uint32_t)(K1[i] >> kRecLenShift);
    k.ptr = nullptr;
    k.hash = hash_inline(k.k0, k.k1, k.len);
    global_insert(T, k, C[i]);
  }
}

// The same sum written as ONE compact list (out_k0 / out_k1 / out_c [0, *out_n); K1 = key bytes
// 8..14 | length << 56) instead of into a table: the profiler's few-valued string columns
// (dq_profile_few_strings).  *out_n stays 0 and *bad is raised when the column did not fit.
__global__ __launch_bounds__(kSmallThreads) void dq_freq_small_merge_flat_kernel(
    const unsigned long long* __restrict__ in_k0, const unsigned long long* __restrict__ in_k1,
    const uint32_t* __restrict__ in_c, const uint32_t* __restrict__ in_n, int n_blocks, unsigned long long* out_k0,
    unsigned long long* out_k1, unsigned long long* out_c, uint32_t* out_n, unsigned int* bad) {
  __shared__ unsigned long long K0[kSmallSlots], K1[kSmallSlots];
  __shared__ unsigned long long C[kSmallSlots];
  __shared__ unsigned int any_fail;
  __shared__ uint32_t n_used;
  const uint32_t t = threadIdx.x;
  {  // one workgroup per column (blockIdx.x), each over that column's lists
    const uint64_t y = blockIdx.x;
    in_k0 += y * (uint64_t)n_blocks * kSmallSlots;
    in_k1 += y * (uint64_t)n_blocks * kSmallSlots;
    in_c += y * (uint64_t)n_blocks * kSmallSlots;
    in_n += y * (uint64_t)n_blocks;
    out_k0 += y * kSmallSlots;
    out_k1 += y * kSmallSlots;
    out_c += y * kSmallSlots;
    out_n += y;
    bad += y;
  }
  if (t == 0) n_used = 0u;
  if (*bad) {
    if (t == 0) *out_n = 0u;
    return;
  }
  if (small_merge_lists(K0, K1, C, in_k0, in_k1, in_c, in_n, n_blocks, &any_fail)) {
    if (t == 0) {
      atomicOr(bad, 1u);
      *out_n = 0u;
    }
    return;
  }
  for (uint32_t i = t; i < (uint32_t)kSmallSlots; i += kSmallThreads) {
    const bool used = C[i] != 0ull;
    const uint64_t m = __ballot(used);
    uint32_t at = 0;
    if (m) {
      const uint32_t lane = t & 63u;
      uint32_t base_w = 0;
      if (lane == (uint32_t)__builtin_ctzll(m)) base_w = atomicAdd(&n_used, (uint32_t)__popcll(m));
      base_w = __shfl(base_w, __builtin_ctzll(m), 64);
      at = base_w + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    if (used) {
      out_k0[at] = K0[i];
      out_k1[at] = K1[i];
      out_c[at] = C[i];
    }
  }
  __syncthreads();
  if (t == 0) *out_n = n_used;
}

hipError_t launch_freq_small_flat(bool string_key, const FreqKeySpec& ks, const DevColumn* d_cols, int n_cols,
                                  int64_t n_rows, int blocks, unsigned long long* d_k0, unsigned long long* d_k1,
                                  uint32_t* d_c, uint32_t* d_n, unsigned int* d_bad, unsigned long long* d_out_k0,
                                  unsigned long long* d_out_k1, unsigned long long* d_out_c, uint32_t* d_out_n,
                                  hipStream_t stream) {
  if (n_rows <= 0 || n_cols <= 0 || n_cols > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)blocks, (unsigned)n_cols);
  if (string_key)
    hipLaunchKernelGGL(dq_freq_small_kernel<true>, grid, dim3(kSmallThreads), 0, stream, ks, d_cols, n_rows, d_k0, d_k1,
                       d_c, d_n, d_bad);
  else
    hipLaunchKernelGGL(dq_freq_small_kernel<false>, grid, dim3(kSmallThreads), 0, stream, ks, d_cols, n_rows, d_k0, d_k1,
                       d_c, d_n, d_bad);
  hipLaunchKernelGGL(dq_freq_small_merge_flat_kernel, dim3((unsigned)n_cols), dim3(kSmallThreads), 0, stream, d_k0, d_k1,
                     d_c, d_n, blocks, d_out_k0, d_out_k1, d_out_c, d_out_n, d_bad);
  return hipGetLastError();
}

hipError_t launch_freq_small(const FreqKeySpec& ks, bool string_key, const DevColumn* d_cols, int64_t n_rows, int blocks,
                             unsigned long long* d_k0, unsigned long long* d_k1, uint32_t* d_c, uint32_t* d_n,
                             unsigned int* d_bad, const FreqTable& T, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  if (string_key)
    hipLaunchKernelGGL(dq_freq_small_kernel<true>, dim3((unsigned)blocks), dim3(kSmallThreads), 0, stream, ks, d_cols, n_rows,
                       d_k0, d_k1, d_c, d_n, d_bad);
  else
    hipLaunchKernelGGL(dq_freq_small_kernel<false>, dim3((unsigned)blocks), dim3(kSmallThreads), 0, stream, ks, d_cols,
                       n_rows, d_k0, d_k1, d_c, d_n, d_bad);
  hipLaunchKernelGGL(dq_freq_small_merge_kernel, dim3(1), dim3(kSmallThreads), 0, stream, d_k0, d_k1, d_c, d_n, blocks, T,
                     d_bad);
  return hipGetLastError();
}

}  // namespace dq
