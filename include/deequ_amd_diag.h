/*
 * deequ_amd_diag.h -- measurement entry points of libdeequ_amd.so.  Not part of the drop-in
 * boundary (deequ_amd.h): no reference call site binds these.  bench.py uses them to price
 * the hash-bound kernels (ApproxCountDistinct, StatefulHyperloglogPlus.scala:89-115) against
 * the VALU hash rate the card sustains, next to the HBM roofline.
 */
#ifndef DEEQU_AMD_DIAG_H
#define DEEQU_AMD_DIAG_H

#include <stdint.h>
#include "deequ_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Runs `reps` launches of a register-only kernel that hashes int64 values with Spark's
 * XXH64 (seed 42), and with `with_hll` != 0 also takes each hash's HLL index/rank and folds it
 * into an LDS register copy, on `device`; no HBM traffic.  Writes the sustained hash rate
 * (hashes per second, best launch) to *hashes_per_sec. */
dq_status dq_diag_hash_rate(int device, int with_hll, int reps, double* hashes_per_sec);

/* Aggregates what `f` has staged, then reports which paths its groupings took (tests assert
 * that a workload exercised the path it is meant to): out[0] = table slots (2048 per slice),
 * out[1] = partition-path aggregations, out[2] = hash bits (log2 slices) of the last one,
 * out[3] = records that went through the sort path (small stagings, retries, skew fallbacks),
 * out[4] = partition-path aggregations of packed digit-key records, out[5] = batches grouped by
 * the few-groups kernel (dq_freq_small_kernel), out[6] = 1 if a wait for another lane's slot
 * publish ever timed out (an error every API call also reports), out[7] = imported wire runs
 * that were in order only by coarser slices than the table's (merged from the enclosing ranges),
 * out[8] = imported wire runs out of order (inserted group by group), out[9] = partition-path
 * aggregations of hashed records (long or multi-column keys), out[10] = hashed records inserted
 * globally (slices handed back, tables that already held groups), out[11] = 1 while the table is
 * compacted (occupied slots only), out[12] = partition-path aggregations of canonical UUID records
 * (dq_uuidpack.h), out[13] = partition-path aggregations of 16-byte-key records (16-byte strings,
 * two 8-byte key columns).  `out` holds 14 values. */
dq_status dq_diag_freq_paths(dq_freq* f, int64_t* out);

/* Test hooks of one table (tests only; never set by the product): flags = 1 makes claimed
 * global slots never turn READY, so a wait for another lane's publish times out (the timeout is
 * a hard error, DQ_ERR_DEVICE).  0 restores normal publishing.  Replaces an environment variable
 * the production library used to read on every dq_freq_create. */
dq_status dq_diag_freq_test_flags(dq_freq* f, int32_t flags);

/* Host build of the library's java.lang.Double.parseDouble (the parser dq_cast_utf8 and the
 * predicate IR's string -> double cast run on the device, compiled from the same source):
 * *ok = 1 and *out = the correctly rounded value, or *ok = 0 (NumberFormatException, NULL in
 * Spark).  Lets CPU tests check it against a reference parser on millions of strings. */
dq_status dq_diag_parse_double(const uint8_t* s, int64_t n, double* out, int32_t* ok);

/* Host build of the predicate interpreter (the source dq_pred_kernel runs on the device,
 * deequ_amd/csrc/dq_predeval.h): validates `p` against the columns' types as plan creation does
 * (same status codes), then evaluates it over `n_rows` rows of HOST columns (offset 0):
 * out[r] = 0 FALSE, 1 TRUE, 2 NULL.  CPU tests check it against the oracle's SQL evaluator. */
dq_status dq_diag_eval_predicate(const dq_predicate* p, const dq_column* columns, int n_columns, int64_t n_rows,
                                 uint8_t* out);

/* Host build of the group-by's record packing of digit-string keys (<= 15 ASCII digits, or
 * Histogram's "NullValue"; deequ_amd/csrc/dq_keypack.h): *ok = 1, *packed = the 8-byte record
 * word and back[0 .. *back_len) = the key bytes it unpacks to; *ok = 0 for any other key. */
/* The group-by's table hash of n inline keys (k0/k1 = key bytes little-endian, len <= 16) as the
 * device computes it: out[2i] = the hash, out[2i+1] = the packed record word or ~0 (tests check
 * both against a host restatement). */
dq_status dq_diag_table_hash(int device, const uint64_t* k0, const uint64_t* k1, const uint32_t* len, int64_t n,
                             uint64_t* out);

dq_status dq_diag_key_pack(const uint8_t* key, int32_t len, uint64_t* packed, uint8_t* back, int32_t* back_len,
                           int32_t* ok);

/* Host build of the group-by's canonical-UUID packing (dq_uuidpack.h): *ok = 1 and words[0..1] =
 * the key's 128-bit value, back[0..36) = the text it unpacks to, when key[0..len) is a canonical
 * lowercase UUID ("xxxxxxxx-xxxx-xxxx-xxxx-xxxxxxxxxxxx"); else *ok = 0. */
dq_status dq_diag_uuid_pack(const uint8_t* key, int32_t len, uint64_t* words, uint8_t* back, int32_t* ok);

#ifdef __cplusplus
}
#endif

#endif /* DEEQU_AMD_DIAG_H */
