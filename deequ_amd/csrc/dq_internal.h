// dq_internal.h -- structures shared by the host planner (dq_api.cpp) and the gfx950
// kernels (dq_scan.hip, dq_hll.hip, dq_pred.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/deequ_amd.h"

namespace dq {

constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
constexpr int kMaxPreds = 8;         // predicates evaluated per scan task
constexpr int kMaxStack = 8;         // generic predicate interpreter stack depth
constexpr int kHllM = 512;           // 2^p registers, p = 9 (StatefulHyperloglogPlus.scala:157-161)
constexpr int kHllIdxShift = 55;     // 64 - p
constexpr uint64_t kHllWPadding = 1ull << 8;
constexpr int kScanRowAlign = 2048;  // chunk granularity: keeps every lane's bitmap word aligned

// A batch column after host preparation: row 0 of the batch is at values[0] and at bit 0 of
// validity[0] (the host realigns sliced Arrow bitmaps).  Device pointers.
struct DevColumn {
  const uint8_t* validity;  // nullptr = all valid
  const void* values;
  const int32_t* offsets;   // utf8
  int32_t type;             // dq_type
  int32_t pad;
};

// Mask produced by the generic predicate kernel: bit r of `t` = predicate TRUE at row r,
// bit r of `nn` = predicate NOT NULL at row r.  64-bit words, LSB-first.
struct DevMask {
  const uint64_t* t;
  const uint64_t* nn;
};

enum FastPredKind : int32_t {
  FP_NONE = 0,
  FP_CMP = 1,           // primary CMP literal
  FP_COALESCE_CMP = 2,  // COALESCE(primary, coalesce literal) CMP literal
  FP_IS_NULL = 3,
  FP_IS_NOT_NULL = 4,
  FP_CONST = 5,         // constant TRUE/FALSE/NULL (lit_i: 1 true, 0 false, -1 null)
  FP_MASK = 6,          // precomputed DevMask[mask]
  FP_BOOL = 7           // the primary (a bool column) itself: TRUE = value bit, NULL = invalid
};

enum CmpOp : int32_t { CMP_EQ = 0, CMP_NE, CMP_LT, CMP_LE, CMP_GT, CMP_GE, CMP_EQNS };

struct FastPred {
  int32_t kind;    // FastPredKind
  int32_t op;      // CmpOp
  int32_t as_f64;  // compare in fp64 (else int64)
  int32_t mask;    // FP_MASK: index into the batch mask table
  int64_t lit_i;
  double lit_f;
  int64_t coal_i;
  double coal_f;
  // Branch-free evaluation (filled by the host from kind/op; each is 0 or ~0u):
  //   cmp  = (x < lit & m_lt) | (x == lit & m_eq) | (!(x < lit | x == lit) & m_gt)
  //   TRUE = cmp & f_cmp | ~valid & f_isnull | valid & f_isnotnull | f_true | mask_t & f_mask
  //   NOT NULL = valid & f_nn_valid | f_nn_one | mask_nn & f_mask
  // (a NaN x is neither < nor == a non-NaN literal, so it lands in "greater": Spark's order)
  uint32_t m_lt, m_eq, m_gt;
  uint32_t f_cmp, f_coal, f_isnull, f_isnotnull, f_true, f_mask, f_nn_valid, f_nn_one;
  // One-compare form of the same operator (0 when it does not apply): bits 0-1 pick the
  // compare (CS_LT: x < lit, CS_LE: x <= lit, CS_EQ: x == lit), bit 2 (CS_INV) negates it:
  // GE = !LT, GT = !LE, NE = !EQ.  An ordered fp64 compare is false for a NaN x, so NaN lands
  // above every (non-NaN) literal, Spark's NaN-safe order; a NaN literal keeps the three masks.
  uint32_t cmp_sel;
};
enum CmpSel : uint32_t { CS_MASKS = 0, CS_LT = 1, CS_LE = 2, CS_EQ = 3, CS_INV = 4 };

enum ScanTaskFlags : int32_t {
  TF_VALUES = 1,      // the task must read the primary column's values
  TF_STATS = 2,       // sum/mean/stddev/min/max wanted
  TF_WHERE = 4,       // filter rows by batch mask `where_mask`
  TF_VALIDITY = 8,    // primary column is read for validity (completeness / null tests)
  TF_HLL = 16         // ApproxCountDistinct of the primary column, fused into the value scan
};

struct ScanTask {
  int32_t primary;     // batch column index or -1 (row-count only task)
  int32_t ptype;       // dq_type of the primary column
  int32_t flags;       // ScanTaskFlags
  int32_t where_mask;  // batch mask index when TF_WHERE
  int32_t n_preds;
  int32_t hll;         // TF_HLL: the task's HLL register set (registers + hll * kHllM)
  FastPred preds[kMaxPreds];
};

// Per-(task, block) partial aggregate and the per-task running accumulator.  Every field is
// 8 bytes; the layout is mirrored by nothing outside this library.
struct ScanAcc {
  int64_t n_rows;   // rows in scope: Σ where TRUE (or all rows)
  int64_t n_wnn;    // Σ where NOT NULL (or all rows)
  int64_t n_sel;    // Σ valid & where TRUE
  int64_t isum;     // wrapping int64 sum of integral values
  int64_t imin, imax;
  double fs, fc;    // Neumaier-compensated fp64 sum: value = fs + fc
  double fmin, fmax;
  int64_t nnan;     // NaNs among selected floats
  double mean, m2;  // moments about the mean over the n_sel selected values
  int64_t pm[kMaxPreds];  // predicate TRUE & where TRUE
  int64_t pn[kMaxPreds];  // predicate NOT NULL & where TRUE
};

// Where a task's block partials live for the current batch.
struct PartRange {
  int64_t offset;
  int32_t count;
  int32_t pad;
};

struct HllTask {
  int32_t column;
  int32_t ctype;
  int32_t where_mask;  // -1 = none
  int32_t reg_set;     // HLL: register set (registers + reg_set * kHllM); unused elsewhere
};

// Profiler pass 1 on a utf8 column (dq_profile.hip): the DataType counts (dt_index * 5 ..) and
// the HLL registers (reg_set) of one (column, where), both from one read of the strings.
struct StrTask {
  int32_t column;
  int32_t where_mask;  // -1 = none
  int32_t reg_set;
  int32_t dt_index;
};

// Correlation task (dq_pair.hip) and its running state CorrelationState(n, xAvg, yAvg, ck, xMk, yMk).
struct CorrTask {
  int32_t x, y;
  int32_t where_mask;  // -1 = none
  int32_t pad;
};
struct CorrAcc {
  double n, xavg, yavg, ck, xmk, ymk;
};

// One instruction of the generic predicate interpreter (dq_pred_insn after validation).
struct PredInsn {
  int32_t opcode;
  int32_t arg;
  int64_t i64;
  double f64;
};

struct PredProgram {
  int32_t first;   // index of first PredInsn in the plan's instruction table
  int32_t n;
};

// ---------------------------------------------------------------- frequency group-by
constexpr int kMaxKeyCols = 8;
constexpr int kMaxLocalKey = 64;     // encoded multi-column keys are built in registers/scratch
constexpr int kFreqHist = 1 << 16;   // count-of-counts bins kept on the device
constexpr int kFreqLdsHist = 2048;   // ... of which the first are aggregated in LDS

struct FreqSlot {  // 32 B; see dq_freq.hip for the ctrl word
  unsigned long long ctrl, count, k0, k1;
};

// The table is an array of 2^bucket_bits slices of kFreqSliceSlots slots; a key lives in the
// slice selected by the top bucket_bits bits of its hash and probes linearly inside it.  A
// slice (64 KiB of slots) is what one workgroup aggregates in LDS (dq_freq_agg_kernel).
constexpr int kFreqSliceLog = 11;
constexpr uint64_t kFreqSliceSlots = 1ull << kFreqSliceLog;
// Records per aggregation work item of a split (hot) bucket in the sorted-bucket path.
constexpr uint64_t kFreqAggPiece = 32768;
// Largest LDS bin count (log2) of one partition pass (dq_freq_part_kernel).
constexpr int kPartMaxBits = 11;

// A staged row of the sorted-bucket path: key bytes 0..14 (zero padded) in k0 and the low 7
// bytes of k1, the key length (<= 15) in the top byte of k1.
struct alignas(16) FreqRec {
  unsigned long long k0, k1;
};

// A staged row of a long or multi-column key (the hashed partition path, round 6): the key's
// table hash and a reference to its bytes, which the stage copied into the table's key heap
// (8-byte aligned, zero padded): ref = heap offset << 24 | key length.  A hole: ref = ~0.
struct alignas(16) HashRec {
  unsigned long long h, ref;
};
constexpr unsigned long long kHashHole = ~0ull;

// A staged row of a canonical UUID key (round 6, dq_uuidpack.h): its 36 text bytes packed into
// 128 bits.  The record is the key itself, so the splits and the slice aggregation group it in
// registers and LDS; the overflow and retry lists hold its bits as a FreqRec {lo, hi}, which
// dq_freq_uuid_to_hashed turns into a hashed record (text into the key heap) before a global insert.
struct alignas(16) UuidRec {
  unsigned long long lo, hi;
};

// A staged row of a 16-byte key (round 6): a single string column of 16-byte keys, or two 8-byte
// fixed-width columns (make_key's encoding: the two values' little-endian bits) -- the key bytes
// themselves, hashed as every 16-byte key is (hash_inline) and written inline into its slot.
struct alignas(16) Raw16Rec {
  unsigned long long lo, hi;
};

struct FreqTable {
  FreqSlot* slots;
  uint64_t mask;                   // capacity - 1 (capacity: a power of two >= kFreqSliceSlots)
  int32_t bucket_bits;             // log2(capacity / kFreqSliceSlots)
  int32_t test_flags;              // kFreqTestNoPublish: a test-only broken publish (0 otherwise)
  unsigned long long* n_groups;    // device counter of claimed slots
  uint8_t* heap;                   // key bytes of keys longer than 16 B
  unsigned long long* heap_used;
  unsigned long long heap_cap;
  unsigned int* overflow;          // bit 0 table full, bit 1 heap full, bit 2 key too long,
                                   // bit 3 a wait for another lane's slot publish timed out
};
constexpr unsigned int kFreqWaitTimeout = 8u;
constexpr int32_t kFreqTestNoPublish = 1;  // dq_diag_freq_test_flags (tests only): claimed slots never turn READY

// A compacted table (the packed aggregation into an empty table, round 6): the occupied slots
// only, each slice's groups in slot order from base[b] (num[b] of them), and per slice a 2048-bit
// occupancy bitmap (bits + 256 b: bit j of byte t = slot 8 t + j) from which dq_freq_expand
// rebuilds the slot image when an operation needs to probe.
struct FreqCompact {
  FreqSlot* slots;
  unsigned long long* base;
  uint32_t* num;
  uint8_t* bits;
  unsigned long long* cursor;
};

struct FreqKeySpec {
  int32_t key_cols[kMaxKeyCols];
  int32_t n_keys;
  int32_t null_as_key;  // Histogram: NULL is a group ("NullValue")
};

struct FreqOut {  // exported groups (device arrays of capacity `cap`)
  unsigned long long* ctrl;
  unsigned long long* count;
  unsigned long long* k0;
  unsigned long long* k1;
  unsigned long long* n;
  unsigned long long cap;
};

struct FreqIn {  // groups to merge in; heap offsets in k0 refer to `heap`
  const unsigned long long* ctrl;
  const unsigned long long* count;
  const unsigned long long* k0;
  const unsigned long long* k1;
  const uint8_t* heap;
  uint64_t n;
  uint64_t stride;  // elements between consecutive groups: 1 = separate arrays, 4 = FreqSlot records
};

// Key-hash exchange and table merges (dq_freq.hip, round 4).  A packed wire record: a key that
// packs into one word (dq_keypack.h) and its count.
struct WirePacked {
  unsigned long long key, count;
};
// One record stream a merge takes in: a part's packed section (kind 0), its general section
// (kind 1: FreqSlot, READY clear, k0 of a long key = offset in `heap`), or a source table's slot
// array (kind 2, src_bits = its slice bits).  skip = 1: out of slice order, inserted group by group.
// bits (wire runs): the slice bits its bounds are cut at -- the receiver's, or fewer when the run
// is in order only by its top `bits` hash bits (a sender that sorted by coarser slices or chunks
// than the receiver's slices); the merge then reads the coarser range and filters by slice.
constexpr int kImportFlatRuns = 16;  // packed runs the import merge takes as one index space
struct ImportRun {
  const void* recs;
  uint64_t n;
  const uint8_t* heap;
  int32_t kind;
  int32_t src_bits;
  int32_t skip;
  int32_t bits;
};
hipError_t launch_wire_count(const FreqTable& T, int n_parts, int chunk_log, uint64_t n_chunks, unsigned long long* d_cnt,
                             unsigned long long* d_kbytes, hipStream_t stream);
hipError_t launch_gather_strided(const unsigned long long* d_scanned, uint64_t stride, uint64_t n, unsigned long long* d_out,
                                 hipStream_t stream);
hipError_t launch_wire_scatter(const FreqTable& T, int n_parts, int chunk_log, uint64_t n_chunks,
                               const unsigned long long* d_pos, const unsigned long long* d_sec,
                               const unsigned long long* d_key_base, unsigned long long* d_key_cursor, uint8_t* d_out,
                               uint8_t* d_keys, hipStream_t stream);
hipError_t launch_import_sketch(const ImportRun* d_runs, int n_runs, uint64_t max_n, uint32_t* d_hll, hipStream_t stream);
hipError_t launch_import_bounds(const ImportRun* d_runs, int n_runs, uint64_t max_n, int rb, uint64_t n_slices,
                                uint32_t* d_start, uint32_t* d_end, unsigned int* d_unsorted, unsigned int* d_drop,
                                int rerun, hipStream_t stream);
hipError_t launch_import_merge(const FreqTable& T, bool packed, bool flat, const ImportRun* d_runs, int n_runs, const uint32_t* d_start,
                               const uint32_t* d_end, int table_empty, unsigned long long* d_hist, unsigned long long* d_big,
                               unsigned long long* d_n_big, unsigned long long big_cap, uint32_t* d_smax, int write_all,
                               uint32_t* d_ovf_list, unsigned long long* d_n_ovf, unsigned long long* d_ovf_recs,
                               unsigned long long* d_new_groups, hipStream_t stream);
hipError_t launch_import_global(const FreqTable& T, const ImportRun* d_runs, int n_runs, uint64_t max_n, int mode, int rb_old,
                                const uint32_t* d_start, const uint32_t* d_end, uint64_t n_slices_old,
                                const uint32_t* d_ovf_list, uint64_t n_ovf, hipStream_t stream);
// Few-groups group-by of one key column (dq_freq.hip): per-workgroup LDS tables, staging lists
// (kFreqSmallSlots entries per workgroup in d_k0 / d_k1 / d_c, d_n[block] used), one merge into T;
// *d_bad != 0: a key longer than 15 bytes or more keys than an LDS table holds (nothing merged).
constexpr int kFreqSmallSlots = 1024;
hipError_t launch_freq_small(const FreqKeySpec& ks, bool string_key, const DevColumn* d_cols, int64_t n_rows, int blocks,
                             unsigned long long* d_k0, unsigned long long* d_k1, uint32_t* d_c, uint32_t* d_n,
                             unsigned int* d_bad, const FreqTable& T, hipStream_t stream);
hipError_t launch_freq_insert(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                              const FreqTable& T, hipStream_t stream,
                              int max_blocks = 4096);
hipError_t launch_freq_hist(const FreqTable& T, unsigned long long* d_hist, unsigned long long* d_big,
                            unsigned long long* d_nbig, unsigned long long big_cap, hipStream_t stream);
hipError_t launch_freq_export(const FreqTable& T, unsigned long long min_count, const FreqOut& out,
                              hipStream_t stream, const uint32_t* d_smax = nullptr);
hipError_t launch_freq_import(const FreqTable& T, const FreqIn& in, hipStream_t stream);
// Flat (columnar) export in slot order (dq_freq.hip): chunk counts -> scanned chunk bases (the
// total at d_chunk_n[n_chunks]); then the groups' ctrl/count/k0/k1 arrays and the scanned key
// byte offsets (n + 1, the total at d_offs[n]); then the key bytes.  d_sums: scan scratch of
// ceil((max(n, n_chunks) + 1) / 4096) words.
uint64_t freq_flat_chunks(uint64_t slots);
hipError_t launch_freq_flat_count(const FreqTable& T, unsigned long long* d_chunk_n, uint64_t n_chunks,
                                  unsigned long long* d_sums, hipStream_t stream);
hipError_t launch_freq_flat_fill(const FreqTable& T, const unsigned long long* d_chunk_base, uint64_t n_chunks, uint64_t n,
                                 unsigned long long* d_ctrl, unsigned long long* d_count, unsigned long long* d_k0,
                                 unsigned long long* d_k1, unsigned long long* d_offs, unsigned long long* d_sums,
                                 hipStream_t stream);
hipError_t launch_freq_flat_keys(const FreqTable& T, const unsigned long long* d_ctrl, const unsigned long long* d_k0,
                                 const unsigned long long* d_k1, const unsigned long long* d_offs, uint64_t n,
                                 uint8_t* d_out, hipStream_t stream);
hipError_t launch_freq_import_flat(const FreqTable& T, const long long* d_counts, const long long* d_offs,
                                   const uint8_t* d_bytes, uint64_t n, hipStream_t stream);
hipError_t launch_freq_hash(const uint64_t* d_k0, const uint64_t* d_k1, const uint32_t* d_len, int64_t n, uint64_t* d_out,
                            hipStream_t stream);
hipError_t launch_freq_lookup(const FreqTable& T, const uint8_t* d_key, uint32_t len, unsigned long long* d_out,
                              hipStream_t stream, const FreqCompact* cmp = nullptr);
hipError_t launch_freq_heap_need(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                 unsigned long long* d_need, unsigned long long* d_max_len, hipStream_t stream);
// Sorted-bucket path (dq_freq.hip): stage rows as FreqRec + an HLL sketch of their hashes (to size
// the table), group them by slice (the bucket split below), then aggregate every slice's bucket
// in LDS (split buckets merge atomically).
hipError_t launch_freq_stage(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, FreqRec* d_out,
                             unsigned long long* d_cursor, uint32_t* d_hll, unsigned long long* d_long_key,
                             hipStream_t stream);
// The bucket split (dq_freq.hip): level 1 (d_in_off == nullptr) over d_in[0, n) by the top
// bits - b2 slice bits, level 2 over the n_regions exact regions of d_in_off by the low b2 bits;
// d_count != nullptr counts (adds to d_count[id]), else scatters into d_out at d_region_start[id]
// + cursor.  max_region: the largest level-2 input region.
hipError_t launch_freq_split(const FreqRec* d_in, uint64_t n, const unsigned long long* d_in_off, uint64_t n_regions,
                             uint64_t max_region, int bits, int b2, unsigned long long* d_count, FreqRec* d_out,
                             const unsigned long long* d_region_start, unsigned long long* d_cursor, hipStream_t stream);
// In-place exclusive scans (d_sums: ceil(n / 4096) scratch words).
hipError_t scan_exclusive_u64(unsigned long long* d_data, uint64_t n, unsigned long long* d_sums, hipStream_t stream);
hipError_t scan_exclusive_u32(uint32_t* d_data, uint64_t n, uint32_t* d_sums, hipStream_t stream);
// pieces[b] = aggregation work items of slice b (b < n), pieces[n] = 0
hipError_t launch_freq_pieces(const unsigned long long* d_counts, uint64_t n, uint32_t* d_pieces, hipStream_t stream);
hipError_t launch_freq_agg(const FreqTable& T, const FreqRec* d_recs, const uint64_t* d_off,
                           const uint32_t* d_piece_start, uint64_t n_buckets, uint64_t max_items, int table_empty,
                           FreqRec* d_retry, unsigned long long* d_n_retry, unsigned long long* d_new_groups,
                           hipStream_t stream);
// Partition path (dq_freq.hip): stage array (d_in_fill == nullptr) or regions -> regions of
// out_cap records by the top id_bits of the table hash; overflow -> d_ovf (d_flag bit 0 when
// that is full too).  Then one owner work item per slice region.  packed: the records are
// packed digit keys (uint64_t, dq_keypack.h), else FreqRec; the overflow / retry lists always
// hold FreqRec.
hipError_t launch_freq_part(const void* d_in, uint64_t in_n, const unsigned long long* d_in_fill, uint64_t in_cap,
                            uint64_t n_in_regions, int id_bits, int bin_bits, void* d_out, uint64_t out_cap,
                            unsigned long long* d_out_fill, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                            uint64_t ovf_cap, unsigned int* d_flag, int rec_kind, hipStream_t stream,
                            unsigned long long* d_staged = nullptr);
constexpr int kRecFree = 0, kRecPacked = 1, kRecHashed = 2, kRecUuid = 3, kRecRaw16 = 4;  // FreqRec, packed word, HashRec, UuidRec, Raw16Rec
// With an empty table it can also produce the count-of-counts histogram (d_hist, counts >=
// kFreqHist into d_big), each slice's largest count (d_smax) and write every slot (write_all:
// the table needs no clearing).
// Stage + level-1 partition in one pass (records straight into their 2^b1 level-1 regions);
// regions -> contiguous (prefix = exclusive sum of the clamped fills) for the sort path.
// one_string: the only key column is utf8 (the kernel's batched-load fast path); packed (needs
// one_string): digit keys staged as packed words, other keys onto the overflow list.
hipError_t launch_freq_pack_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                  hipStream_t stream, unsigned long long* d_long = nullptr);
// dq_profile.hip: ApproxCountDistinct registers (ranks, 512) and the five DataType counts of a
// utf8 column from its flat groups (dq_profile_string_groups); both zeroed by the caller.
hipError_t launch_string_groups(const int64_t* d_counts, const int64_t* d_offs, const uint8_t* d_bytes, int64_t n,
                                uint32_t* d_regs, unsigned long long* d_dtc, hipStream_t stream);
// ... and over n_cols such lists (column y: d_k0 / d_k1 / d_counts + y * max_n, d_n[y], registers
// d_regs + y * kHllM, counts d_dtc + y * 8).
hipError_t launch_string_groups_words(const unsigned long long* d_k0, const unsigned long long* d_k1,
                                      const unsigned long long* d_counts, const uint32_t* d_n, uint32_t max_n, int n_cols,
                                      uint32_t* d_regs, unsigned long long* d_dtc, hipStream_t stream);
// dq_freq.hip: the few-groups kernel over n_cols columns (d_cols[0 .. n_cols), one launch,
// blockIdx.y = column) + each column's lists summed into one compact list: column y's groups at
// out_*[y * kFreqSmallSlots ..][0, out_n[y]), bad[y] raised when it did not fit.  The lists:
// d_k0 / d_k1 / d_c hold n_cols * blocks * kFreqSmallSlots entries, d_n n_cols * blocks.
hipError_t launch_freq_small_flat(bool string_key, const FreqKeySpec& ks, const DevColumn* d_cols, int n_cols,
                                  int64_t n_rows, int blocks, unsigned long long* d_k0, unsigned long long* d_k1,
                                  uint32_t* d_c, uint32_t* d_n, unsigned int* d_bad, unsigned long long* d_out_k0,
                                  unsigned long long* d_out_k1, unsigned long long* d_out_c, uint32_t* d_out_n,
                                  hipStream_t stream);
hipError_t launch_freq_stage_save(const unsigned long long* d_fill, unsigned long long* d_fill_save, uint32_t n_fill,
                                  const uint32_t* d_sketch, uint32_t* d_sketch_save, const unsigned long long* d_ovf_n,
                                  unsigned long long* d_ovf_save, unsigned long long* d_long_key, hipStream_t stream);
hipError_t launch_freq_stage_part(const FreqKeySpec& ks, bool one_string, bool packed, const DevColumn* d_cols,
                                  int64_t n_rows, int b1, void* d_out,
                                  uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                                  uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll, unsigned long long* d_long_key,
                                  unsigned long long* d_staged, hipStream_t stream,
                                  void* d_rows = nullptr);
// The hashed partition path (dq_freq.hip, round 6).  Stage: every row's key (make_key: long
// strings, several columns) is copied to the key heap (one atomic per wave) and written as a
// HashRec in row order (holes for NULL keys); too_long: a multi-column key over kMaxLocalKey.
hipError_t launch_freq_stage_hashed(const FreqKeySpec& ks, bool one_string, const DevColumn* d_cols, int64_t n_rows, HashRec* d_out,
                                    const FreqTable& T, uint32_t* d_hll, unsigned long long* d_too_long,
                                    unsigned long long* d_staged, unsigned long long* d_max_len, hipStream_t stream);
// Heap bytes of exported groups gathered to d_dst at d_off[i] (8-byte aligned; heap keys only).
hipError_t launch_freq_gather_keys(const uint8_t* d_heap, const unsigned long long* d_ctrl, const unsigned long long* d_k0,
                                   const unsigned long long* d_off, uint64_t n, uint8_t* d_dst, hipStream_t stream);
// Exact bytes the stage will append to the heap for n_rows rows (sum of 8-aligned key lengths).
hipError_t launch_freq_key_bytes(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                 unsigned long long* d_out, hipStream_t stream);
// The UUID partition path (dq_freq.hip, round 6; dq_uuidpack.h).  Stage + level-1 split of a
// single utf8 key column of canonical UUIDs into UuidRec regions (d_bad: non-NULL keys that are
// not canonical UUIDs -- the caller rolls such a batch back); in-place conversion of a list of
// UuidRec bits (retry / overflow) into hashed records, their text written to T's heap; the probe
// of a batch's keys (d_out[0] non-canonical, d_out[1] canonical, of a sample).
hipError_t launch_freq_stage_uuid(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, int b1, void* d_out,
                                  uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf, unsigned long long* d_ovf_n,
                                  uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll, unsigned long long* d_bad,
                                  unsigned long long* d_staged, hipStream_t stream);
hipError_t launch_freq_uuid_to_hashed(const FreqTable& T, FreqRec* d_recs, uint64_t n, hipStream_t stream,
                                      int rec_kind = kRecUuid);
// The 16-byte-key form (Raw16Rec): stage + level-1 split of one string column of 16-byte keys
// (d_bad: non-NULL keys of another length) or of two 8-byte fixed-width columns.
hipError_t launch_freq_stage_raw16(const FreqKeySpec& ks, bool one_string, const DevColumn* d_cols, int64_t n_rows,
                                   int b1, void* d_out, uint64_t cap1, unsigned long long* d_fill1, FreqRec* d_ovf,
                                   unsigned long long* d_ovf_n, uint64_t ovf_cap, unsigned int* d_flag, uint32_t* d_hll,
                                   unsigned long long* d_bad, unsigned long long* d_staged, hipStream_t stream);
// Sampled non-NULL keys of a single string column whose length is not 16, added to d_out[0].
hipError_t launch_freq_len16_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows,
                                   unsigned long long* d_out, hipStream_t stream);
// Sampled rows (16384 scattered, as the pack probe) whose encoded key (make_key) is longer than
// 15 bytes, added to *d_out: a multi-column table's choice of hashed records from the start.
hipError_t launch_freq_len_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                 hipStream_t stream);
hipError_t launch_freq_uuid_probe(const FreqKeySpec& ks, const DevColumn* d_cols, int64_t n_rows, unsigned long long* d_out,
                                  hipStream_t stream);
// Global inserts of n hashed records (the list form: FreqRec bits of HashRec), their key bytes
// already in T's heap: the retry / overflow records and the fall-back of the hashed path.
hipError_t launch_freq_insert_hashed(const FreqTable& T, const FreqRec* d_recs, uint64_t n, hipStream_t stream);
hipError_t launch_freq_compact(const void* d_in, bool packed, const unsigned long long* d_fill, uint64_t cap,
                               uint64_t n_regions, const unsigned long long* d_prefix, FreqRec* d_out, hipStream_t stream);
hipError_t launch_freq_agg_region(const FreqTable& T, const void* d_recs, int rec_kind, const unsigned long long* d_fill,
                                  uint64_t cap, uint64_t n_slices, int table_empty, FreqRec* d_retry,
                                  unsigned long long* d_n_retry, unsigned long long* d_new_groups,
                                  unsigned long long* d_hist, unsigned long long* d_big, unsigned long long* d_n_big,
                                  unsigned long long big_cap, uint32_t* d_smax, int write_all, hipStream_t stream,
                                  const FreqCompact* compact = nullptr);
// A compacted table's slot image rebuilt into T (every slot written), and its groups exported
// (as launch_freq_export with slice maxima).
hipError_t launch_freq_expand(const FreqTable& T, const FreqCompact& cmp, hipStream_t stream);
hipError_t launch_freq_export_compact(const FreqCompact& cmp, uint64_t n_slices, unsigned long long min_count,
                                      const FreqOut& out, const uint32_t* d_smax, hipStream_t stream);
hipError_t launch_freq_rehash(const FreqSlot* d_old, uint64_t old_n, const FreqTable& T, hipStream_t stream);

// ---------------------------------------------------------------- launchers (.hip files)
// kind 0 = validity/mask-only tasks, 1 = value tasks of column type `ptype` with exactly
// `np` inline predicates (np > 4 uses the 8-slot kernel; np < 0 = tasks with a where mask
// or mask predicates).  Partials of the group's i-th task go to
// d_partials[i * blocks_per_task + b].
hipError_t launch_scan_group(int kind, int ptype, int np, const ScanTask* d_tasks,
                             const int32_t* d_group, int n_group, const DevColumn* d_cols,
                             const DevMask* d_masks, int64_t n_rows, int blocks_per_task,
                             ScanAcc* d_partials, uint32_t* d_hll_regs, hipStream_t stream);
// The specialised 8-byte value scan (dq_scan_fast.hip): `variant` = predicate form (low 3 bits:
// 0 none, 1 int64 `<`, 2 int64 `==`, 3 fp64 `<`, 4 fp64 `==`; CS_INV of the task's predicate
// negates it) | FAST_STATS | FAST_HLL.
constexpr int FAST_STATS = 8;
constexpr int FAST_HLL = 16;
hipError_t launch_scan_fast(int ptype, int variant, const ScanTask* d_tasks, const int32_t* d_group, int n_group,
                            const DevColumn* d_cols, int64_t n_rows, int blocks_per_task, ScanAcc* d_partials,
                            uint32_t* d_hll_regs, hipStream_t stream);
int scan_fast_blocks_per_cu(int ptype, int variant);  // 0 = unknown
hipError_t launch_diag_hash(int blocks, int iters, bool with_hll, uint64_t* sink, hipStream_t s);
int scan_group_blocks_per_cu(int kind, int ptype, int np);  // 0 = unknown
hipError_t launch_scan_reduce(const ScanAcc* d_partials, const PartRange* d_ranges, int n_tasks,
                              ScanAcc* d_acc, hipStream_t stream);
hipError_t launch_string_pass(const StrTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                              int64_t n_rows, int blocks_per_task, uint32_t* d_registers, unsigned long long* d_counts,
                              hipStream_t stream);
hipError_t launch_hll(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols,
                      const DevMask* d_masks, int64_t n_rows, int blocks_per_task,
                      uint32_t* d_registers, hipStream_t stream);
hipError_t launch_predicates(const PredProgram* d_progs, int n_progs, const PredInsn* d_insns,
                             const uint8_t* d_pool, const DevColumn* d_cols, int64_t n_rows,
                             uint64_t* d_mask_words, int64_t words_per_mask, bool with_cast, hipStream_t stream);
hipError_t launch_rebase_offsets(int32_t* d_offs, int64_t n, int32_t first, hipStream_t stream);
hipError_t launch_realign_bitmap(const uint8_t* src, int64_t bit_offset, int64_t n_bits,
                                 uint8_t* dst, hipStream_t stream);
hipError_t launch_init_acc(ScanAcc* d_acc, int n, hipStream_t stream);
// DataType (dq_profile.hip): tasks reuse HllTask {column, type, where}; 5 u64 counts per task.
hipError_t launch_datatype(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                           int64_t n_rows, int blocks_per_task, unsigned long long* d_counts, hipStream_t stream);
// MinLength / MaxLength (dq_pair.hip): tasks {column, type, where}; 3 u64 per task
// {selected rows, max of ~length, max of length}.
hipError_t launch_strlen(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                         int64_t n_rows, int blocks_per_task, unsigned long long* d_out, hipStream_t stream);
// Correlation (dq_pair.hip): per-block partials (n_tasks x blocks_per_task), then merged into d_acc.
hipError_t launch_corr(const CorrTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                       int64_t n_rows, int blocks_per_task, CorrAcc* d_partials, CorrAcc* d_acc,
                       hipStream_t stream);
hipError_t launch_cast_utf8(const DevColumn& src, int64_t n_rows, int to_type, void* d_values, uint8_t* d_validity,
                            hipStream_t stream);

// ---------------------------------------------------------------- XXH64 (host + device)
constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t kP2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t kP3 = 0x165667B19E3779F9ull;
constexpr uint64_t kP4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t kP5 = 0x27D4EB2F165667C5ull;

__host__ __device__ inline uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
__host__ __device__ inline uint64_t xxh_round(uint64_t acc, uint64_t lane) {
  acc += lane * kP2;
  acc = rotl64(acc, 31);
  return acc * kP1;
}
__host__ __device__ inline uint64_t xxh_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}
// Spark XXH64.hashLong(v, seed): XXH64 of the 8 little-endian bytes of v.
__host__ __device__ inline uint64_t xxh64_u64(uint64_t v, uint64_t seed) {
  uint64_t h = seed + kP5 + 8;
  h ^= xxh_round(0, v);
  h = rotl64(h, 27) * kP1 + kP4;
  return xxh_avalanche(h);
}
// Spark XXH64.hashInt(i, seed): XXH64 of the 4 little-endian bytes of i.
__host__ __device__ inline uint64_t xxh64_u32(uint32_t v, uint64_t seed) {
  uint64_t h = seed + kP5 + 4;
  h ^= (uint64_t)v * kP1;
  h = rotl64(h, 23) * kP2 + kP3;
  return xxh_avalanche(h);
}

// HLL register index and rank (StatefulHyperloglogPlus.scala:96-99).
__host__ __device__ inline void hll_idx_rank(uint64_t x, uint32_t* idx, uint32_t* pw) {
  *idx = (uint32_t)(x >> kHllIdxShift);
  uint64_t w = (x << 9) | kHllWPadding;
#if defined(__HIP_DEVICE_COMPILE__)
  *pw = (uint32_t)__clzll((long long)w) + 1u;
#else
  *pw = (uint32_t)__builtin_clzll(w) + 1u;
#endif
}

// Spark 2.2.2 XxHash64Function (seed 42) of one value by type (InterpretedHashFunction):
// the int family hashes as a 4-byte int, long as 8 bytes, float / double through
// floatToIntBits / doubleToLongBits (one canonical NaN, no -0.0 normalisation in 2.2).
template <typename T> __host__ __device__ inline uint64_t spark_hash(T v);
template <> __host__ __device__ inline uint64_t spark_hash<int8_t>(int8_t v) { return xxh64_u32((uint32_t)(int32_t)v, 42); }
template <> __host__ __device__ inline uint64_t spark_hash<int16_t>(int16_t v) { return xxh64_u32((uint32_t)(int32_t)v, 42); }
template <> __host__ __device__ inline uint64_t spark_hash<int32_t>(int32_t v) { return xxh64_u32((uint32_t)v, 42); }
template <> __host__ __device__ inline uint64_t spark_hash<int64_t>(int64_t v) { return xxh64_u64((uint64_t)v, 42); }
template <> __host__ __device__ inline uint64_t spark_hash<float>(float v) {
  uint32_t bits;
  __builtin_memcpy(&bits, &v, 4);
  if (v != v) bits = 0x7fc00000u;  // Float.floatToIntBits canonical NaN
  return xxh64_u32(bits, 42);
}
template <> __host__ __device__ inline uint64_t spark_hash<double>(double v) {
  uint64_t bits;
  __builtin_memcpy(&bits, &v, 8);
  if (v != v) bits = 0x7ff8000000000000ull;  // Double.doubleToLongBits canonical NaN
  return xxh64_u64(bits, 42);
}

// ---------------------------------------------------------------- device XXH64 on 32-bit halves
// The same Spark XXH64 (seed 42) as xxh64_u64 / xxh64_u32 above, written for the gfx950 VALU,
// where the per-row hash is the bound of every fused HLL pass (each instruction here is one
// issue slot of 64 rows):
//   * a 64x64-bit multiply by a constant is one v_mad_u64_u32 (lo x lo, with the constant
//     addend of the next step folded in) + two v_mul_lo_u32 for the cross terms;
//   * a 64-bit rotate is two v_alignbit_b32; rotl27(S ^ k) = rotl27(S) ^ rotl27(k) folds the
//     seed word into one constant;
//   * the avalanche shifts by 33 / 29 / 32 touch only the halves they move.
// Bit-identical to xxh64_u64 / xxh64_u32 (pinned by the GPU HLL register parity tests).
struct W64 {
  uint32_t lo, hi;
};

template <uint64_t C, uint64_t A = 0>
__device__ inline W64 w64_mul(W64 a) {  // a * C + A (mod 2^64)
  const uint64_t p = (uint64_t)a.lo * (uint32_t)C + A;
  const uint32_t hi = (uint32_t)(p >> 32) + a.lo * (uint32_t)(C >> 32) + a.hi * (uint32_t)C;
  return {(uint32_t)p, hi};
}
template <int R>  // rotl64 by 0 < R < 32
__device__ inline W64 w64_rotl(W64 x) {
  return {__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - R), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - R)};
}
// The avalanche up to (not including) the final h ^= h >> 32, which only moves the high word
// into the low one: the HLL slot reads the high word directly (hll_slot).
__device__ inline W64 w64_avalanche_pre32(W64 h) {
  h.lo ^= h.hi >> 1;                                   // h ^= h >> 33
  h = w64_mul<kP2>(h);
  h.lo ^= __builtin_amdgcn_alignbit(h.hi, h.lo, 29);  // h ^= h >> 29
  h.hi ^= h.hi >> 29;
  return w64_mul<kP3>(h);
}
__device__ inline W64 w64_avalanche(W64 h) {
  h = w64_avalanche_pre32(h);
  h.lo ^= h.hi;                                        // h ^= h >> 32
  return h;
}
constexpr uint64_t rotl64_c(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// xxh64_*_dev return the hash BEFORE its last step (x = h ^ (h >> 32)): xxh64_final() applies it.
__device__ inline W64 xxh64_final(W64 h) { return {h.lo ^ h.hi, h.hi}; }
__device__ inline W64 xxh64_8_dev(uint32_t lo, uint32_t hi) {  // Spark XXH64.hashLong, seed 42
  constexpr uint64_t RS = rotl64_c(42ull + kP5 + 8, 27);
  W64 k = w64_mul<kP2>({lo, hi});
  k = w64_mul<kP1>(w64_rotl<31>(k));
  W64 h = w64_rotl<27>(k);
  h.lo ^= (uint32_t)RS;
  h.hi ^= (uint32_t)(RS >> 32);
  return w64_avalanche_pre32(w64_mul<kP1, kP4>(h));
}
__device__ inline W64 xxh64_4_dev(uint32_t v) {  // Spark XXH64.hashInt, seed 42
  constexpr uint64_t RS = rotl64_c(42ull + kP5 + 4, 23);
  const uint64_t p = (uint64_t)v * (uint32_t)kP1;
  W64 h = w64_rotl<23>({(uint32_t)p, (uint32_t)(p >> 32) + v * (uint32_t)(kP1 >> 32)});
  h.lo ^= (uint32_t)RS;
  h.hi ^= (uint32_t)(RS >> 32);
  return w64_avalanche_pre32(w64_mul<kP2, kP3>(h));
}

// spark_hash<T> on the device, as halves.
template <typename T> __device__ inline W64 spark_hash_dev(T v) {
  return xxh64_4_dev((uint32_t)(int32_t)v);  // the int family hashes as a 4-byte int
}
template <> __device__ inline W64 spark_hash_dev<int64_t>(int64_t v) {
  return xxh64_8_dev((uint32_t)(uint64_t)v, (uint32_t)((uint64_t)v >> 32));
}
// doubleToLongBits / floatToIntBits map every NaN to the canonical one; NaN rows are rare, so
// the rewrite sits behind a wave-uniform branch.
template <> __device__ inline W64 spark_hash_dev<double>(double v) {
  uint64_t bits = __builtin_bit_cast(uint64_t, v);
  if (__ballot(v != v)) bits = (v != v) ? 0x7ff8000000000000ull : bits;
  return xxh64_8_dev((uint32_t)bits, (uint32_t)(bits >> 32));
}
template <> __device__ inline W64 spark_hash_dev<float>(float v) {
  uint32_t bits = __builtin_bit_cast(uint32_t, v);
  if (__ballot(v != v)) bits = (v != v) ? 0x7fc00000u : bits;
  return xxh64_4_dev(bits);
}

// Register index and rank of a hash (StatefulHyperloglogPlus.scala:96-99) from its halves:
// idx = x >>> 55, pw = nlz((x << 9) | W_PADDING) + 1.
__device__ inline uint32_t ffbh_u32(uint32_t v) {  // v_ffbh_u32: leading zeros, ~0u for 0
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
// idx and nlz = pw - 1.  The high word of w = (x << 9) | W_PADDING is zero for one hash in 2^32:
// that case (nlz >= 32) is taken on a wave-uniform branch instead of paying a 64-bit count
// on every row.
// `h` is the pre-final hash (xxh64_*_dev): x = h ^ (h >> 32) has x.hi = h.hi, and the bits of
// w below its top 23 only matter when those 23 (bits 22..0 of x.hi) are all zero, so the
// common case counts on h.hi << 9 alone.
__device__ inline void hll_slot(W64 h, uint32_t& idx, uint32_t& nlz) {
  idx = h.hi >> (kHllIdxShift - 32);
  nlz = ffbh_u32(h.hi << 9);
  if (__ballot(nlz == ~0u)) {
    const W64 x = xxh64_final(h);
    const uint32_t w_hi = __builtin_amdgcn_alignbit(x.hi, x.lo, 23);  // (x << 9) >> 32
    const uint32_t w_lo = (x.lo << 9) | (uint32_t)kHllWPadding;
    if (nlz == ~0u) nlz = (w_hi != 0u) ? ffbh_u32(w_hi) : 32u + ffbh_u32(w_lo);
  }
}

// Hash one value and raise its register in the workgroup's LDS copy: a register only grows,
// so every row issues one ds_max_u32 with no return value (nothing to wait for); a row that is
// not selected raises nothing (rank 0).  `s` = 1 (row selected) or 0.
template <typename T>
__device__ inline void hll_hash_update(uint32_t* regs, T v, uint32_t s) {
  uint32_t idx, nlz;
  hll_slot(spark_hash_dev<T>(v), idx, nlz);
  // rank * s = nlz * s + s: one v_mad_u32_u24 (the compiler would rebuild an add and a select
  // from the plain expression)
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %2" : "=v"(r) : "v"(nlz), "v"(s));
  __hip_atomic_fetch_max(&regs[idx], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// M[idx] = max(M[idx], pw) on a workgroup's LDS register copy; the atomic is skipped when the
// register already holds >= pw (after a few thousand rows almost every update is a no-op).
__device__ inline void hll_update_lds(uint32_t* regs, uint64_t x) {
  uint32_t idx, pw;
  hll_idx_rank(x, &idx, &pw);
  if (pw > regs[idx]) atomicMax(&regs[idx], pw);
}

}  // namespace dq
