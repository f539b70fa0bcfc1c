/*
 * deequ_amd.h -- C-ABI of the MI355X-native backend for deequ's metric hot path.
 *
 * This is the drop-in boundary named by SURVEY.md §8(b).  In the reference there is no
 * FFI: the seam is the Scala trait pair
 *     ScanShareableAnalyzer.aggregationFunctions() / fromAggregationResult()
 *         (src/main/scala/com/amazon/deequ/analyzers/Analyzer.scala:169-197)
 *     State.sum                                    (Analyzer.scala:34-48)
 * and the single launch site of the fused scan
 *     data.agg(aggs.head, aggs.tail: _*).collect().head   (runners/AnalysisRunner.scala:313)
 * plus the grouping launch site
 *     FrequencyBasedAnalyzer.computeFrequencies   (analyzers/GroupingAnalyzers.scala:53-80).
 * A JNI shim replaces those call sites for GPU-eligible analyzers: it
 * creates a plan from the analyzers, feeds Arrow-layout column batches, and turns the POD
 * states returned here into the unchanged Scala `State` case classes, which then flow into
 * Analyzer.calculateMetric (Analyzer.scala:107-128) exactly as Spark-produced states do.
 *
 * Conventions
 *   - Every function returns dq_status (0 = OK).  No C++ exception crosses the ABI.
 *     dq_last_error() returns a thread-local message for the last failure.
 *   - Columns use the Arrow layout: validity bitmap LSB-first, 1 = valid (NULL pointer = no
 *     nulls), fixed-width values, utf8 = int32 offsets + bytes.  A column's buffers are either
 *     host memory (copied to HBM by the library) or device memory on the context's GPU
 *     (DQ_COL_DEVICE; used in place, never copied).
 *   - Plans are not thread-safe; use one plan per calling thread.  Contexts may be shared.
 */
#ifndef DEEQU_AMD_H
#define DEEQU_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQ_ABI_VERSION 4

/* ---------------------------------------------------------------- status codes */
typedef enum dq_status {
  DQ_OK = 0,
  DQ_ERR_INVALID = 1,      /* bad argument (maps to IllegalArgumentException)           */
  DQ_ERR_UNSUPPORTED = 2,  /* op/type/predicate not on the GPU path: route it to Spark   */
  DQ_ERR_DEVICE = 3,       /* HIP runtime failure or no usable gfx950 device             */
  DQ_ERR_OOM = 4,          /* device allocation failed                                   */
  DQ_ERR_STATE = 5,        /* call out of order (e.g. consume after finish without reset)*/
  DQ_ERR_SPACE = 6         /* caller's output buffer too small: required sizes returned  */
} dq_status;

/* ---------------------------------------------------------------- column types */
typedef enum dq_type {
  DQ_T_BOOL = 1,     /* Arrow bit-packed boolean                    (Spark BooleanType) */
  DQ_T_INT8 = 2,     /*                                             (ByteType)          */
  DQ_T_INT16 = 3,    /*                                             (ShortType)         */
  DQ_T_INT32 = 4,    /*                                             (IntegerType)       */
  DQ_T_INT64 = 5,    /*                                             (LongType)          */
  DQ_T_FLOAT32 = 6,  /*                                             (FloatType)         */
  DQ_T_FLOAT64 = 7,  /*                                             (DoubleType)        */
  DQ_T_UTF8 = 8      /* int32 offsets + UTF-8 bytes                 (StringType)        */
} dq_type;

#define DQ_COL_DEVICE 0x1 /* validity/values/offsets are device pointers on ctx's GPU */

typedef struct dq_column {
  int32_t type;             /* dq_type                                                   */
  int32_t flags;            /* DQ_COL_*                                                  */
  int64_t length;           /* number of rows in this batch                             */
  int64_t offset;           /* Arrow slot offset of row 0 (elements; bits for bitmaps)  */
  const uint8_t* validity;  /* LSB-first bitmap, 1 = valid; NULL = no nulls             */
  const void* values;       /* fixed-width values, bit-packed bools, or utf8 bytes      */
  const int32_t* offsets;   /* utf8 only: length+1 offsets (from `offset`)              */
} dq_column;

/* ---------------------------------------------------------------- analyzer ops */
typedef enum dq_op_kind {
  DQ_OP_SIZE = 1,                  /* Size(where)                       Size.scala:35-47        */
  DQ_OP_COMPLETENESS = 2,          /* Completeness(column, where)       Completeness.scala:26-46*/
  DQ_OP_COMPLIANCE = 3,            /* Compliance(instance, pred, where) Compliance.scala:37-53  */
  DQ_OP_SUM = 4,                   /* Sum(column, where)                Sum.scala:35-52         */
  DQ_OP_MEAN = 5,                  /* Mean(column, where)               Mean.scala:36-54        */
  DQ_OP_STDDEV = 6,                /* StandardDeviation(column, where)  StandardDeviation.scala:47-73 */
  DQ_OP_MINIMUM = 7,               /* Minimum(column, where)            Minimum.scala:35-53     */
  DQ_OP_MAXIMUM = 8,               /* Maximum(column, where)            Maximum.scala:35-53     */
  DQ_OP_APPROX_COUNT_DISTINCT = 9, /* ApproxCountDistinct(column, where) ApproxCountDistinct.scala:47-64 */
  DQ_OP_DATATYPE = 10,             /* DataType(column, where)           DataType.scala:152-183  */
  DQ_OP_MIN_LENGTH = 11,           /* MinLength(column, where)          MinLength.scala:25-41   */
  DQ_OP_MAX_LENGTH = 12,           /* MaxLength(column, where)          MaxLength.scala:25-41   */
  DQ_OP_CORRELATION = 13           /* Correlation(column, column2, where) Correlation.scala:77-105 */
} dq_op_kind;

/*
 * Predicate IR: an analyzed Catalyst boolean expression (casts resolved) in postfix form.
 * It covers what deequ's Check DSL emits for numeric columns (Check.scala:594-943:
 * comparisons, COALESCE, IN, BETWEEN, IS [NOT] NULL, AND/OR/NOT) with SQL three-valued
 * logic.  Anything else is rejected with DQ_ERR_UNSUPPORTED at plan time.
 *
 * Value instructions push a typed value (int64, fp64 or UTF-8 string, each with a NULL flag);
 * boolean instructions pop/push three-valued booleans.  Numeric comparisons compare in the type
 * given by `arg` (DQ_CMP_AS_INT64 / DQ_CMP_AS_FLOAT64), converting operands first; two strings
 * compare byte-wise (unsigned, then by length), as Spark's UTF8String.compareTo.
 *
 * Type rules the library enforces (anything it cannot evaluate exactly as Spark would is
 * DQ_ERR_UNSUPPORTED, so the caller routes the analyzer to Spark; a malformed program -- stack
 * underflow, a column out of range -- is DQ_ERR_INVALID):
 *   - DQ_CMP_AS_INT64 with a floating-point operand;
 *   - a FloatType value (a FLOAT32 column or DQ_P_CAST to FLOAT32) compared or COALESCEd with an
 *     integral operand: Spark coerces that pair to FloatType, so the integral side must carry an
 *     explicit DQ_P_CAST to FLOAT32 (an integral literal may instead be rounded to float by the
 *     encoder and pushed with DQ_P_LIT_FLOAT);
 *   - a string compared with a non-string (only DQ_P_CAST_DOUBLE converts strings);
 *   - DQ_P_CAST of a string.
 */
typedef enum dq_pred_opcode {
  DQ_P_COLUMN = 1,     /* push value of batch column `arg`                                  */
  DQ_P_LIT_INT = 2,    /* push int64 literal `i64`                                          */
  DQ_P_LIT_FLOAT = 3,  /* push fp64 literal `f64`                                           */
  DQ_P_LIT_NULL = 4,   /* push NULL                                                         */
  DQ_P_COALESCE = 5,   /* pop b, a; push a if a non-NULL else b                             */
  DQ_P_LIT_STRING = 6, /* push UTF-8 literal strings[i64 .. i64 + arg) of the predicate      */
  DQ_P_CAST_DOUBLE = 7, /* pop value; push it as fp64: Spark 2.2 Cast(-> DoubleType), which a
                           comparison of a string with a number inserts (PromoteStrings): a string
                           through java.lang.Double.parseDouble of its trimmed text, NULL when
                           unparsable; correctly rounded for every input (decimal of any
                           length and exponent, hexadecimal, NaN / Infinity, f/d suffix).   */
  DQ_P_CAST = 8,       /* pop value; push Cast(value -> `arg`), `arg` a dq_type: INT8..INT64,
                           FLOAT32, FLOAT64 or BOOL, of a numeric or boolean value (Spark 2.2.2
                           Cast, non-ANSI: integral narrowing keeps the low bits; fractional ->
                           int/long is Java d2i/d2l, NaN -> 0, saturating; -> short/byte is d2i
                           then the low bits; integral -> float rounds the integer itself (l2f);
                           -> boolean is value != 0; boolean -> numeric 1/0).  The analyzer's
                           Cast nodes (`cast(l as int) > 3`, the FloatType side of `f = 16777217`)
                           map 1:1 onto it.  A cast of a string other than DQ_P_CAST_DOUBLE is
                           DQ_ERR_UNSUPPORTED (route the analyzer to Spark).                     */
  DQ_P_EQ = 10, DQ_P_NE = 11, DQ_P_LT = 12, DQ_P_LE = 13, DQ_P_GT = 14, DQ_P_GE = 15,
  DQ_P_EQ_NULLSAFE = 16, /* <=>                                                             */
  DQ_P_IS_NULL = 20,   /* pop value; push boolean (never NULL)                              */
  DQ_P_IS_NOT_NULL = 21,
  DQ_P_AND = 30, DQ_P_OR = 31, DQ_P_NOT = 32,
  DQ_P_TRUE = 33, DQ_P_FALSE = 34
} dq_pred_opcode;

#define DQ_CMP_AS_INT64 0
#define DQ_CMP_AS_FLOAT64 1

typedef struct dq_pred_insn {
  int32_t opcode;  /* dq_pred_opcode                                   */
  int32_t arg;     /* column index (DQ_P_COLUMN) or DQ_CMP_AS_* (cmp)  */
  int64_t i64;
  double f64;
} dq_pred_insn;

typedef struct dq_predicate {
  const dq_pred_insn* code;  /* NULL/0 = no predicate                     */
  int32_t n_insns;
  int32_t strings_len;       /* bytes in `strings`                        */
  const uint8_t* strings;    /* pool for DQ_P_LIT_STRING (may be NULL)    */
} dq_predicate;

typedef struct dq_op {
  int32_t kind;              /* dq_op_kind                                     */
  int32_t column;            /* batch column index; ignored for SIZE/COMPLIANCE */
  int32_t column2;           /* CORRELATION: the second column (secondColumn)    */
  int32_t reserved;          /* 0                                                */
  dq_predicate predicate;    /* COMPLIANCE only                                */
  dq_predicate where;        /* optional filter (Analyzers.conditionalSelection) */
} dq_op;

/* ---------------------------------------------------------------- states */
#define DQ_HLL_NUM_WORDS 52   /* StatefulHyperloglogPlus.scala:154 */

/*
 * POD image of the Scala State returned for one op.  `has_value` = 0 is Scala `None`
 * (Spark returned SQL NULL, e.g. Mean over an all-NULL column).  Which fields are meaningful
 * depends on `kind`:
 *   SIZE                         NumMatches(num_matches)
 *   COMPLETENESS, COMPLIANCE     NumMatchesAndCount(num_matches, count)
 *   SUM                          SumState(sum)
 *   MEAN                         MeanState(sum, count)
 *   STDDEV                       StandardDeviationState(n, avg, m2)
 *   MINIMUM / MAXIMUM            MinState(value) / MaxState(value)
 *   APPROX_COUNT_DISTINCT        ApproxCountDistinctState(words)  (always has_value = 1)
 *   DATATYPE                     DataTypeHistogram(words[0..4] = numNull, numFractional,
 *                                numIntegral, numBoolean, numString)  (always has_value = 1:
 *                                the StatefulDataType UDAF never returns NULL)
 *   MIN_LENGTH / MAX_LENGTH      MinState(value) / MaxState(value) of the string lengths
 *   CORRELATION                  CorrelationState(n, avg = xAvg, y_avg, ck, x_mk, y_mk)
 */
typedef struct dq_state {
  int32_t kind;
  int32_t has_value;
  int64_t num_matches;
  int64_t count;
  double sum;
  double n, avg, m2;
  double value;
  int64_t words[DQ_HLL_NUM_WORDS];
  double y_avg, ck, x_mk, y_mk;  /* CORRELATION (with n, avg) */
} dq_state;

/* ---------------------------------------------------------------- context / plan */
typedef struct dq_ctx dq_ctx;
typedef struct dq_plan dq_plan;

const char* dq_last_error(void);
int dq_abi_version(void);

/* Number of gfx950 devices visible to this process (0 on a host without a GPU). */
dq_status dq_device_count(int* out);

/* Give the device blocks the library keeps cached for reuse (every buffer a plan or frequency
 * table freed -- staging, sort buffers, tables; at most 128 GiB -- kept so that a free is not a
 * device-wide hipFree synchronisation) back to the HIP runtime.  No reference counterpart:
 * Spark's executors free their memory through the JVM. */
dq_status dq_release_cached_memory(int device);

dq_status dq_ctx_create(int device, int flags, dq_ctx** out);
dq_status dq_ctx_destroy(dq_ctx* ctx);

/* Build a plan for `n_ops` analyzers over batches with `n_columns` columns of the given
 * types.  All scan-shareable ops of a plan run in one fused pass per batch
 * (AnalysisRunner.scala:306-313).  Returns DQ_ERR_UNSUPPORTED (and sets *out = NULL) if any
 * op cannot run on the GPU; the caller then routes that op to Spark. */
dq_status dq_plan_create(dq_ctx* ctx, const dq_op* ops, int n_ops,
                         const int32_t* column_types, int n_columns, dq_plan** out);
dq_status dq_plan_destroy(dq_plan* plan);

/* dq_plan_create from the analyzer list serialized as bytes -- what the JVM side builds with a
 * little-endian ByteBuffer (GpuPlanEncoder), so the JNI stub passes one byte[]
 * and the library, not hand-written JNI code, decodes and validates it.  Layout:
 *   u32 magic 0x504F5144 ("DQOP"), u32 version 1, u32 n_ops, then per op
 *   i32 kind, i32 column, i32 column2,
 *   i32 n_pred, i32 pred_strings_len, i32 n_where, i32 where_strings_len,
 *   n_pred x {i32 opcode, i32 arg, i64 i64, f64 f64} (24 B), pred_strings_len bytes,
 *   n_where x {...}, where_strings_len bytes.
 * A truncated or inconsistent blob is DQ_ERR_INVALID (checked before any device work). */
#define DQ_PACKED_MAGIC 0x504F5144u
dq_status dq_plan_create_packed(dq_ctx* ctx, const uint8_t* blob, size_t blob_len, const int32_t* column_types,
                                int n_columns, dq_plan** out);

/* Check whether a single op is GPU-eligible for the given schema without building a plan. */
dq_status dq_op_supported(const dq_op* op, const int32_t* column_types, int n_columns);

/* Enqueue one batch (a row partition).  Asynchronous on the plan's HIP stream; host buffers
 * must stay valid until the next dq_plan_* call on this plan returns.  May be called any
 * number of times; results accumulate in HBM in call order (deterministic). */
dq_status dq_plan_consume(dq_plan* plan, const dq_column* columns, int n_columns,
                          int64_t n_rows);

/* Wait for all consumed batches and write one dq_state per op (in op order). */
dq_status dq_plan_finish(dq_plan* plan, dq_state* out, int n_out);

/* Status of op `op` after dq_plan_finish: DQ_OK, or an error the op alone failed with (the
 * per-analyzer scope of AnalysisRunner.scala:340-353: the JNI layer fails or reroutes that
 * analyzer only).  Every op this library plans evaluates exactly, so it reports DQ_OK today;
 * the entry point keeps the per-op scope in the ABI. */
dq_status dq_plan_op_status(dq_plan* plan, int op);

/* ---------------------------------------------------------------- Arrow C Data Interface
 * The JVM side of the seam hands Spark partitions over as Arrow record batches
 * (ArrowUtils / ArrowWriter -> org.apache.arrow.c.Data.exportVectorSchemaRoot), i.e. the
 * standard C Data Interface structs below (layout fixed by the Arrow specification).  These
 * entry points replace the hand-filled dq_column array of dq_plan_consume / dq_freq_consume at
 * the launch sites AnalysisRunner.scala:313 (data.agg) and GroupingAnalyzers.scala:53-80.
 *
 * Accepted input: a struct array ("+s", one child per plan column, in plan column order -- a
 * record batch) or a single top-level array (a one-column batch).  Child formats: "b" bool,
 * "c" int8, "s" int16, "i" int32, "l" int64, "f" float32, "g" float64, "u" utf8.  Offsets of
 * sliced arrays (struct offset + child offset) are honoured; a NULL validity buffer means no
 * NULLs.  Rejected with DQ_ERR_UNSUPPORTED (route the batch to Spark): dictionary-encoded,
 * nested, large_utf8 ("U"), decimal, temporal formats and struct-level NULL rows.  Malformed
 * structs (released, buffer counts, children shorter than the batch) give DQ_ERR_INVALID.
 * The caller keeps ownership: release callbacks are never invoked by the library, and the
 * buffers must stay valid until the next call on the plan / table returns (host buffers) or
 * until the plan's stream has drained (DQ_COL_DEVICE: buffers in HBM on the context's GPU). */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif /* ARROW_C_DATA_INTERFACE */

/* Map an Arrow batch onto dq_columns without touching any GPU (pure host; the JNI layer can
 * call it to derive the plan's column types): types[i] / columns[i] for each of the batch's
 * columns (at most max_columns), *n_columns and *n_rows.  `flags` = DQ_COL_DEVICE when the
 * buffers are device pointers.  DQ_ERR_SPACE (with *n_columns set) when max_columns is short. */
dq_status dq_arrow_columns(const struct ArrowSchema* schema, const struct ArrowArray* array, int flags,
                           int32_t* types, dq_column* columns, int max_columns, int* n_columns,
                           int64_t* n_rows);
/* dq_plan_consume of one Arrow batch (its columns in plan column order). */
dq_status dq_plan_consume_arrow(dq_plan* plan, const struct ArrowSchema* schema,
                                const struct ArrowArray* array, int flags);

/* Page-lock a host buffer the caller will hand over again and again (e.g. the JNI layer's Arrow
 * allocator pool), so its batches cross PCIe by DMA at full rate instead of through the
 * runtime's pageable staging; unregister before freeing it.  Host batches are double-buffered in
 * HBM either way: dq_plan_consume returns once a batch's bytes are on the device, while its scan
 * still runs, so the caller fills the next batch during the scan. */
dq_status dq_host_register(void* ptr, size_t bytes);
dq_status dq_host_unregister(void* ptr);

/* Clear accumulated results so the plan can scan a new dataset. */
dq_status dq_plan_reset(dq_plan* plan);

/* The HIP stream (hipStream_t) the plan launches on, for external timing/sync. */
void* dq_plan_stream(dq_plan* plan);

/* ---------------------------------------------------------------- state algebra (host) */
/* `Analyzers.merge` (Analyzer.scala:367-386) over Option[State]: out = a + b with None
 * handling; `a` and `b` must have the same kind.  Mirrors each State.sum. */
dq_status dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out);

/* `DoubleValuedState.metricValue()` of a state with has_value = 1. */
dq_status dq_state_metric(const dq_state* s, double* out);

/* DeequHyperLogLogPlusPlusUtils.count (StatefulHyperloglogPlus.scala:210-257). */
double dq_hll_count(const int64_t words[DQ_HLL_NUM_WORDS]);
/* DeequHyperLogLogPlusPlusUtils.merge (StatefulHyperloglogPlus.scala:188-208). */
void dq_hll_merge(const int64_t a[DQ_HLL_NUM_WORDS], const int64_t b[DQ_HLL_NUM_WORDS],
                  int64_t out[DQ_HLL_NUM_WORDS]);
/* wordsToBytes / wordsFromBytes (StatefulHyperloglogPlus.scala:170-186): 416 big-endian bytes. */
void dq_hll_words_to_bytes(const int64_t words[DQ_HLL_NUM_WORDS], uint8_t out[416]);
void dq_hll_words_from_bytes(const uint8_t in[416], int64_t words[DQ_HLL_NUM_WORDS]);

/* Spark 2.2.2 XxHash64Function with seed 42 for one value (host reference, used by tests). */
uint64_t dq_xxh64(const void* data, size_t len, uint64_t seed);

/* Spark 2.2.2 Cast(StringType -> LongType | DoubleType) of one utf8 column, as
 * ColumnProfiler.castNumericStringColumns does before pass 2 (ColumnProfiler.scala:346-355,
 * 427-445).  Writes n_rows values and a validity bitmap (LSB-first, NULL = unparsable) into
 * DEVICE buffers on ctx's GPU.  Doubles are java.lang.Double.parseDouble, correctly rounded
 * for every input (Clinger's fast path, Eisel-Lemire over a 128-bit power-of-five table, an
 * exact big-integer comparison near rounding boundaries; hexadecimal literals rounded half-even).
 * *n_unsupported is always set to 0 (kept for ABI stability: nothing is routed back). */
dq_status dq_cast_utf8(dq_ctx* ctx, const dq_column* src, int64_t n_rows, int32_t to_type,
                       void* d_values, uint8_t* d_validity, int64_t* n_unsupported);

/* dq_cast_utf8 of n columns of n_rows rows each in one call (castNumericStringColumns casts every
 * string column pass 1 typed numeric): column i (utf8) -> to_types[i] into d_values[i] /
 * d_validity[i].  The casts overlap on the device; the call returns when all are done. */
dq_status dq_cast_utf8_batch(dq_ctx* ctx, int32_t n, const dq_column* srcs, int64_t n_rows,
                             const int32_t* to_types, void* const* d_values, uint8_t* const* d_validity);

/* ApproxCountDistinct and DataType of a utf8 column from its groups instead of its rows: the
 * column's distinct non-NULL strings (flat, as dq_freq_export_flat lists them: counts[i], key
 * bytes [key_offsets[i], key_offsets[i + 1])) and its NULL count.  Every group is hashed and
 * classified once and weighted by its count -- the same registers (a maximum does not see
 * duplicates) and the same five DataType counts as the per-row pass (StatefulHyperloglogPlus
 * .update, StatefulDataType.update over every row).  hll_out / dtype_out receive what
 * dq_plan_finish gives ApproxCountDistinct and DataType on that column.  DQ_FLAT_DEVICE: the
 * three buffers are device memory on the context's device. */
dq_status dq_profile_string_groups(dq_ctx* ctx, const int64_t* counts, const int64_t* key_offsets,
                                   const uint8_t* key_bytes, int64_t n_groups, int64_t n_nulls, int flags,
                                   dq_state* hll_out, dq_state* dtype_out);

/* ColumnProfiler pass 1 on n utf8 columns of one batch, each tried as a few-valued column: the
 * few-groups kernel (per-workgroup LDS tables of DQ_FEW_MAX_GROUPS keys of at most 15 bytes) and
 * one merge per column, all columns in one call (their launches overlap; one wait).  Column i
 * fits when it has at most DQ_FEW_MAX_GROUPS distinct non-NULL strings, none longer than 15
 * bytes (and a string heap of at least 16 bytes); then results[i].ok = 1 and:
 *   - results[i].completeness / .hll / .dtype are what dq_plan_finish gives Completeness,
 *     ApproxCountDistinct and DataType on the column (states from the groups weighted by their
 *     counts: the same registers and counts as the per-row pass);
 *   - its groups are group_counts / group_keys (16 bytes each, zero padded) / group_lens
 *     [i * DQ_FEW_MAX_GROUPS, + results[i].n_groups), non-NULL strings only (NULLs are
 *     results[i].n_nulls).
 * A column that does not fit has ok = 0 and nothing else set.  Columns are grouped 32 at a time
 * (bounded scratch); a chunk whose device scratch cannot be allocated leaves its columns at ok = 0
 * (the caller's per-row pass handles them) instead of failing the call. */
#define DQ_FEW_MAX_GROUPS 1024
typedef struct dq_few_result {
  int32_t ok;
  int32_t n_groups;
  int64_t n_nulls;
  dq_state completeness, hll, dtype;
} dq_few_result;
dq_status dq_profile_few_strings(dq_ctx* ctx, int32_t n, const dq_column* cols, int64_t n_rows, dq_few_result* results,
                                 int64_t* group_counts, uint8_t* group_keys, int32_t* group_lens);

/* ---------------------------------------------------------------- frequency group-by
 * Replaces FrequencyBasedAnalyzer.computeFrequencies (GroupingAnalyzers.scala:53-80) and the
 * group-by of Histogram (Histogram.scala:54-69).  A dq_freq is the device-resident state
 * FrequenciesAndNumRows(frequencies, numRows) (GroupingAnalyzers.scala:124-157): consuming a
 * batch groups its rows (rows with a NULL grouping value are dropped, numRows counts every
 * row); importing groups is FrequenciesAndNumRows.sum (outer join adding counts).
 *
 * Group keys are exchanged in an encoded form: fixed-width columns as little-endian value bytes
 * (1 B bool/int8, 2 B int16, 4 B int32/float32, 8 B int64/float64; floats as raw bits), strings
 * as UTF-8 bytes; with several grouping columns the parts are concatenated in column order and
 * every string part is prefixed with its u32 length.  With DQ_FREQ_NULL_AS_KEY (Histogram), a
 * NULL string is the key "NullValue" and a NULL of any other type is the empty key. */
typedef struct dq_freq dq_freq;

#define DQ_FREQ_NULL_AS_KEY 0x1
/* Few groups or nothing: one key column, grouped only by the few-groups kernel (per-workgroup
 * LDS tables of 1024 keys of at most 15 bytes).  A batch it cannot hold -- more distinct keys, a
 * longer key -- fails dq_freq_consume with DQ_ERR_SPACE, and every later consume fails alike: the
 * caller drops the table.  ColumnProfiler uses it to try every string column as a
 * low-cardinality histogram in pass 1 (no reference counterpart: a speculative schedule of the
 * same aggregations). */
#define DQ_FREQ_FEW_ONLY 0x2

typedef struct dq_freq_summary {
  int64_t num_rows;      /* FrequenciesAndNumRows.numRows: every consumed row          */
  int64_t num_groups;    /* number of groups (CountDistinct, Distinctness numerator)   */
  int64_t num_unique;    /* groups with count == 1 (Uniqueness numerator)              */
  int64_t grouped_rows;  /* sum of the group counts                                    */
  double entropy;        /* sum over groups of -(c/num_rows) ln(c/num_rows)            */
} dq_freq_summary;

typedef struct dq_freq_group {
  int64_t count;
  int64_t key_offset;    /* into the caller's key byte buffer                         */
  int32_t key_len;
  int32_t reserved;
} dq_freq_group;

dq_status dq_freq_create(dq_ctx* ctx, const int32_t* key_columns, int n_keys,
                         const int32_t* column_types, int n_columns, int flags, dq_freq** out);
dq_status dq_freq_destroy(dq_freq* f);
/* Optional: size the table's staging for `rows` more rows before consuming them (e.g. the row
 * count of every partition about to be consumed), so staging is not regrown batch by batch. */
dq_status dq_freq_reserve(dq_freq* f, int64_t rows);
/* Optional: the caller expects at most `groups` groups (e.g. ColumnProfiler's approximate
 * distinct count before its histogram pass, ColumnProfiler.scala:535-557).  A handful of groups
 * is aggregated in LDS per workgroup instead of being staged and sorted. */
dq_status dq_freq_expect_groups(dq_freq* f, int64_t groups);
dq_status dq_freq_reset(dq_freq* f);
dq_status dq_freq_consume(dq_freq* f, const dq_column* columns, int n_columns, int64_t n_rows);
/* dq_freq_consume of one Arrow batch (dq_plan_consume_arrow's rules; all the batch's columns). */
dq_status dq_freq_consume_arrow(dq_freq* f, const struct ArrowSchema* schema, const struct ArrowArray* array,
                                int flags);
dq_status dq_freq_get_summary(dq_freq* f, dq_freq_summary* out);
/* Number of groups and total encoded key bytes (to size dq_freq_export's buffers). */
dq_status dq_freq_size(dq_freq* f, int64_t* n_groups, int64_t* key_bytes);
/* Every group, in an unspecified order. */
dq_status dq_freq_export(dq_freq* f, dq_freq_group* groups, int64_t max_groups, uint8_t* key_bytes,
                         int64_t key_cap, int64_t* n_out);
/* The most frequent groups for Histogram's top-maxDetailBins (Histogram.scala:79): every group
 * whose count is at least the n-th largest count -- all ties at the cut included, so the caller
 * can apply its own tie order (Spark's rdd.top breaks ties arbitrarily) -- sorted by count
 * descending, then encoded key ascending.  *n_out / *key_bytes_out receive the sizes; when they
 * exceed max_groups / key_cap nothing is written and DQ_ERR_SPACE is returned. */
dq_status dq_freq_top(dq_freq* f, int n, dq_freq_group* groups, int64_t max_groups, uint8_t* key_bytes,
                      int64_t key_cap, int64_t* n_out, int64_t* key_bytes_out);
/* dst += src on the device (FrequenciesAndNumRows.sum, GroupingAnalyzers.scala:128-148): both
 * tables on one device, grouping the same key types; src is unchanged. */
dq_status dq_freq_merge(dq_freq* dst, dq_freq* src);
/* Merge groups (and `num_rows`) into the table: FrequenciesAndNumRows.sum. */
/* Count of one group (0 if the key is absent), key in the encoded form above.  Used to fold a
 * literal "NullValue" string into Histogram's NULL bin when Histogram shares the frequency
 * table of its column (Histogram.scala:63-64: NULL is replaced by that literal before grouping). */
dq_status dq_freq_lookup(dq_freq* f, const uint8_t* key, int64_t key_len, int64_t* count);
dq_status dq_freq_import(dq_freq* f, const dq_freq_group* groups, int64_t n, const uint8_t* key_bytes,
                         int64_t num_rows);

/* ---- Columnar (Arrow-layout) state interchange: FrequenciesAndNumRows.frequencies as the
 * DataFrame columns HdfsStateProvider persists (StateProvider.scala:222-240) and loads
 * (:280-311), with no per-group record anywhere.  Group i = (counts[i], the encoded key
 * key_bytes[key_offsets[i] .. key_offsets[i + 1])); key_offsets holds n + 1 values (Arrow's
 * large-offset layout).  DQ_FLAT_DEVICE: the three buffers are device memory on the table's
 * device, else host memory. */
#define DQ_FLAT_DEVICE 0x1
/* Every group in slot order (the same table exports the same columns).  *n_out / *key_bytes_out
 * receive the sizes; when they exceed max_groups / key_cap (or a buffer is NULL) nothing is
 * written and DQ_ERR_SPACE is returned -- the export stays on the device for the filling call,
 * which hands it over. */
dq_status dq_freq_export_flat(dq_freq* f, int64_t* counts, int64_t* key_offsets, uint8_t* key_bytes,
                              int64_t max_groups, int64_t key_cap, int flags, int64_t* n_out, int64_t* key_bytes_out);
/* FrequenciesAndNumRows.sum of n flat groups (+ num_rows): duplicate keys add up, as the
 * reference's outer join does (GroupingAnalyzers.scala:128-148).  Offsets are validated first. */
dq_status dq_freq_import_flat(dq_freq* f, const int64_t* counts, const int64_t* key_offsets, const uint8_t* key_bytes,
                              int64_t n, int64_t num_rows, int flags);

/* ---------------------------------------------------------------- multi-GPU key-hash exchange
 * The frequency family's one real exchange step: Spark shuffles the partial
 * group counts by key hash into spark.sql.shuffle.partitions before the final aggregate
 * (GroupingAnalyzers.scala:67-72).  Here every rank partitions its local table by owner rank
 * (a hash of the encoded key), the ranks exchange the partitions with one all-to-all (RCCL over
 * xGMI), and every owner merges what it receives with dq_freq_import_parts -- after which the
 * owners hold disjoint keys, and their count-of-counts histograms add up to the global one. */
typedef struct dq_freq_wire {  /* one group in device memory (32 B)                         */
  uint64_t ctrl;               /* key length (low 24 bits) | 1 << 30 if the key is in key bytes */
  int64_t count;
  uint64_t k0, k1;             /* key bytes (<= 16 B, little-endian), or k0 = key-byte offset  */
} dq_freq_wire;

typedef struct dq_freq_wire_packed {  /* a group whose key packs into one word (16 B):        */
  uint64_t key;                       /* a decimal digit string of <= 15 bytes -- nibble i =   */
  int64_t count;                      /* digit i, the length in the top nibble -- or 0xA for   */
} dq_freq_wire_packed;                /* Histogram's "NullValue" group                         */

/* Write every group of `f`, partitioned by owner (0 .. n_parts-1), into DEVICE buffers on f's
 * GPU.  Part p follows parts 0..p-1 in d_out and is part_packed[p] dq_freq_wire_packed records
 * (16 B: keys that pack) then part_groups[p] dq_freq_wire records (32 B: every other key), each
 * section in the order of f's table slices -- so the receiver merges a part slice by slice with
 * no sort.  Long keys (8-byte padded) of part p follow those of parts 0..p-1 in d_key_bytes, k0
 * relative to the start of part p's key region.  The sizes go to the three host arrays (n_parts
 * each); if a buffer is too small nothing is written and DQ_ERR_SPACE is returned (call once with
 * out_bytes = 0 to size them: part p takes 16 part_packed[p] + 32 part_groups[p] bytes).
 * Replaces the map side of the groupBy's hash exchange (GroupingAnalyzers.scala:67-72). */
dq_status dq_freq_partition(dq_freq* f, int n_parts, void* d_out, int64_t out_bytes, uint8_t* d_key_bytes,
                            int64_t key_cap, int64_t* part_packed, int64_t* part_groups,
                            int64_t* part_key_bytes);
/* Merge the parts other ranks partitioned for this one (laid out as dq_freq_partition writes
 * them, one after the other in d_parts / d_key_bytes) into f: each of f's slices is merged once,
 * in LDS, from the matching records of every part (FrequenciesAndNumRows.sum's outer join,
 * GroupingAnalyzers.scala:128-148); num_rows is added to numRows. */
dq_status dq_freq_import_parts(dq_freq* f, int n_parts, const void* d_parts, const int64_t* part_packed,
                               const int64_t* part_groups, const uint8_t* d_key_bytes,
                               const int64_t* part_key_bytes, int64_t num_rows);
/* Merge n general groups held in DEVICE memory (dq_freq_wire, any order) into f. */
dq_status dq_freq_import_wire(dq_freq* f, const dq_freq_wire* d_groups, int64_t n,
                              const uint8_t* d_key_bytes, int64_t key_bytes, int64_t num_rows);
/* Count-of-counts of f: hist[c] = number of groups with count c (1 <= c < n_bins, hist[0] = 0);
 * counts >= n_bins go to big[] ascending (*n_big; DQ_ERR_SPACE if big_cap is too small). */
dq_status dq_freq_count_histogram(dq_freq* f, int64_t* hist, int64_t n_bins, int64_t* big,
                                  int64_t big_cap, int64_t* n_big);
/* The dq_freq_summary of a (summed) count-of-counts histogram and numRows, with the same fixed
 * summation order as dq_freq_get_summary. */
dq_status dq_freq_summary_from_histogram(const int64_t* hist, int64_t n_bins, const int64_t* big,
                                         int64_t n_big, int64_t num_rows, dq_freq_summary* out);

/* ---------------------------------------------------------------- multi-GPU groups (RCCL)
 * One process (or one JVM executor thread) per GPU, each with its own dq_ctx, joined into a
 * dq_group -- an RCCL communicator over xGMI -- so that a driver that is not torch (the JNI shim)
 * can run the sharded path.  Each rank scans its own row shard; the group then
 * replaces Spark's final aggregation (AnalysisRunner.scala:313: partial states of every partition
 * merged by the aggregate) and the shuffle of the frequency family (GroupingAnalyzers.scala:
 * 67-72).  Every dq_group_* call is collective: all ranks call it in the same order. */
typedef struct dq_group dq_group;

#define DQ_GROUP_ID_BYTES 128

/* A fresh group id on the rank that creates the group (ncclGetUniqueId); the caller ships the
 * bytes to every other rank (e.g. through the Spark driver) before dq_group_create. */
dq_status dq_group_unique_id(uint8_t id[DQ_GROUP_ID_BYTES]);
dq_status dq_group_create(dq_ctx* ctx, int n_ranks, int rank, const uint8_t id[DQ_GROUP_ID_BYTES],
                          dq_group** out);
dq_status dq_group_destroy(dq_group* g);

/* In place: states[0..n_ops) of this rank's shard become those of the whole dataset -- ONE
 * all-gather of the POD states over RCCL, then the fold in rank order of dq_states_merge_ranks
 * (deterministic: every rank computes the same bytes). */
dq_status dq_group_allgather_merge(dq_group* g, dq_state* states, int n_ops);

/* The fold dq_group_allgather_merge applies (host only): gathered = n_ranks blocks of n_ops
 * states in rank order; out[i] = Analyzers.merge of gathered[r * n_ops + i] over r = 0, 1, ...
 * (State.sum per kind, Analyzer.scala:367-386; e.g. StandardDeviation.scala:37-44). */
dq_status dq_states_merge_ranks(const dq_state* gathered, int n_ranks, int n_ops, dq_state* out);

/* Every dq_group_* call is collective; a failure of any rank's local step fails the call on
 * every rank (agreed on before data moves), so no rank is left blocked in a collective.
 *
 * The key-hash exchange: every rank partitions `local` by owner (dq_freq_partition), the parts
 * travel in one RCCL all-to-all (grouped send/recv), and each rank merges what it receives into
 * `owned` (an empty table with the same key columns) -- which then holds the keys this rank owns,
 * disjoint across ranks.  *num_rows = the dataset's numRows (sum over ranks). */
dq_status dq_group_freq_exchange(dq_group* g, dq_freq* local, dq_freq* owned, int64_t* num_rows);

/* dq_freq_summary of the whole dataset from the owned tables: the count-of-counts histograms
 * all-reduced (sum) over RCCL, counts beyond the histogram all-gathered, then the fixed-order
 * dq_freq_summary_from_histogram -- equal, bit for bit, to a single table over all rows. */
dq_status dq_group_freq_summary(dq_group* g, dq_freq* owned, int64_t num_rows, dq_freq_summary* out);

/* Histogram's top-maxDetailBins over the whole dataset (Histogram.scala:78-79, rdd.top + the
 * groupBy's exchange): the union of every owner's dq_freq_top(owned, n), cut at the n-th largest
 * count with all ties kept, count descending then encoded key ascending -- dq_freq_top's contract
 * over the union of the ranks' rows.  Same buffer protocol as dq_freq_top: on DQ_ERR_SPACE
 * *n_out / *key_bytes_out hold the sizes and every rank retries with larger buffers. */
dq_status dq_group_freq_top(dq_group* g, dq_freq* owned, int n, dq_freq_group* groups, int64_t max_groups,
                            uint8_t* key_bytes, int64_t key_cap, int64_t* n_out, int64_t* key_bytes_out);

#ifdef __cplusplus
}
#endif
#endif /* DEEQU_AMD_H */
