// dq_pred.hip -- generic predicate evaluation into row masks.
//
// Spark parses every Compliance predicate and `where` filter with `expr(String)`
// (Compliance.scala:49, Analyzer.scala:413-432) and evaluates it per row with SQL
// three-valued logic.  The fused scan kernel evaluates the common single-comparison forms
// inline; every other predicate of a plan is run here first, once per batch, by a small
// postfix interpreter (the plan's validated dq_pred_insn program).  Each wave evaluates 64
// consecutive rows and writes two 64-bit ballot words: TRUE bits and NOT-NULL bits.  The scan
// kernel then reads those masks (2 bits per row instead of the referenced columns' bytes).
#include "dq_parse.h"

namespace dq {

namespace {

enum ValType : uint8_t { VT_INT = 0, VT_FLT = 1, VT_BOOL = 2, VT_STR = 3 };

struct Val {
  int64_t i;      // int / bool value; string length for VT_STR
  double f;
  uint8_t type;
  uint8_t null;
  const uint8_t* s;  // VT_STR bytes
};

// UTF8String.compareTo: unsigned byte-wise, then shorter first.
__device__ inline int ord_str(const Val& a, const Val& b) {
  const int64_t n = a.i < b.i ? a.i : b.i;
  for (int64_t k = 0; k < n; ++k) {
    const int d = (int)a.s[k] - (int)b.s[k];
    if (d) return d < 0 ? -1 : 1;
  }
  return (int)(a.i > b.i) - (int)(a.i < b.i);
}

__device__ inline bool col_valid(const DevColumn& c, int64_t row) {
  return c.validity == nullptr || ((c.validity[row >> 3] >> (row & 7)) & 1u);
}

__device__ inline Val load_col(const DevColumn& c, int64_t row) {
  Val v;
  v.null = col_valid(c, row) ? 0 : 1;
  v.i = 0;
  v.f = 0.0;
  v.type = VT_INT;
  v.s = nullptr;
  switch (c.type) {
    case DQ_T_UTF8: {
      const int32_t b = c.offsets[row], e = c.offsets[row + 1];
      v.s = static_cast<const uint8_t*>(c.values) + b;
      v.i = e - b;
      v.type = VT_STR;
      break;
    }
    case DQ_T_BOOL: {
      const uint8_t* b = static_cast<const uint8_t*>(c.values);
      v.i = (b[row >> 3] >> (row & 7)) & 1u;
      v.type = VT_BOOL;
      break;
    }
    case DQ_T_INT8: v.i = static_cast<const int8_t*>(c.values)[row]; break;
    case DQ_T_INT16: v.i = static_cast<const int16_t*>(c.values)[row]; break;
    case DQ_T_INT32: v.i = static_cast<const int32_t*>(c.values)[row]; break;
    case DQ_T_INT64: v.i = static_cast<const int64_t*>(c.values)[row]; break;
    case DQ_T_FLOAT32: v.f = static_cast<const float*>(c.values)[row]; v.type = VT_FLT; break;
    case DQ_T_FLOAT64: v.f = static_cast<const double*>(c.values)[row]; v.type = VT_FLT; break;
    default: v.null = 1; break;
  }
  return v;
}

__device__ inline double as_f64(const Val& v) { return v.type == VT_FLT ? v.f : (double)v.i; }

__device__ inline int ord_f64(double a, double b) {
  const bool an = a != a, bn = b != b;
  if (an | bn) return (int)an - (int)bn;
  return (int)(a > b) - (int)(a < b);
}

__device__ inline bool cmp_result(int opcode, int ord) {
  switch (opcode) {
    case DQ_P_EQ: return ord == 0;
    case DQ_P_NE: return ord != 0;
    case DQ_P_LT: return ord < 0;
    case DQ_P_LE: return ord <= 0;
    case DQ_P_GT: return ord > 0;
    case DQ_P_GE: return ord >= 0;
    default: return ord == 0;
  }
}

// CAST: the program may cast a string to double (Double.parseDouble, whose exact slow path
// carries ~1 KB of private scratch per lane); programs without one run a kernel without it.
template <bool CAST>
__device__ void eval_program(const PredInsn* code, int n, const uint8_t* pool, const DevColumn* cols, int64_t row,
                             bool& t, bool& nn) {
  Val st[kMaxStack];
  int sp = 0;
  for (int pc = 0; pc < n; ++pc) {
    const PredInsn ins = code[pc];
    switch (ins.opcode) {
      case DQ_P_COLUMN: st[sp++] = load_col(cols[ins.arg], row); break;
      case DQ_P_LIT_INT: st[sp++] = Val{ins.i64, 0.0, VT_INT, 0}; break;
      case DQ_P_LIT_FLOAT: st[sp++] = Val{0, ins.f64, VT_FLT, 0}; break;
      case DQ_P_LIT_NULL: st[sp++] = Val{0, 0.0, VT_INT, 1}; break;
      case DQ_P_LIT_STRING: st[sp++] = Val{(int64_t)ins.arg, 0.0, VT_STR, 0, pool + ins.i64}; break;
      case DQ_P_CAST_DOUBLE: {  // Spark 2.2 Cast(-> DoubleType): parseDouble of a string
        Val& a = st[sp - 1];
        if (CAST && a.type == VT_STR) {
          double v = 0.0;
          int r = 0;
          if constexpr (CAST) r = a.null ? 0 : parse_double(PtrSrc{a.s}, (int32_t)a.i, &v);
          a.null = (r == 1) ? a.null : 1;
          a.f = v;
        } else {
          a.f = as_f64(a);
        }
        a.type = VT_FLT;
        break;
      }
      case DQ_P_TRUE: st[sp++] = Val{1, 0.0, VT_BOOL, 0}; break;
      case DQ_P_FALSE: st[sp++] = Val{0, 0.0, VT_BOOL, 0}; break;
      case DQ_P_COALESCE: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r = a.null ? b : a;
        if ((a.type == VT_FLT) != (b.type == VT_FLT)) {  // common type is fp64
          r.f = as_f64(r);
          r.type = VT_FLT;
        }
        st[sp - 1] = r;
        break;
      }
      case DQ_P_EQ: case DQ_P_NE: case DQ_P_LT: case DQ_P_LE: case DQ_P_GT: case DQ_P_GE:
      case DQ_P_EQ_NULLSAFE: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r{0, 0.0, VT_BOOL, 0};
        if (a.null || b.null) {
          if (ins.opcode == DQ_P_EQ_NULLSAFE) r.i = (a.null && b.null) ? 1 : 0;
          else r.null = 1;
        } else {
          int ord;
          if (a.type == VT_STR) ord = ord_str(a, b);
          else if (ins.arg == DQ_CMP_AS_FLOAT64) ord = ord_f64(as_f64(a), as_f64(b));
          else ord = (int)(a.i > b.i) - (int)(a.i < b.i);
          r.i = cmp_result(ins.opcode, ord) ? 1 : 0;
        }
        st[sp - 1] = r;
        break;
      }
      case DQ_P_IS_NULL: st[sp - 1] = Val{st[sp - 1].null ? 1 : 0, 0.0, VT_BOOL, 0}; break;
      case DQ_P_IS_NOT_NULL: st[sp - 1] = Val{st[sp - 1].null ? 0 : 1, 0.0, VT_BOOL, 0}; break;
      case DQ_P_NOT: {
        Val a = st[sp - 1];
        if (!a.null) a.i = a.i ? 0 : 1;
        st[sp - 1] = a;
        break;
      }
      case DQ_P_AND: case DQ_P_OR: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r{0, 0.0, VT_BOOL, 0};
        const bool at = !a.null && a.i, af = !a.null && !a.i;
        const bool bt = !b.null && b.i, bf = !b.null && !b.i;
        if (ins.opcode == DQ_P_AND) {
          if (af || bf) r.i = 0;
          else if (a.null || b.null) r.null = 1;
          else r.i = 1;
        } else {
          if (at || bt) r.i = 1;
          else if (a.null || b.null) r.null = 1;
          else r.i = 0;
        }
        st[sp - 1] = r;
        break;
      }
      default: break;
    }
  }
  const Val top = st[sp - 1];
  nn = !top.null;
  t = nn && top.i != 0;
}

}  // namespace

template <bool CAST>
__global__ __launch_bounds__(kBlock) void dq_pred_kernel(const PredProgram* __restrict__ progs,
                                                         const PredInsn* __restrict__ insns,
                                                         const uint8_t* __restrict__ pool,
                                                         const DevColumn* __restrict__ cols,
                                                         int64_t n_rows, uint64_t* out,
                                                         int64_t words_per_mask) {
  const PredProgram prog = progs[blockIdx.y];
  const PredInsn* code = insns + prog.first;
  const int lane = threadIdx.x & 63;
  const int64_t n_words = (n_rows + 63) >> 6;
  uint64_t* out_t = out + (int64_t)(2 * blockIdx.y) * words_per_mask;
  uint64_t* out_n = out_t + words_per_mask;
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < n_words;
       w += (int64_t)gridDim.x * (kBlock / 64)) {
    const int64_t row = (w << 6) + lane;
    bool t = false, nn = false;
    if (row < n_rows) eval_program<CAST>(code, prog.n, pool, cols, row, t, nn);
    const uint64_t bt = __ballot(t);
    const uint64_t bn = __ballot(nn);
    if (lane == 0) {
      out_t[w] = bt;
      out_n[w] = bn;
    }
  }
}

// dst bit i = src bit (bit_offset + i): realigns a sliced Arrow bitmap so that bit 0 of
// byte 0 is row 0 of the batch.
__global__ void dq_realign_kernel(const uint8_t* __restrict__ src, int64_t bit_offset,
                                  int64_t n_bits, uint8_t* __restrict__ dst) {
  const int64_t n_bytes = (n_bits + 7) >> 3;
  const int64_t src_bytes = (bit_offset + n_bits + 7) >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_bytes;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bit = bit_offset + (i << 3);
    const int64_t b = bit >> 3;
    const uint32_t sh = (uint32_t)(bit & 7);
    uint32_t v = src[b] >> sh;
    if (sh && b + 1 < src_bytes) v |= (uint32_t)src[b + 1] << (8 - sh);
    dst[i] = (uint8_t)v;
  }
}

hipError_t launch_predicates(const PredProgram* d_progs, int n_progs, const PredInsn* d_insns,
                             const uint8_t* d_pool, const DevColumn* d_cols, int64_t n_rows,
                             uint64_t* d_mask_words, int64_t words_per_mask, bool with_cast, hipStream_t stream) {
  if (n_progs <= 0 || n_rows <= 0) return hipSuccess;
  const int64_t n_words = (n_rows + 63) >> 6;
  int64_t blocks = (n_words + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  if (with_cast)
    hipLaunchKernelGGL(dq_pred_kernel<true>, dim3((unsigned)blocks, n_progs), dim3(kBlock), 0, stream,
                       d_progs, d_insns, d_pool, d_cols, n_rows, d_mask_words, words_per_mask);
  else
    hipLaunchKernelGGL(dq_pred_kernel<false>, dim3((unsigned)blocks, n_progs), dim3(kBlock), 0, stream,
                       d_progs, d_insns, d_pool, d_cols, n_rows, d_mask_words, words_per_mask);
  return hipGetLastError();
}

// offs[i] -= first: utf8 offsets of a host batch copied verbatim, rebased to its first byte
__global__ void dq_rebase_offsets_kernel(int32_t* __restrict__ offs, int64_t n, int32_t first) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    offs[i] -= first;
}

hipError_t launch_rebase_offsets(int32_t* d_offs, int64_t n, int32_t first, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 1023) / 1024;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_rebase_offsets_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_offs, n, first);
  return hipGetLastError();
}

hipError_t launch_realign_bitmap(const uint8_t* src, int64_t bit_offset, int64_t n_bits,
                                 uint8_t* dst, hipStream_t stream) {
  const int64_t n_bytes = (n_bits + 7) >> 3;
  if (n_bytes <= 0) return hipSuccess;
  int64_t blocks = (n_bytes + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(dq_realign_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src,
                     bit_offset, n_bits, dst);
  return hipGetLastError();
}

}  // namespace dq
