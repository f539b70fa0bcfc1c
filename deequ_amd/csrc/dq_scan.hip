// dq_scan.hip -- fused single-pass multi-column reduction for the scan-shareable analyzers.
//
// Replaces the one Spark job that AnalysisRunner.runScanningAnalyzers launches over every
// scan-shareable aggregation (runners/AnalysisRunner.scala:306-313): Size, Completeness,
// Compliance, Sum, Mean, StandardDeviation, Minimum, Maximum.
//
// HBM-bound by design (no MFMA: nothing here is a contraction).  Each lane streams 16 B of
// values per load (2 int64/fp64 rows, 4 int32/fp32 rows, ...), the matching validity bits,
// and keeps every statistic in registers; a field-wise wave-shuffle + LDS combine writes one
// partial per (task, block), and a second tiny launch merges the partials in a FIXED order,
// so the result is bitwise reproducible run to run.
//
// Kernels are specialised per (value type, number of inline predicates) so each keeps its own
// register budget; blockIdx.y indexes the tasks of one specialisation group, blockIdx.x a
// contiguous kScanRowAlign-aligned row chunk.
//
// Semantics per task (see dq_api.cpp for the state mapping):
//   n_rows / n_wnn : Σ where-TRUE / Σ where-NOT-NULL   (Analyzers.conditionalCount, :428-432)
//   n_sel          : Σ valid ∧ where-TRUE              (Completeness numerator, Mean count, n)
//   isum           : wrapping int64 sum (Spark Sum over integral types is LongType)
//   fs + fc        : Neumaier-compensated fp64 sum     (Spark: sequential fp64 sum)
//   imin/imax, fmin/fmax/nnan : Spark NaN-safe min/max (NaN is the largest double)
//   mean, m2       : moments about the mean, from per-lane shifted sums then Chan merges
//                    with the exact formula of StandardDeviationState.sum
//                    (StandardDeviation.scala:37-44); no per-element fp64 divide
//   pm / pn        : per predicate Σ TRUE / Σ NOT NULL among where-TRUE rows
//                    (Compliance: sum(cast(when(where, pred) as int)), Compliance.scala:49)
#include "dq_internal.h"

namespace dq {

namespace {

template <typename T> struct IsIntegral { static constexpr bool value = true; };
template <> struct IsIntegral<float> { static constexpr bool value = false; };
template <> struct IsIntegral<double> { static constexpr bool value = false; };

struct alignas(16) Vec16 {
  uint32_t w[4];
};

template <int NP>
struct ThreadAcc {
  uint32_t n_rows, n_wnn, n_sel, nnan;
  int64_t isum, imin, imax;
  double fs, fc, fmin, fmax;
  double shift, s1, s2;
  uint32_t pm[NP > 0 ? NP : 1], pn[NP > 0 ? NP : 1];
};

template <int NP>
__device__ inline void thread_acc_init(ThreadAcc<NP>& a) {
  a.n_rows = a.n_wnn = a.n_sel = a.nnan = 0;
  a.isum = 0;
  a.imin = INT64_MAX;
  a.imax = INT64_MIN;
  a.fs = a.fc = 0.0;
  a.fmin = __builtin_huge_val();
  a.fmax = -__builtin_huge_val();
  a.shift = a.s1 = a.s2 = 0.0;
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) a.pm[p] = a.pn[p] = 0;
}

// Spark's NaN-safe three-way comparison (Utils.nanSafeCompareDoubles): NaN == NaN and NaN is
// larger than every other double; -0.0 == 0.0.
__device__ inline int ord_f64(double a, double b) {
  const bool an = a != a, bn = b != b;
  if (an | bn) return (int)an - (int)bn;
  return (int)(a > b) - (int)(a < b);
}
__device__ inline int ord_i64(int64_t a, int64_t b) { return (int)(a > b) - (int)(a < b); }

__device__ inline bool apply_cmp(int op, int ord) {
  switch (op) {
    case CMP_EQ: return ord == 0;
    case CMP_NE: return ord != 0;
    case CMP_LT: return ord < 0;
    case CMP_LE: return ord <= 0;
    case CMP_GT: return ord > 0;
    case CMP_GE: return ord >= 0;
    default: return ord == 0;
  }
}

// Neumaier step: s + x with the rounding error carried in c.
__device__ inline void neumaier_add(double& s, double& c, double x) {
  const double t = s + x;
  c += (fabs(s) >= fabs(x)) ? ((s - t) + x) : ((x - t) + s);
  s = t;
}

// One element of the primary column.
template <typename T, int NP>
__device__ inline void accumulate_element(ThreadAcc<NP>& a, T v, uint32_t sel) {
  const bool first = sel && (a.n_sel == 0);
  a.n_sel += sel;
  double xd;
  if constexpr (IsIntegral<T>::value) {
    const int64_t xi = (int64_t)v;
    a.isum += sel ? xi : 0;
    a.imin = (sel && xi < a.imin) ? xi : a.imin;
    a.imax = (sel && xi > a.imax) ? xi : a.imax;
    xd = (double)xi;
  } else {
    xd = (double)v;
    const bool isnan = xd != xd;
    neumaier_add(a.fs, a.fc, sel ? xd : 0.0);
    a.nnan += (sel && isnan) ? 1u : 0u;
    a.fmin = (sel && !isnan && xd < a.fmin) ? xd : a.fmin;
    a.fmax = (sel && !isnan && xd > a.fmax) ? xd : a.fmax;
  }
  a.shift = first ? xd : a.shift;
  const double d = sel ? (xd - a.shift) : 0.0;
  a.s1 += d;
  a.s2 = fma(d, d, a.s2);
}

// Inline predicate over one element -> (TRUE, NOT NULL) bits.
template <typename T>
__device__ inline void eval_fast_pred(const FastPred& fp, T v, uint32_t valid, uint32_t mt,
                                      uint32_t mnn, uint32_t& r, uint32_t& nn) {
  switch (fp.kind) {
    case FP_CMP:
    case FP_COALESCE_CMP: {
      const bool use_coal = (fp.kind == FP_COALESCE_CMP) && !valid;
      int ord;
      if (fp.as_f64) {
        const double x = use_coal ? fp.coal_f : (double)v;
        ord = ord_f64(x, fp.lit_f);
      } else {
        const int64_t x = use_coal ? fp.coal_i : (int64_t)v;
        ord = ord_i64(x, fp.lit_i);
      }
      nn = (fp.kind == FP_COALESCE_CMP) ? 1u : valid;
      r = apply_cmp(fp.op, ord) ? 1u : 0u;
      break;
    }
    case FP_IS_NULL: r = valid ^ 1u; nn = 1u; break;
    case FP_IS_NOT_NULL: r = valid; nn = 1u; break;
    case FP_CONST: r = fp.lit_i == 1 ? 1u : 0u; nn = fp.lit_i == -1 ? 0u : 1u; break;
    case FP_MASK: r = mt; nn = mnn; break;
    default: r = 0u; nn = 0u; break;
  }
}

template <int RPL>
__device__ inline uint32_t load_bits(const uint8_t* bm, int64_t row0, int64_t left) {
  // row0 % RPL == 0 and bit 0 of bm[0] is row 0, so the RPL bits never straddle a byte for
  // RPL <= 8; RPL == 16 reads an aligned u16 (one byte at the very end, so no byte past
  // ceil(n_rows / 8) is ever touched).
  if constexpr (RPL == 16) {
    if (left > 8) return (uint32_t)(*reinterpret_cast<const uint16_t*>(bm + (row0 >> 3)));
    return (uint32_t)bm[row0 >> 3];
  } else {
    const uint32_t byte = bm[row0 >> 3];
    return (byte >> (uint32_t)(row0 & 7)) & ((1u << RPL) - 1u);
  }
}

// ----------------------------------------------------------------------------- merges
__device__ inline void moments_merge(double& na, double& ma, double& m2a, double nb, double mb,
                                     double m2b) {
  // StandardDeviationState.sum (StandardDeviation.scala:37-44); empty sides are identities
  if (nb == 0.0) return;
  if (na == 0.0) {
    na = nb;
    ma = mb;
    m2a = m2b;
    return;
  }
  const double new_n = na + nb;
  const double delta = mb - ma;
  const double delta_n = delta / new_n;
  ma = ma + delta_n * nb;
  m2a = m2a + m2b + delta * delta_n * na * nb;
  na = new_n;
}

__device__ inline void two_sum_merge(double& s, double& c, double s2, double c2) {
  const double t = s + s2;
  const double bb = t - s;
  const double err = (s - (t - bb)) + (s2 - bb);
  c = c + c2 + err;
  s = t;
}

__device__ inline void acc_init(ScanAcc& a) {
  a.n_rows = a.n_wnn = a.n_sel = 0;
  a.isum = 0;
  a.imin = INT64_MAX;
  a.imax = INT64_MIN;
  a.fs = a.fc = 0.0;
  a.fmin = __builtin_huge_val();
  a.fmax = -__builtin_huge_val();
  a.nnan = 0;
  a.mean = a.m2 = 0.0;
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) a.pm[p] = a.pn[p] = 0;
}

// a <- a + b (b is the later partial); fixed operand order keeps results reproducible.
__device__ inline void acc_merge(ScanAcc& a, const ScanAcc& b) {
  double na = (double)a.n_sel;
  moments_merge(na, a.mean, a.m2, (double)b.n_sel, b.mean, b.m2);
  a.n_rows += b.n_rows;
  a.n_wnn += b.n_wnn;
  a.n_sel += b.n_sel;
  a.isum = (int64_t)((uint64_t)a.isum + (uint64_t)b.isum);
  a.imin = b.imin < a.imin ? b.imin : a.imin;
  a.imax = b.imax > a.imax ? b.imax : a.imax;
  two_sum_merge(a.fs, a.fc, b.fs, b.fc);
  a.fmin = b.fmin < a.fmin ? b.fmin : a.fmin;
  a.fmax = b.fmax > a.fmax ? b.fmax : a.fmax;
  a.nnan += b.nnan;
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) {
    a.pm[p] += b.pm[p];
    a.pn[p] += b.pn[p];
  }
}

// ---- wave-level reductions (fixed shfl_down tree; result in lane 0)
__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_down((unsigned long long)v, d, 64);
  return v;
}
__device__ inline int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int64_t o = (int64_t)__shfl_down((long long)v, d, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int64_t o = (int64_t)__shfl_down((long long)v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ inline double wave_min_f64(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const double o = __shfl_down(v, d, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline double wave_max_f64(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const double o = __shfl_down(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ inline void wave_two_sum(double& s, double& c) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const double os = __shfl_down(s, d, 64);
    const double oc = __shfl_down(c, d, 64);
    if ((threadIdx.x & 63) < d) two_sum_merge(s, c, os, oc);
  }
}
__device__ inline void wave_moments(double& n, double& m, double& m2) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const double on = __shfl_down(n, d, 64);
    const double om = __shfl_down(m, d, 64);
    const double om2 = __shfl_down(m2, d, 64);
    if ((threadIdx.x & 63) < d) moments_merge(n, m, m2, on, om, om2);
  }
}

// Reduce one ScanAcc-shaped set of per-thread values to the block's partial, field by field
// (short live ranges), wave results staged in LDS, waves combined in order by thread 0.
template <int NPRED>
__device__ void block_reduce_store(uint64_t n_rows, uint64_t n_wnn, uint64_t n_sel, uint64_t nnan,
                                   int64_t isum, int64_t imin, int64_t imax, double fs, double fc,
                                   double fmin, double fmax, double mean, double m2,
                                   const uint64_t* pm, const uint64_t* pn, int n_preds,
                                   ScanAcc* out) {
  __shared__ ScanAcc part[kBlock / 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  ScanAcc& P = part[wave];
  uint64_t r;
  r = wave_sum_u64(n_rows); if (lane == 0) P.n_rows = (int64_t)r;
  r = wave_sum_u64(n_wnn); if (lane == 0) P.n_wnn = (int64_t)r;
  double dn = (double)n_sel;
  r = wave_sum_u64(n_sel); if (lane == 0) P.n_sel = (int64_t)r;
  r = wave_sum_u64(nnan); if (lane == 0) P.nnan = (int64_t)r;
  r = wave_sum_u64((uint64_t)isum); if (lane == 0) P.isum = (int64_t)r;
  int64_t i = wave_min_i64(imin); if (lane == 0) P.imin = i;
  i = wave_max_i64(imax); if (lane == 0) P.imax = i;
  double f = wave_min_f64(fmin); if (lane == 0) P.fmin = f;
  f = wave_max_f64(fmax); if (lane == 0) P.fmax = f;
  wave_two_sum(fs, fc);
  if (lane == 0) { P.fs = fs; P.fc = fc; }
  wave_moments(dn, mean, m2);
  if (lane == 0) { P.mean = mean; P.m2 = m2; }
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) {
    if (p < NPRED && p < n_preds) {
      r = wave_sum_u64(pm[p]); if (lane == 0) P.pm[p] = (int64_t)r;
      r = wave_sum_u64(pn[p]); if (lane == 0) P.pn[p] = (int64_t)r;
    } else if (lane == 0) {
      P.pm[p] = 0;
      P.pn[p] = 0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll 1
    for (int w = 1; w < kBlock / 64; ++w) acc_merge(part[0], part[w]);
    *out = part[0];
  }
}

template <int NP>
__device__ inline void thread_finish(const ThreadAcc<NP>& t, int n_preds, ScanAcc* out) {
  double mean = 0.0, m2 = 0.0;
  if (t.n_sel > 0) {
    const double n = (double)t.n_sel;
    mean = t.shift + t.s1 / n;
    m2 = t.s2 - t.s1 * t.s1 / n;
    m2 = (m2 < 0.0) ? 0.0 : m2;  // rounding; NaN/Inf propagate
  }
  uint64_t pm[NP > 0 ? NP : 1], pn[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) {
    pm[p] = t.pm[p];
    pn[p] = t.pn[p];
  }
  block_reduce_store<NP>(t.n_rows, t.n_wnn, t.n_sel, t.nnan, t.isum, t.imin, t.imax, t.fs, t.fc,
                         t.fmin, t.fmax, mean, m2, pm, pn, n_preds, out);
}

__device__ inline void chunk_of_block(int64_t n_rows, int64_t& row_begin, int64_t& row_end) {
  const int64_t n_chunks = (n_rows + kScanRowAlign - 1) / kScanRowAlign;
  const int64_t per_block = (n_chunks + gridDim.x - 1) / gridDim.x;
  row_begin = min((int64_t)blockIdx.x * per_block * kScanRowAlign, n_rows);
  row_end = min(row_begin + per_block * kScanRowAlign, n_rows);
}

}  // namespace

// Tasks that read the primary column's values.  NP = number of inline predicates (exact).
template <typename T, int NP>
__global__ __launch_bounds__(kBlock) void dq_scan_values_kernel(
    const ScanTask* __restrict__ tasks, const int32_t* __restrict__ group,
    const DevColumn* __restrict__ cols, const DevMask* __restrict__ masks, int64_t n_rows,
    ScanAcc* partials) {
  constexpr int RPL = 16 / (int)sizeof(T);
  constexpr int UNROLL = sizeof(T) >= 8 ? 4 : (sizeof(T) == 4 ? 2 : 1);
  constexpr int64_t ROWS_PER_ITER = (int64_t)kBlock * RPL * UNROLL;
  constexpr uint32_t FULL = (1u << RPL) - 1u;

  const int task_id = group[blockIdx.y];
  const ScanTask& task = tasks[task_id];
  int64_t row_begin, row_end;
  chunk_of_block(n_rows, row_begin, row_end);

  const DevColumn& col = cols[task.primary];
  const T* __restrict__ values = static_cast<const T*>(col.values);
  const uint8_t* __restrict__ validity = col.validity;
  const bool has_where = (task.flags & TF_WHERE) != 0;
  const uint8_t* wt_bm = nullptr;
  const uint8_t* wn_bm = nullptr;
  if (has_where) {
    wt_bm = reinterpret_cast<const uint8_t*>(masks[task.where_mask].t);
    wn_bm = reinterpret_cast<const uint8_t*>(masks[task.where_mask].nn);
  }
  FastPred fps[NP > 0 ? NP : 1];
  const uint8_t* mt_bm[NP > 0 ? NP : 1];
  const uint8_t* mn_bm[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    fps[p] = task.preds[p];
    mt_bm[p] = mn_bm[p] = nullptr;
    if (fps[p].kind == FP_MASK) {
      mt_bm[p] = reinterpret_cast<const uint8_t*>(masks[fps[p].mask].t);
      mn_bm[p] = reinterpret_cast<const uint8_t*>(masks[fps[p].mask].nn);
    }
  }

  ThreadAcc<NP> a;
  thread_acc_init(a);
  const int tid = threadIdx.x;
  for (int64_t base = row_begin; base < row_end; base += ROWS_PER_ITER) {
    Vec16 vec[UNROLL];
    uint32_t vb[UNROLL], wtb[UNROLL], wnb[UNROLL], inb[UNROLL];
    // ---- load phase: every load of the group is issued before any use
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t row0 = base + ((int64_t)u * kBlock + tid) * RPL;
      const int64_t left = row_end - row0;
      inb[u] = left >= RPL ? FULL : (left > 0 ? ((1u << (uint32_t)left) - 1u) : 0u);
      vec[u] = Vec16{{0u, 0u, 0u, 0u}};
      vb[u] = wtb[u] = wnb[u] = 0u;
      if (left >= RPL) {
        vec[u] = *reinterpret_cast<const Vec16*>(values + row0);
      } else if (left > 0) {  // last partial vector: element loads, nothing past the end
        T tmp[RPL];
#pragma unroll
        for (int k = 0; k < RPL; ++k) tmp[k] = k < left ? values[row0 + k] : T(0);
        __builtin_memcpy(&vec[u], tmp, 16);
      }
      if (left > 0) {
        vb[u] = validity ? load_bits<RPL>(validity, row0, left) : FULL;
        if (has_where) {
          wtb[u] = load_bits<RPL>(wt_bm, row0, left);
          wnb[u] = load_bits<RPL>(wn_bm, row0, left);
        } else {
          wtb[u] = wnb[u] = FULL;
        }
      }
    }
    // ---- compute phase
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t wt = wtb[u] & inb[u];
      const uint32_t sel = vb[u] & wt;
      a.n_rows += __builtin_popcount(wt);
      a.n_wnn += __builtin_popcount(wnb[u] & inb[u]);
      const T* vals = reinterpret_cast<const T*>(&vec[u]);
#pragma unroll
      for (int k = 0; k < RPL; ++k) accumulate_element<T, NP>(a, vals[k], (sel >> k) & 1u);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        uint32_t mtb = 0u, mnb = 0u;
        if (fps[p].kind == FP_MASK && inb[u]) {
          const int64_t row0 = base + ((int64_t)u * kBlock + tid) * RPL;
          mtb = load_bits<RPL>(mt_bm[p], row0, row_end - row0);
          mnb = load_bits<RPL>(mn_bm[p], row0, row_end - row0);
        }
        uint32_t cm = 0u, cn = 0u;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
          uint32_t r, nn;
          eval_fast_pred<T>(fps[p], vals[k], (vb[u] >> k) & 1u, (mtb >> k) & 1u, (mnb >> k) & 1u, r, nn);
          const uint32_t w = (wt >> k) & 1u;
          cm += w & nn & r;
          cn += w & nn;
        }
        a.pm[p] += cm;
        a.pn[p] += cn;
      }
    }
  }
  thread_finish<NP>(a, NP, &partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x]);
}

// Tasks that need no values (Completeness, Size(where), IS [NOT] NULL / mask / constant
// predicates): 32 rows per lane per step, bit arithmetic only.
__global__ __launch_bounds__(kBlock) void dq_scan_bits_kernel(
    const ScanTask* __restrict__ tasks, const int32_t* __restrict__ group,
    const DevColumn* __restrict__ cols, const DevMask* __restrict__ masks, int64_t n_rows,
    ScanAcc* partials) {
  const int task_id = group[blockIdx.y];
  const ScanTask& task = tasks[task_id];
  int64_t row_begin, row_end;
  chunk_of_block(n_rows, row_begin, row_end);
  const uint32_t* validity = nullptr;
  if (task.primary >= 0) validity = reinterpret_cast<const uint32_t*>(cols[task.primary].validity);
  const bool has_where = (task.flags & TF_WHERE) != 0;
  const uint32_t* wt_w = has_where ? reinterpret_cast<const uint32_t*>(masks[task.where_mask].t) : nullptr;
  const uint32_t* wn_w = has_where ? reinterpret_cast<const uint32_t*>(masks[task.where_mask].nn) : nullptr;
  const int n_preds = task.n_preds;
  uint64_t n_rows_c = 0, n_wnn = 0, n_sel = 0;
  uint64_t pm[kMaxPreds], pn[kMaxPreds];
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) pm[p] = pn[p] = 0;
  for (int64_t row0 = row_begin + (int64_t)threadIdx.x * 32; row0 < row_end;
       row0 += (int64_t)kBlock * 32) {
    const int64_t left = row_end - row0;
    const uint32_t in = left >= 32 ? 0xffffffffu : ((1u << (uint32_t)left) - 1u);
    const int64_t w = row0 >> 5;
    uint32_t vword = 0xffffffffu;
    if (validity) {
      if (left >= 32) {
        vword = validity[w];
      } else {  // tail: byte loads, never past ceil(n_rows / 8)
        const uint8_t* vbp = reinterpret_cast<const uint8_t*>(validity) + (w << 2);
        vword = 0u;
        for (int b = 0; b < (int)((left + 7) >> 3); ++b) vword |= (uint32_t)vbp[b] << (8 * b);
      }
    }
    const uint32_t valid = vword & in;
    const uint32_t wt = (has_where ? wt_w[w] : 0xffffffffu) & in;
    const uint32_t wn = (has_where ? wn_w[w] : 0xffffffffu) & in;
    n_rows_c += __builtin_popcount(wt);
    n_wnn += __builtin_popcount(wn);
    n_sel += __builtin_popcount(valid & wt);
#pragma unroll
    for (int p = 0; p < kMaxPreds; ++p) {
      if (p >= n_preds) break;
      const FastPred& fp = task.preds[p];
      uint32_t r = 0u, nn = 0u;
      switch (fp.kind) {
        case FP_IS_NULL: r = ~valid & in; nn = in; break;
        case FP_IS_NOT_NULL: r = valid; nn = in; break;
        case FP_CONST: r = fp.lit_i == 1 ? in : 0u; nn = fp.lit_i == -1 ? 0u : in; break;
        case FP_MASK: {
          const uint32_t* mt = reinterpret_cast<const uint32_t*>(masks[fp.mask].t);
          const uint32_t* mn = reinterpret_cast<const uint32_t*>(masks[fp.mask].nn);
          r = mt[w] & in;
          nn = mn[w] & in;
          break;
        }
        default: break;
      }
      pm[p] += __builtin_popcount(wt & nn & r);
      pn[p] += __builtin_popcount(wt & nn);
    }
  }
  block_reduce_store<kMaxPreds>(n_rows_c, n_wnn, n_sel, 0, 0, INT64_MAX, INT64_MIN, 0.0, 0.0,
                                __builtin_huge_val(), -__builtin_huge_val(), 0.0, 0.0, pm, pn,
                                n_preds, &partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x]);
}

// One block per task: merge the task's block partials in a fixed order, then fold the batch
// result into the running accumulator (batch order).  Deterministic.
__global__ __launch_bounds__(kBlock) void dq_scan_reduce_kernel(const ScanAcc* __restrict__ partials,
                                                                const PartRange* __restrict__ ranges,
                                                                ScanAcc* acc) {
  const int task_id = blockIdx.x;
  const ScanAcc* p = partials + ranges[task_id].offset;
  const int blocks_per_task = ranges[task_id].count;
  __shared__ ScanAcc slot[kBlock];
  // thread i merges the contiguous range [i*k, (i+1)*k) in block order
  const int k = (blocks_per_task + kBlock - 1) / kBlock;
  const int b0 = threadIdx.x * k;
  ScanAcc a;
  acc_init(a);
  for (int b = b0; b < b0 + k && b < blocks_per_task; ++b) acc_merge(a, p[b]);
  slot[threadIdx.x] = a;
  __syncthreads();
  // fixed pairwise tree over thread order
  for (int s = 1; s < kBlock; s <<= 1) {
    if ((threadIdx.x % (2 * s)) == 0) acc_merge(slot[threadIdx.x], slot[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ScanAcc run = acc[task_id];
    acc_merge(run, slot[0]);
    acc[task_id] = run;
  }
}

__global__ void dq_init_acc_kernel(ScanAcc* acc, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    ScanAcc a;
    acc_init(a);
    acc[i] = a;
  }
}

// ----------------------------------------------------------------------------- launchers
template <typename T>
static hipError_t launch_values_np(int np, dim3 grid, hipStream_t s, const ScanTask* t,
                                   const int32_t* g, const DevColumn* c, const DevMask* m,
                                   int64_t n, ScanAcc* part) {
  switch (np) {
    case 0: hipLaunchKernelGGL((dq_scan_values_kernel<T, 0>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
    case 1: hipLaunchKernelGGL((dq_scan_values_kernel<T, 1>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
    case 2: hipLaunchKernelGGL((dq_scan_values_kernel<T, 2>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
    case 3: hipLaunchKernelGGL((dq_scan_values_kernel<T, 3>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
    case 4: hipLaunchKernelGGL((dq_scan_values_kernel<T, 4>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
    default: hipLaunchKernelGGL((dq_scan_values_kernel<T, kMaxPreds>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part); break;
  }
  return hipGetLastError();
}

hipError_t launch_scan_group(int kind, int ptype, int np, const ScanTask* d_tasks,
                             const int32_t* d_group, int n_group, const DevColumn* d_cols,
                             const DevMask* d_masks, int64_t n_rows, int blocks_per_task,
                             ScanAcc* d_partials, hipStream_t stream) {
  if (n_group <= 0) return hipSuccess;
  dim3 grid(blocks_per_task, n_group);
  if (kind == 0) {
    hipLaunchKernelGGL(dq_scan_bits_kernel, grid, dim3(kBlock), 0, stream, d_tasks, d_group, d_cols,
                       d_masks, n_rows, d_partials);
    return hipGetLastError();
  }
  switch (ptype) {
    case DQ_T_INT8: return launch_values_np<int8_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
    case DQ_T_INT16: return launch_values_np<int16_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
    case DQ_T_INT32: return launch_values_np<int32_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
    case DQ_T_INT64: return launch_values_np<int64_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
    case DQ_T_FLOAT32: return launch_values_np<float>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
    default: return launch_values_np<double>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials);
  }
}

hipError_t launch_scan_reduce(const ScanAcc* d_partials, const PartRange* d_ranges, int n_tasks,
                              ScanAcc* d_acc, hipStream_t stream) {
  if (n_tasks <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_scan_reduce_kernel, dim3(n_tasks), dim3(kBlock), 0, stream, d_partials,
                     d_ranges, d_acc);
  return hipGetLastError();
}

hipError_t launch_init_acc(ScanAcc* d_acc, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_init_acc_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_acc, n);
  return hipGetLastError();
}

}  // namespace dq
