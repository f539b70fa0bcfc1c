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
//   fmin/fmax/nnan : Spark NaN-safe min/max (NaN is the largest double) of (double)x for every
//                    column type (integral min/max commute with the monotone cast); nnan > 0 iff
//                    a selected value is NaN, fmin > fmax iff every selected value is NaN.
//                    (imin/imax stay in the partial layout, unused by the value scan)
//   mean, m2       : moments about the mean, from per-lane shifted sums then Chan merges
//                    with the exact formula of StandardDeviationState.sum
//                    (StandardDeviation.scala:37-44); no per-element fp64 divide
//   pm / pn        : per predicate Σ TRUE / Σ NOT NULL among where-TRUE rows
//                    (Compliance: sum(cast(when(where, pred) as int)), Compliance.scala:49)
//   HLL registers  : ApproxCountDistinct of a numeric column rides on the same pass (TF_HLL):
//                    each selected row is hashed (Spark XXH64, seed 42) into a workgroup copy of
//                    the 512 registers in LDS, folded into the task's set with atomicMax at the
//                    end (StatefulHyperloglogPlus.scala:89-139) -- the column is read once
#include "dq_scan_common.h"

namespace dq {

namespace {

template <typename T> struct IsIntegral { static constexpr bool value = true; };
template <> struct IsIntegral<float> { static constexpr bool value = false; };
template <> struct IsIntegral<double> { static constexpr bool value = false; };


template <int NP>
struct ThreadAcc {
  uint32_t n_rows, n_wnn, n_sel;
  uint64_t nan_wave;  // fp: selected NaN seen (a wave ballot in the tail, a lane flag in the main loop; OR-ed by ballot at the end)
  int64_t isum, imin, imax;
  double fs, fc, fmin, fmax;
  double shift, s1, s2;
  uint32_t pm[NP > 0 ? NP : 1], pn[NP > 0 ? NP : 1];
  // wave-uniform counters of the main loop (ballot + scalar popcount, no VALU): selected rows
  // and one-compare predicate counts; lane counters above cover the diverged tail
  uint64_t n_sel_w;
  uint64_t pm_w[NP > 0 ? NP : 1], pn_w[NP > 0 ? NP : 1];
};

template <int NP>
__device__ inline void thread_acc_init(ThreadAcc<NP>& a) {
  a.n_rows = a.n_wnn = a.n_sel = 0;
  a.nan_wave = 0;
  a.isum = 0;
  a.imin = INT64_MAX;
  a.imax = INT64_MIN;
  a.fs = a.fc = 0.0;
  a.fmin = __builtin_huge_val();
  a.fmax = -__builtin_huge_val();
  a.shift = a.s1 = a.s2 = 0.0;
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) a.pm[p] = a.pn[p] = 0;
  a.n_sel_w = 0;
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) a.pm_w[p] = a.pn_w[p] = 0;
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


// Lane statistics -> block partial.  The moments are formed per wave (the shift is
// wave-uniform, so the lanes' Σd and Σd² simply add), from the wave-uniform main-loop counts
// plus the lanes' tail counts.  fp columns carry (fs, fc) = compensated Σx of the selected values
// (the Sum) and s1 = Σd about the shift (the moments).  Lane 0 carries the wave's totals into the
// block reduction; the other lanes carry identities.

template <typename T, int NP>
__device__ inline void thread_finish(const ThreadAcc<NP>& t, int n_preds, ScanAcc* out) {
  const bool lane0 = (threadIdx.x & 63) == 0;
  const uint64_t n_w = wave_sum_u64((uint64_t)t.n_sel) + t.n_sel_w;  // lane 0
  const double S1 = wave_sum_f64(t.s1), S2 = wave_sum_f64(t.s2);     // lane 0
  double mean = 0.0, m2 = 0.0;
  double fs = t.fs, fc = t.fc;
  uint64_t n_out = 0;
  if (lane0 && n_w > 0) {
    n_out = n_w;
    const double n = (double)n_w;
    mean = t.shift + S1 / n;
    m2 = S2 - S1 * S1 / n;
    m2 = (m2 < 0.0) ? 0.0 : m2;  // rounding; NaN/Inf propagate
  }
  // (the ragged tail runs diverged, so lanes may hold different copies of the flag: OR them)
  const bool wave_nan = __ballot(t.nan_wave != 0) != 0;
  const uint64_t nnan = (lane0 && wave_nan) ? 1u : 0u;
  uint64_t pm[NP > 0 ? NP : 1], pn[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) {
    pm[p] = t.pm[p] + (lane0 ? t.pm_w[p] : 0u);
    pn[p] = t.pn[p] + (lane0 ? t.pn_w[p] : 0u);
  }
  block_reduce_store<NP>(t.n_rows, t.n_wnn, n_out, nnan, t.isum, t.imin, t.imax, fs, fc,
                         t.fmin, t.fmax, mean, m2, pm, pn, n_preds, out);
}


// Statistics over R rows of one lane (selection bits `sel`), against the wave's shift.  The pass
// is bound by VALU issue once HLL rides on it, so each statistic is written for the fewest
// instructions: a selected-row test is one compare reused by every statistic (the min/max
// updates AND it into their compare mask), and int64 -> double is cvt(hi) * 2^32 + cvt(lo) as
// one fma (the same correctly rounded value as (double)xi).
// Min/Max of an integral column are kept on (double)xi: Spark's state is min(col).cast(double)
// (Minimum.scala:40) and round-to-nearest is monotone, so min((double)x) == (double)min(x); a
// v_min_f64 / v_max_f64 pair on the converted value replaces two 64-bit compare-and-selects.
template <typename T, int NP, int R>
__device__ inline void accumulate_rows(ThreadAcc<NP>& a, const T* vals, uint32_t sel, double shift,
                                       double& dsum) {
  if constexpr (IsIntegral<T>::value) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const bool s = (sel >> k) & 1u;
      const int64_t xi = (int64_t)vals[k];
      a.isum += s ? xi : 0;
      double xd;
      if constexpr (sizeof(T) == 8) {  // cvt(hi) * 2^32 + cvt(lo), one rounding
        xd = fma((double)(int32_t)((uint64_t)xi >> 32), 0x1p32, (double)(uint32_t)(uint64_t)xi);
      } else {
        xd = (double)xi;
      }
      const double d = s ? (xd - shift) : 0.0;
      a.s1 += d;
      a.s2 = fma(d, d, a.s2);
      // an unselected row offers a quiet NaN (one select on the high word), which the
      // hardware min / max drop
      const uint64_t xb = __builtin_bit_cast(uint64_t, xd);
      const uint32_t xh = s ? (uint32_t)(xb >> 32) : 0x7ff80000u;
      const double xn = __builtin_bit_cast(double, ((uint64_t)xh << 32) | (uint32_t)xb);
      a.fmin = vmin_f64(a.fmin, xn);
      a.fmax = vmax_f64(a.fmax, xn);
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const bool s = (sel >> k) & 1u;
      const double x = (double)vals[k];
      // the fp64 Sum is taken over the raw values (compensated per iteration by the caller):
      // n * shift + Σd would lose what x - shift rounds away when |x| >> |shift|
      const double d = s ? (x - shift) : 0.0;
      dsum += s ? x : 0.0;
      a.s1 += d;
      a.s2 = fma(d, d, a.s2);
      // min / max through minnum / maxnum of the value, or of a quiet NaN (one select on the
      // high word) for an unselected row: minnum / maxnum drop a NaN operand, so a NaN never
      // wins min (Spark's NaN-safe order) and the max is restored from the NaN flag.
      const uint64_t xb = __builtin_bit_cast(uint64_t, x);
      const uint32_t xh = s ? (uint32_t)(xb >> 32) : 0x7ff80000u;
      const double xn = __builtin_bit_cast(double, ((uint64_t)xh << 32) | (uint32_t)xb);
      a.fmin = vmin_f64(a.fmin, xn);
      a.fmax = vmax_f64(a.fmax, xn);
      // any selected NaN.  The main loop (R > 1) tests its iteration's Σd once instead: a
      // selected NaN makes it NaN (see nan_recheck)
      if constexpr (R == 1) a.nan_wave |= __ballot(s & (x != x));
    }
  }
}

// Compare bits of R values against the literal, branch-free in the operator: lt / eq are
// computed, "greater" is neither (which also puts a NaN x above every literal, Spark's
// NaN-safe order), and the uniform selectors pick the operator's answer.
template <typename V, int R>
__device__ inline uint32_t cmp_bits(const V* x, V lit, const FastPred& fp) {
  uint32_t r = 0u;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const uint32_t lt = x[k] < lit ? ~0u : 0u;
    const uint32_t eq = x[k] == lit ? ~0u : 0u;
    const uint32_t b = (lt & fp.m_lt) | (eq & fp.m_eq) | (~(lt | eq) & fp.m_gt);
    r |= b & (1u << k);
  }
  return r;
}

// The one-compare form (FastPred::cmp_sel): one v_cmp per value, the operator's negation
// applied once to the R bits.
template <int CS, typename V, int R>
__device__ inline uint32_t cmp_bits1(const V* x, V lit) {
  uint32_t r = 0u;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    bool b;
    if constexpr (CS == CS_LT) b = x[k] < lit;
    else if constexpr (CS == CS_LE) b = x[k] <= lit;
    else b = x[k] == lit;
    r |= b ? (1u << k) : 0u;
  }
  return r;
}

template <typename V, int R>
__device__ inline uint32_t cmp_dispatch(const V* x, V lit, const FastPred& fp) {
  constexpr uint32_t FULL = (R == 32) ? 0xffffffffu : ((1u << R) - 1u);
  const uint32_t inv = (fp.cmp_sel & CS_INV) ? FULL : 0u;
  switch (fp.cmp_sel & 3u) {  // uniform
    case CS_LT: return cmp_bits1<CS_LT, V, R>(x, lit) ^ inv;
    case CS_LE: return cmp_bits1<CS_LE, V, R>(x, lit) ^ inv;
    case CS_EQ: return cmp_bits1<CS_EQ, V, R>(x, lit) ^ inv;
    default: return cmp_bits<V, R>(x, lit, fp);
  }
}

// One inline predicate over R rows: counts TRUE and NOT NULL among where-TRUE rows (lane bits).
template <typename T, int NP, int R>
__device__ inline void predicate_one(ThreadAcc<NP>& a, int p, const FastPred& fp, const T* vals,
                                     uint32_t valid, uint32_t wt, uint32_t mt, uint32_t mn) {
  constexpr uint32_t FULL = (R == 32) ? 0xffffffffu : ((1u << R) - 1u);
  uint32_t c = 0u;
  if (fp.f_cmp) {  // uniform
    if (IsIntegral<T>::value && !fp.as_f64) {
      int64_t x[R];
      if (fp.f_coal) {  // uniform
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = ((valid >> k) & 1u) ? (int64_t)vals[k] : fp.coal_i;
      } else {
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = (int64_t)vals[k];
      }
      c = cmp_dispatch<int64_t, R>(x, fp.lit_i, fp);
    } else {
      double x[R];
      if (fp.f_coal) {
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = ((valid >> k) & 1u) ? (double)vals[k] : fp.coal_f;
      } else {
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = (double)vals[k];
      }
      c = cmp_dispatch<double, R>(x, fp.lit_f, fp);
    }
  }
  const uint32_t r = ((c & fp.f_cmp) | (~valid & fp.f_isnull) | (valid & fp.f_isnotnull) |
                      fp.f_true | (mt & fp.f_mask)) & FULL;
  const uint32_t nn = ((valid & fp.f_nn_valid) | fp.f_nn_one | (mn & fp.f_mask)) & FULL;
  a.pm[p] += __builtin_popcount(wt & nn & r);
  a.pn[p] += __builtin_popcount(wt & nn);
}

template <typename T, int NP, int R>
__device__ inline void predicate_rows(ThreadAcc<NP>& a, const FastPred* fps, const T* vals,
                                      uint32_t valid, uint32_t wt, const uint32_t* mt,
                                      const uint32_t* mn) {
#pragma unroll
  for (int p = 0; p < NP; ++p) predicate_one<T, NP, R>(a, p, fps[p], vals, valid, wt, mt[p], mn[p]);
}

// Main-loop form of predicate_rows: a plain `column CMP literal` (kind FP_CMP with a one-compare
// selector) is counted with one v_cmp per row and a ballot popcount on the scalar unit; other
// kinds fall back to the lane bit path.  Uniform control flow only (wave-uniform counters).
template <typename T, int NP, int R>
__device__ inline void predicate_rows_wave(ThreadAcc<NP>& a, const FastPred* fps, const T* vals,
                                           uint32_t valid, uint32_t wt, uint32_t sel,
                                           const uint32_t* mt, const uint32_t* mn) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const FastPred& fp = fps[p];
    const uint32_t cs = fp.cmp_sel & 3u;
    if (fp.kind == FP_CMP && cs != CS_MASKS) {  // uniform
      const bool inv = (fp.cmp_sel & CS_INV) != 0;
      const bool f64 = !IsIntegral<T>::value || fp.as_f64;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const bool in = (sel >> k) & 1u;  // valid & where TRUE (FP_CMP: NOT NULL = valid)
        bool b;
        if (f64) {
          const double x = (double)vals[k];
          b = cs == CS_LT ? x < fp.lit_f : (cs == CS_LE ? x <= fp.lit_f : x == fp.lit_f);
        } else {
          const int64_t x = (int64_t)vals[k];
          b = cs == CS_LT ? x < fp.lit_i : (cs == CS_LE ? x <= fp.lit_i : x == fp.lit_i);
        }
        a.pm_w[p] += __builtin_popcountll(__ballot(in & (b != inv)));
        a.pn_w[p] += __builtin_popcountll(__ballot(in));
      }
    } else {
      predicate_one<T, NP, R>(a, p, fp, vals, valid, wt, mt[p], mn[p]);
    }
  }
}

}  // namespace

// Tasks that read the primary column's values.  NP = number of inline predicates (exact).
// The block's row chunk is addressed through buffer descriptors (32-bit offsets, hardware
// range check), the main loop runs over whole iterations with no bounds checks, and the
// ragged end of the chunk is finished element by element.
// EXT = the task has a `where` mask or mask-based predicates.  Every load of the main loop is
// unconditional: an absent buffer gets a zero-size descriptor (the hardware range check
// returns 0 without touching memory) and a uniform "absent" mask is OR-ed in afterwards, so
// no load sits behind a branch (which would force a vmcnt(0) per load).
template <typename T, int NP, bool EXT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu((NP <= 3 && !EXT && sizeof(T) >= 4) ? 6 : 1))) void dq_scan_values_kernel(
    const ScanTask* __restrict__ tasks, const int32_t* __restrict__ group,
    const DevColumn* __restrict__ cols, const DevMask* __restrict__ masks, int64_t n_rows,
    ScanAcc* partials, uint32_t* __restrict__ hll_regs) {
  constexpr int RPL = 16 / (int)sizeof(T);
  constexpr int UNROLL = sizeof(T) >= 8 ? 4 : (sizeof(T) == 4 ? 2 : 1);
  constexpr uint32_t ROWS_PER_ITER = (uint32_t)kBlock * RPL * UNROLL;
  constexpr uint32_t FULL = (1u << RPL) - 1u;
  constexpr int NPS = NP > 0 ? NP : 1;

  const int task_id = group[blockIdx.y];
  const ScanTask& task = tasks[task_id];
  int64_t row_begin, row_end;
  chunk_of_block(n_rows, row_begin, row_end);
  const uint32_t span = (uint32_t)(row_end - row_begin);  // host keeps span * 8 < 4 GiB
  // fused ApproxCountDistinct: the workgroup's copy of the 512 registers (uniform per block)
  __shared__ uint32_t lregs[kHllM];
  const bool hll_on = (task.flags & TF_HLL) != 0;
  // Sum/Mean/StdDev/Min/Max of the primary column wanted (uniform per block: a scalar branch)
  const bool stats_on = (task.flags & TF_STATS) != 0;
  if (hll_on) {
    for (int r = threadIdx.x; r < kHllM; r += kBlock) lregs[r] = 0u;
    __syncthreads();
  }

  const DevColumn& col = cols[task.primary];
  const __amdgpu_buffer_rsrc_t rv =
      make_rsrc(static_cast<const T*>(col.values) + row_begin, span * (uint32_t)sizeof(T));
  const bool has_valid = col.validity != nullptr;
  const uint32_t no_valid = has_valid ? 0u : ~0u;
  const uint32_t bm_bytes = (span + 7u) >> 3;
  const __amdgpu_buffer_rsrc_t rvalid =
      make_rsrc(has_valid ? col.validity + (row_begin >> 3) : nullptr, has_valid ? bm_bytes : 0u);
  const bool has_where = EXT && (task.flags & TF_WHERE) != 0;
  const uint32_t no_where = has_where ? 0u : ~0u;
  __amdgpu_buffer_rsrc_t rwt = make_rsrc(nullptr, 0), rwn = make_rsrc(nullptr, 0);
  if (has_where) {
    rwt = make_rsrc(reinterpret_cast<const uint8_t*>(masks[task.where_mask].t) + (row_begin >> 3), bm_bytes);
    rwn = make_rsrc(reinterpret_cast<const uint8_t*>(masks[task.where_mask].nn) + (row_begin >> 3), bm_bytes);
  }
  FastPred fps[NPS];
  __amdgpu_buffer_rsrc_t rmt[NPS], rmn[NPS];
  rmt[0] = rmn[0] = make_rsrc(nullptr, 0);  // (NP == 0: the tail still reads slot 0)
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    fps[p] = task.preds[p];
    rmt[p] = rmn[p] = make_rsrc(nullptr, 0);
    if (EXT && fps[p].kind == FP_MASK) {
      rmt[p] = make_rsrc(reinterpret_cast<const uint8_t*>(masks[fps[p].mask].t) + (row_begin >> 3), bm_bytes);
      rmn[p] = make_rsrc(reinterpret_cast<const uint8_t*>(masks[fps[p].mask].nn) + (row_begin >> 3), bm_bytes);
    }
  }

  // Wave-uniform shift for the moments: the first valid, finite value among the wave's
  // first rows (any sample of the column keeps Σ(x - c)² well conditioned).
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  double shift = 0.0;
  for (uint32_t probe = 0; probe < 4; ++probe) {
    const uint32_t r = (probe * (kBlock / 64) + wave) * 64u + lane;
    bool ok = false;
    double x = 0.0;
    if (r < span) {
      x = (double)buf_elem<T>(rv, r);
      ok = (has_valid ? ((buf_bits<1>(rvalid, r)) & 1u) : 1u) && (x - x == 0.0);
    }
    const uint64_t m = __ballot(ok);
    if (m) {
      const int src = __builtin_ctzll(m);
      shift = __shfl(x, src, 64);
      // near DBL_MAX, x - shift could overflow for values of the other sign: no shift then
      if (!(fabs(shift) <= 0x1p1000)) shift = 0.0;
      break;
    }
  }

  ThreadAcc<NP> a;
  thread_acc_init(a);
  const uint32_t tid = threadIdx.x;
  const uint32_t full_iters = span / ROWS_PER_ITER;
#pragma unroll 1
  for (uint32_t it = 0; it < full_iters; ++it) {
    dq_v4u vec[UNROLL];
    uint32_t vb[UNROLL], wtb[UNROLL], wnb[UNROLL];
    uint32_t mtb[UNROLL][NPS], mnb[UNROLL][NPS];
    // ---- load phase: every load of the iteration is issued before any use
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint32_t r0 = it * ROWS_PER_ITER + ((uint32_t)u * kBlock + tid) * RPL;
      vec[u] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(r0 * (uint32_t)sizeof(T)), 0, 0);
      vb[u] = buf_bits<RPL>(rvalid, r0);
      if constexpr (EXT) {
        wtb[u] = buf_bits<RPL>(rwt, r0);
        wnb[u] = buf_bits<RPL>(rwn, r0);
#pragma unroll
        for (int p = 0; p < NPS; ++p) {
          mtb[u][p] = buf_bits<RPL>(rmt[p], r0);
          mnb[u][p] = buf_bits<RPL>(rmn[p], r0);
        }
      } else {
        wtb[u] = wnb[u] = FULL;
#pragma unroll
        for (int p = 0; p < NPS; ++p) mtb[u][p] = mnb[u][p] = 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {  // absent buffers read as 0: restore "all valid/TRUE"
      vb[u] = (vb[u] | no_valid) & FULL;
      wtb[u] = (wtb[u] | no_where) & FULL;
      wnb[u] = (wnb[u] | no_where) & FULL;
    }
    // ---- compute phase
    double dsum = -0.0;  // (-0.0 + d == d for every d: the first add folds away)
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const T* vals = reinterpret_cast<const T*>(&vec[u]);
      const uint32_t sel = vb[u] & wtb[u];
      a.n_rows += __builtin_popcount(wtb[u]);
      a.n_wnn += __builtin_popcount(wnb[u]);
#pragma unroll
      for (int k = 0; k < RPL; ++k) a.n_sel_w += __builtin_popcountll(__ballot((sel >> k) & 1u));
      if (stats_on) accumulate_rows<T, NP, RPL>(a, vals, sel, shift, dsum);
      predicate_rows_wave<T, NP, RPL>(a, fps, vals, vb[u], wtb[u], sel, mtb[u], mnb[u]);
    }
    if (hll_on) {  // every row is hashed (branch-free); unselected rows raise nothing
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const T* vals = reinterpret_cast<const T*>(&vec[u]);
        const uint32_t sel = vb[u] & wtb[u];
#pragma unroll
        for (int k = 0; k < RPL; ++k)
          hll_hash_update<T>(lregs, vals[k], (sel >> k) & 1u);
      }
    }
    if constexpr (!IsIntegral<T>::value) {
      if (stats_on) {
        // NaN detection, one compare per iteration: a selected NaN makes this lane's Σd NaN
        // (unselected rows contribute an exact 0), so only a NaN Σd -- a NaN, or +Inf and -Inf
        // together -- re-tests the iteration's rows exactly.  Rare and lane-divergent.
        if (__builtin_expect(dsum != dsum, 0)) {
#pragma unroll
          for (int u = 0; u < UNROLL; ++u) {
            const T* vals = reinterpret_cast<const T*>(&vec[u]);
            const uint32_t sel = vb[u] & wtb[u];
#pragma unroll
            for (int k = 0; k < RPL; ++k)
              if (((sel >> k) & 1u) && vals[k] != vals[k]) a.nan_wave = 1u;
          }
        }
        neumaier_add(a.fs, a.fc, dsum);
      }
    }
  }
  // ---- ragged end of the chunk: one row per lane
  double dsum = 0.0;
  for (uint32_t r = full_iters * ROWS_PER_ITER + tid; r < span; r += kBlock) {
    const T v = buf_elem<T>(rv, r);
    const uint32_t valid = (buf_bits<1>(rvalid, r) | no_valid) & 1u;
    const uint32_t wt = (buf_bits<1>(rwt, r) | no_where) & 1u;
    const uint32_t wn = (buf_bits<1>(rwn, r) | no_where) & 1u;
    uint32_t mt[NPS], mn[NPS];
#pragma unroll
    for (int p = 0; p < NPS; ++p) {
      mt[p] = buf_bits<1>(rmt[p], r) & 1u;
      mn[p] = buf_bits<1>(rmn[p], r) & 1u;
    }
    a.n_rows += wt;
    a.n_wnn += wn;
    a.n_sel += valid & wt;
    if (stats_on) accumulate_rows<T, NP, 1>(a, &v, valid & wt, shift, dsum);
    predicate_rows<T, NP, 1>(a, fps, &v, valid, wt, mt, mn);
    if (hll_on) hll_hash_update<T>(lregs, v, valid & wt & 1u);
  }
  if constexpr (!IsIntegral<T>::value) neumaier_add(a.fs, a.fc, dsum);
  if (hll_on) {  // fold the workgroup's registers into the task's set (max: order independent)
    __syncthreads();
    uint32_t* out = hll_regs + (int64_t)task.hll * kHllM;
    for (int r = threadIdx.x; r < kHllM; r += kBlock) {
      const uint32_t v = lregs[r];
      if (v) atomicMax(&out[r], v);
    }
  }
  a.shift = shift;
  if (stats_on) {  // (block-uniform) the cancellation guard of the shifted moments
    const uint64_t n_w = wave_sum_u64((uint64_t)a.n_sel) + a.n_sel_w;  // lane 0
    const double S1 = wave_sum_f64(a.s1), S2 = wave_sum_f64(a.s2);
    double wn = 0.0, wmean = 0.0;
    bool cancel = false;
    if (lane == 0 && n_w > 0) {
      wn = (double)n_w;
      wmean = shift + S1 / wn;
      cancel = moments_cancel(wn, S1, S2);
    }
    if (__syncthreads_or(cancel)) {
      // redo Σd, Σd² of the chunk about its mean, one row per lane; the lanes' selected counts
      // move with them (the block's total is unchanged)
      const double m = block_mean_of_waves(wn, wmean);
      if (fabs(m) <= 0x1p1000) {
        a.shift = m;
        a.s1 = a.s2 = 0.0;
        a.n_sel = 0u;
        a.n_sel_w = 0u;
        for (uint32_t r = tid; r < span; r += kBlock) {
          const double x = (double)buf_elem<T>(rv, r);
          const uint32_t s = (buf_bits<1>(rvalid, r) | no_valid) & (buf_bits<1>(rwt, r) | no_where) & 1u;
          const double dd = s ? (x - m) : 0.0;
          a.s1 += dd;
          a.s2 = fma(dd, dd, a.s2);
          a.n_sel += s;
        }
      }
    }
  }
  thread_finish<T, NP>(a, NP, &partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x]);
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
        case FP_BOOL: {  // the primary bool column's value bits (same tail rule as validity)
          const uint8_t* vb = static_cast<const uint8_t*>(cols[task.primary].values) + (w << 2);
          uint32_t bits = 0u;
          if (left >= 32) {
            bits = *reinterpret_cast<const uint32_t*>(vb);
          } else {
            for (int b = 0; b < (int)((left + 7) >> 3); ++b) bits |= (uint32_t)vb[b] << (8 * b);
          }
          r = bits & valid;
          nn = valid;
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
                                   int64_t n, ScanAcc* part, uint32_t* hr) {
  if (np < 0) {  // EXT: where masks / mask predicates, all predicate slots
    hipLaunchKernelGGL((dq_scan_values_kernel<T, kMaxPreds, true>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr);
    return hipGetLastError();
  }
  switch (np) {
    case 0: hipLaunchKernelGGL((dq_scan_values_kernel<T, 0, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
    case 1: hipLaunchKernelGGL((dq_scan_values_kernel<T, 1, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
    case 2: hipLaunchKernelGGL((dq_scan_values_kernel<T, 2, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
    case 3: hipLaunchKernelGGL((dq_scan_values_kernel<T, 3, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
    case 4: hipLaunchKernelGGL((dq_scan_values_kernel<T, 4, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
    default: hipLaunchKernelGGL((dq_scan_values_kernel<T, kMaxPreds, false>), grid, dim3(kBlock), 0, s, t, g, c, m, n, part, hr); break;
  }
  return hipGetLastError();
}

hipError_t launch_scan_group(int kind, int ptype, int np, const ScanTask* d_tasks,
                             const int32_t* d_group, int n_group, const DevColumn* d_cols,
                             const DevMask* d_masks, int64_t n_rows, int blocks_per_task,
                             ScanAcc* d_partials, uint32_t* d_hll_regs, hipStream_t stream) {
  if (n_group <= 0) return hipSuccess;
  dim3 grid(blocks_per_task, n_group);
  if (kind == 0) {
    hipLaunchKernelGGL(dq_scan_bits_kernel, grid, dim3(kBlock), 0, stream, d_tasks, d_group, d_cols,
                       d_masks, n_rows, d_partials);
    return hipGetLastError();
  }
  switch (ptype) {
    case DQ_T_INT8: return launch_values_np<int8_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials, d_hll_regs);
    case DQ_T_INT16: return launch_values_np<int16_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials,
                                                        d_hll_regs);
    case DQ_T_INT32: return launch_values_np<int32_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials,
                                                        d_hll_regs);
    case DQ_T_INT64: return launch_values_np<int64_t>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials,
                                                        d_hll_regs);
    case DQ_T_FLOAT32: return launch_values_np<float>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials,
                                                        d_hll_regs);
    default: return launch_values_np<double>(np, grid, stream, d_tasks, d_group, d_cols, d_masks, n_rows, d_partials,
                                                        d_hll_regs);
  }
}

// Workgroups of one value-scan specialisation that fit on a CU at once (VGPR-bound), so the
// host can size the grid to whole rounds of resident workgroups: a grid of 1.33 rounds leaves
// the last third of the pass running at a third of the occupancy.
template <typename T>
static const void* values_kernel_ptr(int np) {
  if (np < 0) return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, kMaxPreds, true>);
  switch (np) {
    case 0: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, 0, false>);
    case 1: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, 1, false>);
    case 2: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, 2, false>);
    case 3: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, 3, false>);
    case 4: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, 4, false>);
    default: return reinterpret_cast<const void*>(&dq_scan_values_kernel<T, kMaxPreds, false>);
  }
}

int scan_group_blocks_per_cu(int kind, int ptype, int np) {
  const void* fn;
  if (kind == 0) {
    fn = reinterpret_cast<const void*>(&dq_scan_bits_kernel);
  } else {
    switch (ptype) {
      case DQ_T_INT8: fn = values_kernel_ptr<int8_t>(np); break;
      case DQ_T_INT16: fn = values_kernel_ptr<int16_t>(np); break;
      case DQ_T_INT32: fn = values_kernel_ptr<int32_t>(np); break;
      case DQ_T_INT64: fn = values_kernel_ptr<int64_t>(np); break;
      case DQ_T_FLOAT32: fn = values_kernel_ptr<float>(np); break;
      default: fn = values_kernel_ptr<double>(np); break;
    }
  }
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kBlock, 0) != hipSuccess || nb < 1) return 0;
  return nb;
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
