// dq_scan_common.h -- device helpers shared by the value-scan kernels (dq_scan.hip, the general
// kernels; dq_scan_fast.hip, the specialised 8-byte-column kernel): the ScanAcc merge algebra
// (StandardDeviationState.sum, StandardDeviation.scala:37-44), fixed-order wave / block
// reductions, chunking and buffer-descriptor loads.  Internal, not part of the ABI.
#pragma once

#include "dq_internal.h"

namespace dq {
namespace {

// Neumaier step: s + x with the rounding error carried in c.
__device__ inline void neumaier_add(double& s, double& c, double x) {
  const double t = s + x;
  c += (fabs(s) >= fabs(x)) ? ((s - t) + x) : ((x - t) + s);
  s = t;
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
__device__ __attribute__((always_inline)) inline void block_reduce_store(uint64_t n_rows, uint64_t n_wnn, uint64_t n_sel, uint64_t nnan,
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
  // The waves' partials merged in wave order, field group by field group on separate threads:
  // the same result as acc_merge(part[0], part[w]) for w = 1..3, without holding two whole
  // ScanAcc records in one thread's registers (which would set the kernel's VGPR count).
  const int t = threadIdx.x;
  constexpr int W = kBlock / 64;
  if (t < kMaxPreds) {
    int64_t m = part[0].pm[t], n = part[0].pn[t];
#pragma unroll 1
    for (int w = 1; w < W; ++w) {
      m += part[w].pm[t];
      n += part[w].pn[t];
    }
    out->pm[t] = m;
    out->pn[t] = n;
  } else if (t == kMaxPreds) {
    int64_t nr = part[0].n_rows, nw = part[0].n_wnn, nn = part[0].nnan;
    uint64_t is = (uint64_t)part[0].isum;
#pragma unroll 1
    for (int w = 1; w < W; ++w) {
      nr += part[w].n_rows;
      nw += part[w].n_wnn;
      nn += part[w].nnan;
      is += (uint64_t)part[w].isum;
    }
    out->n_rows = nr;
    out->n_wnn = nw;
    out->nnan = nn;
    out->isum = (int64_t)is;
  } else if (t == kMaxPreds + 1) {
    int64_t lo = part[0].imin, hi = part[0].imax;
    double fl = part[0].fmin, fh = part[0].fmax;
#pragma unroll 1
    for (int w = 1; w < W; ++w) {
      lo = part[w].imin < lo ? part[w].imin : lo;
      hi = part[w].imax > hi ? part[w].imax : hi;
      fl = part[w].fmin < fl ? part[w].fmin : fl;
      fh = part[w].fmax > fh ? part[w].fmax : fh;
    }
    out->imin = lo;
    out->imax = hi;
    out->fmin = fl;
    out->fmax = fh;
  } else if (t == kMaxPreds + 2) {
    double fs = part[0].fs, fc = part[0].fc;
#pragma unroll 1
    for (int w = 1; w < W; ++w) two_sum_merge(fs, fc, part[w].fs, part[w].fc);
    out->fs = fs;
    out->fc = fc;
  } else if (t == kMaxPreds + 3) {
    double n = (double)part[0].n_sel, mean = part[0].mean, m2 = part[0].m2;
    int64_t ns = part[0].n_sel;
#pragma unroll 1
    for (int w = 1; w < W; ++w) {
      moments_merge(n, mean, m2, (double)part[w].n_sel, part[w].mean, part[w].m2);
      ns += part[w].n_sel;
    }
    out->n_sel = ns;
    out->mean = mean;
    out->m2 = m2;
  }
}

__device__ inline double wave_sum_f64(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_down(v, d, 64);
  return v;
}

// Cancellation guard of the shifted moments.  Both value scans take a wave's Σd, Σd² about a
// shift c (a value of the column the wave saw first) and form m2 = S2 - S1²/n, whose relative
// rounding is about eps * S2 / m2: harmless while c lies near the data, but when c is an outlier
// (a 1e8 sentinel among N(0, 1) values) S1²/n is nearly all of S2 and the difference cancels.
// Spark's per-row update has no such mode (CentralMomentAgg, StandardDeviation.scala:37-44
// merge), so a wave whose S1²/n exceeds kMomentCancel * m2 makes its workgroup redo the moments
// of its chunk about the chunk's mean (then S1 ~ 0 and S2 ~ m2).  Ordinary data never comes close:
// a uniform column gives at most 3, a normal one needs c beyond 4 sigma.
constexpr double kMomentCancel = 16.0;
__device__ inline bool moments_cancel(double n, double S1, double S2) {
  const double q = S1 * S1 / n;
  return q > kMomentCancel * (S2 - q);  // (NaN / Inf moments: false, nothing to rescue)
}

// The workgroup's mean from its waves' (n, mean) (lane 0 of each wave supplies them), merged in
// wave order; every thread gets the same value.  Called at most once per kernel.
__device__ inline double block_mean_of_waves(double n_w, double mean_w) {
  __shared__ double s_n[kBlock / 64], s_m[kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    s_n[threadIdx.x >> 6] = n_w;
    s_m[threadIdx.x >> 6] = mean_w;
  }
  __syncthreads();
  double n = 0.0, m = 0.0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w) {
    if (s_n[w] > 0.0) {
      const double nn = n + s_n[w];
      m += (s_m[w] - m) * (s_n[w] / nn);
      n = nn;
    }
  }
  return m;
}

__device__ inline void chunk_of_block(int64_t n_rows, int64_t& row_begin, int64_t& row_end) {
  const int64_t n_chunks = (n_rows + kScanRowAlign - 1) / kScanRowAlign;
  const int64_t per_block = (n_chunks + gridDim.x - 1) / gridDim.x;
  row_begin = min((int64_t)blockIdx.x * per_block * kScanRowAlign, n_rows);
  row_end = min(row_begin + per_block * kScanRowAlign, n_rows);
}

typedef uint32_t dq_v4u __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// `RPL` validity/mask bits of the rows starting at chunk row `r0` (r0 % RPL == 0).
template <int RPL>
__device__ inline uint32_t buf_bits(__amdgpu_buffer_rsrc_t rs, uint32_t r0) {
  if constexpr (RPL == 16) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)(r0 >> 3), 0, 0);
  } else {
    const uint32_t byte = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(r0 >> 3), 0, 0);
    return (byte >> (r0 & 7u)) & ((1u << RPL) - 1u);
  }
}

template <typename T>
__device__ inline T buf_elem(__amdgpu_buffer_rsrc_t rs, uint32_t row) {
  if constexpr (sizeof(T) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(row * 8u), 0, 0);
    return __builtin_bit_cast(T, (uint64_t)v[0] | ((uint64_t)v[1] << 32));
  } else if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(row * 4u), 0, 0));
  } else if constexpr (sizeof(T) == 2) {
    return __builtin_bit_cast(T, (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)(row * 2u), 0, 0));
  } else {
    return __builtin_bit_cast(T, (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)row, 0, 0));
  }
}

// v_min_f64 / v_max_f64 as the hardware does them: a quiet-NaN operand is dropped.  (minnum /
// maxnum through the compiler add a canonicalising op per operand.)
__device__ inline double vmin_f64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ inline double vmax_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

}  // namespace
}  // namespace dq
