// dq_pair.hip -- the scan-shareable analyzers outside the one-column value scan (dq_scan.hip):
//
// 1. MinLength / MaxLength (MinLength.scala:25-41, MaxLength.scala:25-41):
//      min / max(length(conditionalSelection(column, where))).cast(double)
//    on a utf8 column, where Spark 2.2.2 `length` is UTF8String.numChars: the number of first
//    bytes visited by the walk i += numBytesForFirstByte(b[i]) (0xC0-0xDF -> 2, 0xE0-0xEF -> 3,
//    0xF0-0xF7 -> 4, 0xF8-0xFB -> 5, 0xFC-0xFD -> 6, anything else 1; 0xFE/0xFF, an index error
//    in 2.2.2, step 1 here).  Three integers per task (selected rows, max of ~length, max of
//    length), folded with device atomics: order independent, bit-exact.
// 2. Correlation (Correlation.scala:26-105, catalyst/StatefulCorrelation.scala:24-49): Spark
//    2.2.2 Corr over rows where both inputs are non-NULL (cast to double).  Each lane sums
//    dx, dy, dx^2, dy^2, dx*dy against a wave-uniform shift (no fp64 divide per row), converts to
//    (n, xAvg, yAvg, ck, xMk, yMk) and lanes/waves/blocks are combined with CorrelationState.sum
//    (Correlation.scala:37-52) in a fixed order, so results are bitwise reproducible.
#include "dq_internal.h"

namespace dq {

namespace {

__device__ inline bool bit_at(const uint8_t* bm, int64_t row) { return (bm[row >> 3] >> (row & 7)) & 1u; }
__device__ inline bool word_bit(const uint64_t* w, int64_t row) { return (w[row >> 6] >> (row & 63)) & 1ull; }

__device__ inline uint32_t first_byte_step(uint32_t c) {
  return c < 0xC0u ? 1u : c < 0xE0u ? 2u : c < 0xF0u ? 3u : c < 0xF8u ? 4u : c < 0xFCu ? 5u : c < 0xFEu ? 6u : 1u;
}

__device__ inline uint64_t num_chars(const uint8_t* p, int32_t n) {
  uint64_t chars = 0;
  for (int32_t i = 0; i < n; i += (int32_t)first_byte_step(p[i])) ++chars;
  return chars;
}

__device__ inline uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
  return v;
}
__device__ inline uint64_t wave_max(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ inline double as_double(const DevColumn& c, int64_t row) {
  switch (c.type) {
    case DQ_T_INT8: return (double)static_cast<const int8_t*>(c.values)[row];
    case DQ_T_INT16: return (double)static_cast<const int16_t*>(c.values)[row];
    case DQ_T_INT32: return (double)static_cast<const int32_t*>(c.values)[row];
    case DQ_T_INT64: return (double)static_cast<const int64_t*>(c.values)[row];
    case DQ_T_FLOAT32: return (double)static_cast<const float*>(c.values)[row];
    default: return static_cast<const double*>(c.values)[row];
  }
}

// CorrelationState.sum (Correlation.scala:37-52); empty sides are identities.
__device__ inline void corr_merge(CorrAcc& a, const CorrAcc& b) {
  if (b.n == 0.0) return;
  if (a.n == 0.0) {
    a = b;
    return;
  }
  const double n1 = a.n, n2 = b.n, n = n1 + n2;
  const double dx = b.xavg - a.xavg, dxn = dx / n;
  const double dy = b.yavg - a.yavg, dyn = dy / n;
  a.xavg = a.xavg + dxn * n2;
  a.yavg = a.yavg + dyn * n2;
  a.ck = a.ck + b.ck + dx * dyn * n1 * n2;
  a.xmk = a.xmk + b.xmk + dx * dxn * n1 * n2;
  a.ymk = a.ymk + b.ymk + dy * dyn * n1 * n2;
  a.n = n;
}

__device__ inline CorrAcc shfl_down_acc(const CorrAcc& a, int d) {
  CorrAcc o;
  o.n = __shfl_down(a.n, d, 64);
  o.xavg = __shfl_down(a.xavg, d, 64);
  o.yavg = __shfl_down(a.yavg, d, 64);
  o.ck = __shfl_down(a.ck, d, 64);
  o.xmk = __shfl_down(a.xmk, d, 64);
  o.ymk = __shfl_down(a.ymk, d, 64);
  return o;
}

}  // namespace

// blockIdx.y = task {column, type, where}, blockIdx.x = contiguous row range.
__global__ __launch_bounds__(kBlock) void dq_strlen_kernel(const HllTask* __restrict__ tasks,
                                                           const DevColumn* __restrict__ cols,
                                                           const DevMask* __restrict__ masks, int64_t n_rows,
                                                           unsigned long long* out) {
  const HllTask task = tasks[blockIdx.y];
  const DevColumn& col = cols[task.column];
  const uint64_t* wt = task.where_mask >= 0 ? masks[task.where_mask].t : nullptr;
  const uint8_t* chars = static_cast<const uint8_t*>(col.values);
  const int64_t per_block = (n_rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(r0 + per_block, n_rows);
  uint64_t cnt = 0, max_not = 0, max_len = 0;
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
    // conditionalSelection: a row whose filter is not TRUE is a NULL input (Analyzer.scala:409-420)
    if ((col.validity && !bit_at(col.validity, row)) || (wt && !word_bit(wt, row))) continue;
    const int32_t b = col.offsets[row], e = col.offsets[row + 1];
    const uint64_t len = num_chars(chars + b, e - b);
    ++cnt;
    max_not = (~len) > max_not ? ~len : max_not;
    max_len = len > max_len ? len : max_len;
  }
  cnt = wave_sum(cnt);
  max_not = wave_max(max_not);
  max_len = wave_max(max_len);
  if ((threadIdx.x & 63) == 0 && cnt) {
    unsigned long long* o = out + (int64_t)blockIdx.y * 3;
    atomicAdd(&o[0], (unsigned long long)cnt);
    atomicMax(&o[1], (unsigned long long)max_not);
    atomicMax(&o[2], (unsigned long long)max_len);
  }
}

// blockIdx.y = task {x, y, where}, blockIdx.x = contiguous row range; one CorrAcc partial per block.
__global__ __launch_bounds__(kBlock) void dq_corr_kernel(const CorrTask* __restrict__ tasks,
                                                         const DevColumn* __restrict__ cols,
                                                         const DevMask* __restrict__ masks, int64_t n_rows,
                                                         CorrAcc* partials) {
  const CorrTask task = tasks[blockIdx.y];
  const DevColumn& X = cols[task.x];
  const DevColumn& Y = cols[task.y];
  const uint64_t* wt = task.where_mask >= 0 ? masks[task.where_mask].t : nullptr;
  const int64_t per_block = (n_rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(r0 + per_block, n_rows);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  auto selected = [&](int64_t row) {
    return (!X.validity || bit_at(X.validity, row)) && (!Y.validity || bit_at(Y.validity, row)) &&
           (!wt || word_bit(wt, row));
  };
  // wave-uniform shift: the first selected pair with finite values among the wave's first rows
  double sx = 0.0, sy = 0.0;
  for (uint32_t probe = 0; probe < 4; ++probe) {
    const int64_t row = r0 + (int64_t)(probe * (kBlock / 64) + wave) * 64 + lane;
    bool ok = false;
    double x = 0.0, y = 0.0;
    if (row < r1 && selected(row)) {
      x = as_double(X, row);
      y = as_double(Y, row);
      ok = (x - x == 0.0) && (y - y == 0.0);
    }
    const uint64_t m = __ballot(ok);
    if (m) {
      const int src = __builtin_ctzll(m);
      sx = __shfl(x, src, 64);
      sy = __shfl(y, src, 64);
      break;
    }
  }
  double n = 0.0, s_x = 0.0, s_y = 0.0, s_xx = 0.0, s_yy = 0.0, s_xy = 0.0;
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
    if (!selected(row)) continue;
    const double dx = as_double(X, row) - sx, dy = as_double(Y, row) - sy;
    n += 1.0;
    s_x += dx;
    s_y += dy;
    s_xx += dx * dx;
    s_yy += dy * dy;
    s_xy += dx * dy;
  }
  CorrAcc a;
  a.n = n;
  a.xavg = a.yavg = a.ck = a.xmk = a.ymk = 0.0;
  if (n > 0.0) {
    a.xavg = sx + s_x / n;
    a.yavg = sy + s_y / n;
    a.ck = s_xy - s_x * s_y / n;
    a.xmk = s_xx - s_x * s_x / n;
    a.ymk = s_yy - s_y * s_y / n;
    a.xmk = a.xmk < 0.0 ? 0.0 : a.xmk;  // rounding; NaN/Inf propagate
    a.ymk = a.ymk < 0.0 ? 0.0 : a.ymk;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const CorrAcc o = shfl_down_acc(a, d);
    if ((int)lane < d) corr_merge(a, o);
  }
  __shared__ CorrAcc part[kBlock / 64];
  if (lane == 0) part[wave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    CorrAcc r = part[0];
    for (int w = 1; w < kBlock / 64; ++w) corr_merge(r, part[w]);
    partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = r;
  }
}

// blockIdx.x = task: a fixed pairwise tree over the task's block partials, merged into the
// task's running state (batches in call order).
__global__ __launch_bounds__(kBlock) void dq_corr_reduce_kernel(const CorrAcc* __restrict__ partials,
                                                                int blocks_per_task, CorrAcc* acc) {
  __shared__ CorrAcc slot[kBlock];
  const CorrAcc* p = partials + (int64_t)blockIdx.x * blocks_per_task;
  const int k = (blocks_per_task + kBlock - 1) / kBlock;
  const int b0 = threadIdx.x * k;
  CorrAcc a;
  a.n = a.xavg = a.yavg = a.ck = a.xmk = a.ymk = 0.0;
  for (int b = b0; b < b0 + k && b < blocks_per_task; ++b) corr_merge(a, p[b]);
  slot[threadIdx.x] = a;
  __syncthreads();
  for (int s = 1; s < kBlock; s <<= 1) {
    if ((threadIdx.x % (2 * s)) == 0) corr_merge(slot[threadIdx.x], slot[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    CorrAcc run = acc[blockIdx.x];
    corr_merge(run, slot[0]);
    acc[blockIdx.x] = run;
  }
}

hipError_t launch_strlen(const HllTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                         int64_t n_rows, int blocks_per_task, unsigned long long* d_out, hipStream_t stream) {
  if (n_tasks <= 0 || n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_strlen_kernel, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream, d_tasks, d_cols,
                     d_masks, n_rows, d_out);
  return hipGetLastError();
}

hipError_t launch_corr(const CorrTask* d_tasks, int n_tasks, const DevColumn* d_cols, const DevMask* d_masks,
                       int64_t n_rows, int blocks_per_task, CorrAcc* d_partials, CorrAcc* d_acc,
                       hipStream_t stream) {
  if (n_tasks <= 0 || n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(dq_corr_kernel, dim3(blocks_per_task, n_tasks), dim3(kBlock), 0, stream, d_tasks, d_cols,
                     d_masks, n_rows, d_partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dq_corr_reduce_kernel, dim3(n_tasks), dim3(kBlock), 0, stream, d_partials, blocks_per_task,
                     d_acc);
  return hipGetLastError();
}

}  // namespace dq
