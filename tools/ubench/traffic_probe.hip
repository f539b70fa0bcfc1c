// traffic_probe.hip -- known-byte kernels for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 per ACCESS SHAPE (the guide validates FETCH_SIZE = half the bytes only for wide
// coalesced streaming reads: MI355X_MICROARCH.md §HBM).  Each probe kernel moves a known number
// of bytes in one shape the library's kernels use; the buffers are 2-4 GiB (far beyond the
// 256 MiB Infinity Cache) and every probe touches fresh data.  The program prints one JSON line
// per probe: kernel name, algorithmic bytes read / written, lines touched.  tools/ubench/
// traffic_probe.sh runs it under one `rocprofv3 --pmc` pass per counter and divides.
// Build: hipcc -O3 --offload-arch=gfx950 traffic_probe.hip -o traffic_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ inline uint64_t mix(uint64_t x) {
  x ^= x >> 31;
  x *= 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  return x;
}

// 1. wide streaming read: 16 B per lane, consecutive lanes consecutive 16 B
__global__ void probe_read_wide16(const uint4* __restrict__ in, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// 2. streaming read, 8 B per lane
__global__ void probe_read_b64(const uint64_t* __restrict__ in, uint64_t n, uint32_t* sink) {
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= in[i];
  if (acc == 0x12345678ull) sink[0] = (uint32_t)acc;
}
// 3. streaming read, 4 B per lane (256 B per wave instruction)
__global__ void probe_read_b32(const uint32_t* __restrict__ in, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= in[i];
  if (acc == 0x12345678u) sink[0] = acc;
}
// 4. bitmap-shaped read: 16 lanes x 4 B = 64 contiguous bytes per wave instruction (a validity
//    bitmap read beside 8-byte values: 1 bit per row), waves sweeping the buffer in order
__global__ void probe_read_64B_per_wave(const uint32_t* __restrict__ in, uint64_t n_words, uint32_t* sink) {
  uint32_t acc = 0;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (lane < 16u)
    for (uint64_t c = wave; c * 16 < n_words; c += waves) acc ^= in[c * 16 + lane];
  if (acc == 0x12345678u) sink[0] = acc;
}
// 5. random 8-B gathers from a large table
__global__ void probe_gather8(const uint64_t* __restrict__ table, uint64_t table_n, uint64_t n, uint32_t* sink) {
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= table[mix(i) % table_n];
  if (acc == 0x12345678ull) sink[0] = (uint32_t)acc;
}
// 6. wide streaming write: 16 B per lane
__global__ void probe_write_wide16(uint4* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
// 7. streaming write, 8 B per lane
__global__ void probe_write_b64(uint64_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = i;
}
// 8. runs of 12 x 8 B (96 B, the split's ~12 records per bin per tile) at random 8-B-aligned
//    positions: lanes 0-59 of a wave write 5 runs, every run somewhere else in the buffer
__global__ void probe_write_runs96(uint64_t* __restrict__ out, uint64_t out_n, uint64_t n_runs) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  if (lane >= 60u) return;
  for (uint64_t r = wave * 5 + lane / 12; r < n_runs; r += waves * 5) {
    const uint64_t base = mix(r) % (out_n - 12);
    out[base + lane % 12] = r;
  }
}
// 9. the same runs, line-aligned: 16 x 8 B = one whole 128-B line per run
__global__ void probe_write_lines128(uint64_t* __restrict__ out, uint64_t out_lines, uint64_t n_runs) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t r = wave * 4 + lane / 16; r < n_runs; r += waves * 4) {
    const uint64_t line = mix(r) % out_lines;
    out[line * 16 + lane % 16] = r;
  }
}
// 10. 8-B stores at random positions
__global__ void probe_scatter8(uint64_t* __restrict__ out, uint64_t out_n, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[mix(i) % out_n] = i;
}

// 11-14. the C2 value scan's exact access shape (dq_scan_fast.hip fast_load): each workgroup owns
//    a contiguous chunk addressed through its own buffer descriptors; per iteration a lane loads
//    4 x 16 B of values (2 rows each) and the validity BYTE of each pair (4 lanes share a byte, a
//    wave reads 16 contiguous validity bytes per instruction); iteration it + 1 is loaded while it
//    is consumed, so the last look-ahead falls past the chunk (range-checked to 0).  AUX is the
//    cache-policy operand (2 = non-temporal, as the scan uses for large passes).
typedef uint32_t pv4u __attribute__((ext_vector_type(4)));
template <int AUX, bool VALUES, bool VALID>
__global__ __launch_bounds__(256) void probe_scan_shape(const uint64_t* __restrict__ values, const uint8_t* __restrict__ valid,
                                                        uint64_t n_rows, uint32_t* sink) {
  const uint64_t per = n_rows / gridDim.x;  // host: n_rows % (gridDim.x * 2048) == 0
  const uint64_t r_begin = (uint64_t)blockIdx.x * per;
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(values + r_begin), 0, (int)(per * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(valid + r_begin / 8), 0, (int)(per / 8), 0x00020000);
  const uint32_t iters = (uint32_t)(per / 2048);
  uint32_t acc = 0;
  pv4u v[4];
  uint32_t b[4];
  auto load = [&](uint32_t it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t r0 = it * 2048u + ((uint32_t)u * 256u + threadIdx.x) * 2u;
      if (VALUES) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(r0 * 8u), 0, AUX);
      if (VALID) b[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rb, (int)(r0 >> 3), 0, AUX);
    }
  };
  load(0);
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (VALUES) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
      if (VALID) acc += b[u];
    }
    load(it + 1);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t GB = 1ull << 30;
  const uint64_t big = 2 * GB;
  uint8_t *a, *b, *t;
  uint32_t* sink;
  CHK(hipMalloc(&a, big));
  CHK(hipMalloc(&b, big));
  CHK(hipMalloc(&t, 4 * GB));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(a, 1, big));
  CHK(hipMemset(b, 2, big));
  CHK(hipMemset(t, 3, 4 * GB));
  CHK(hipDeviceSynchronize());
  const dim3 grid(256 * 8), block(256);
  auto fence = [&]() { CHK(hipDeviceSynchronize()); };
  auto line = [](const char* k, double rd, double wr, const char* shape, const char* kname = nullptr) {
    printf("{\"kernel\": \"%s\", \"kname\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"shape\": \"%s\"}\n", k,
           kname ? kname : k, rd, wr, shape);
  };
  // reads (each from a fresh half so no probe reads what the previous one left in the caches)
  probe_read_wide16<<<grid, block>>>((const uint4*)a, GB / 16, sink); fence();
  line("probe_read_wide16", (double)GB, 0, "16 B per lane, coalesced streaming");
  probe_read_b64<<<grid, block>>>((const uint64_t*)(a + GB), GB / 8, sink); fence();
  line("probe_read_b64", (double)GB, 0, "8 B per lane, coalesced streaming");
  probe_read_b32<<<grid, block>>>((const uint32_t*)b, GB / 4, sink); fence();
  line("probe_read_b32", (double)GB, 0, "4 B per lane, coalesced streaming");
  probe_read_64B_per_wave<<<grid, block>>>((const uint32_t*)(b + GB), GB / 4, sink); fence();
  line("probe_read_64B_per_wave", (double)GB, 0, "64 contiguous bytes per wave instruction (bitmap-shaped)");
  const uint64_t n_gather = 1ull << 26;
  probe_gather8<<<grid, block>>>((const uint64_t*)t, 4 * GB / 8, n_gather, sink); fence();
  line("probe_gather8", 8.0 * n_gather, 0, "random 8-B gathers from a 4 GiB table");
  // writes
  probe_write_wide16<<<grid, block>>>((uint4*)a, GB / 16); fence();
  line("probe_write_wide16", 0, (double)GB, "16 B per lane, coalesced streaming");
  probe_write_b64<<<grid, block>>>((uint64_t*)(a + GB), GB / 8); fence();
  line("probe_write_b64", 0, (double)GB, "8 B per lane, coalesced streaming");
  const uint64_t n_runs = (GB / 96);
  probe_write_runs96<<<grid, block>>>((uint64_t*)t, 4 * GB / 8, n_runs); fence();
  line("probe_write_runs96", 0, 96.0 * n_runs, "runs of 12 x 8 B at random 8-B-aligned positions");
  const uint64_t n_lines = GB / 128;
  probe_write_lines128<<<grid, block>>>((uint64_t*)b, big / 128, n_lines); fence();
  line("probe_write_lines128", 0, 128.0 * n_lines, "whole 128-B lines at random positions");
  const uint64_t n_scatter = 1ull << 26;
  probe_scatter8<<<grid, block>>>((uint64_t*)(t), 4 * GB / 8, n_scatter); fence();
  line("probe_scatter8", 0, 8.0 * n_scatter, "random 8-B stores into a 4 GiB buffer");
  // the scan's shape: 2^27 rows of 8-byte values (1 GiB) + their 16 MiB validity bitmap, 1024
  // workgroups; values in a, validity in b (fresh: the write probes left t / b / a behind, and the
  // values region alternates so no probe reads what the previous one touched)
  const uint64_t rows = 1ull << 27;
  const double vbytes = 8.0 * rows, bbytes = rows / 8.0;
  const dim3 sgrid(1024);
  probe_scan_shape<2, true, true><<<sgrid, block>>>((const uint64_t*)a, b, rows, sink); fence();
  line("probe_scan_shape_nt", vbytes + bbytes, 0, "the C2 scan's loads: 16 B values + 1 validity byte per lane, chunk descriptors, aux=nt", "probe_scan_shape<2, true, true>");
  probe_scan_shape<0, true, true><<<sgrid, block>>>((const uint64_t*)(a + GB), b + GB / 2, rows, sink); fence();
  line("probe_scan_shape_default", vbytes + bbytes, 0, "the same loads, default cache policy", "probe_scan_shape<0, true, true>");
  probe_scan_shape<2, true, false><<<sgrid, block>>>((const uint64_t*)t, nullptr, rows, sink); fence();
  line("probe_scan_values_nt", vbytes, 0, "the scan's value loads only, aux=nt", "probe_scan_shape<2, true, false>");
  probe_scan_shape<2, false, true><<<sgrid, block>>>(nullptr, t + 2 * GB, rows, sink); fence();
  line("probe_scan_validity_nt", 0 + bbytes, 0, "the scan's validity-byte loads only (16 B per wave instruction), aux=nt", "probe_scan_shape<2, false, true>");
  probe_scan_shape<0, false, true><<<sgrid, block>>>(nullptr, t + 3 * GB, rows, sink); fence();
  line("probe_scan_validity_default", 0 + bbytes, 0, "the scan's validity-byte loads only, default policy", "probe_scan_shape<0, false, true>");
  CHK(hipFree(a));
  CHK(hipFree(b));
  CHK(hipFree(t));
  CHK(hipFree(sink));
  return 0;
}
