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
  auto line = [](const char* k, double rd, double wr, const char* shape) {
    printf("{\"kernel\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"shape\": \"%s\"}\n", k, rd, wr, shape);
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
  CHK(hipFree(a));
  CHK(hipFree(b));
  CHK(hipFree(t));
  CHK(hipFree(sink));
  return 0;
}
