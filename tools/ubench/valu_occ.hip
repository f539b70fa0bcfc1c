// valu_occ.hip -- how the gfx950 SIMD's VALU issue rate depends on occupancy (waves per SIMD)
// and per-wave instruction-level parallelism (independent dependency chains), for a full-rate
// op (v_add_u32), a half-rate op (v_alignbit_b32), the multiply pair of the XXH64 kernels
// (v_mad_u64_u32, v_mul_lo_u32) and a dependent mul_lo -> mad -> add chain.
// Output: cycles per wave-instruction per SIMD = elapsed cycles * SIMDs / wave-instructions.
// Build: hipcc -O3 --offload-arch=gfx950 valu_occ.hip -o valu_occ
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kIters = 4096;

template <int OP> __device__ inline void step(uint32_t& a, uint32_t b, uint32_t c, uint64_t& w) {
  if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
  else if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 3) {
    uint64_t cc;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w), "=s"(cc) : "v"(a), "v"(b));
  } else if constexpr (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(c));
  else if constexpr (OP == 5) asm volatile("v_add_f64 %0, %0, %1" : "+v"(w) : "v"((uint64_t)b));
}

template <int OP, int C>
__global__ __launch_bounds__(256) void k_occ(unsigned long long* cyc, uint32_t* sink, uint32_t seed) {
  uint32_t a[C];
  uint64_t w[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    a[k] = threadIdx.x ^ (seed + k);
    w[k] = a[k] * 0x9e3779b97f4a7c15ull;
  }
  const uint32_t b = seed * 3u + 0x9e3779b9u, c = seed + 12345u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < 32 / C; ++u) {
#pragma unroll
      for (int k = 0; k < C; ++k) step<OP>(a[k], b, c, w[k]);
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < C; ++k) r ^= a[k] ^ (uint32_t)w[k];
  if (r == 0x5a5a5a5au) sink[0] = r;
}

typedef void (*Fn)(unsigned long long*, uint32_t*, uint32_t);

template <int OP>
static void run_op(const char* name, int cus, unsigned long long* d_cyc, uint32_t* d_sink) {
  const Fn fns[4] = {k_occ<OP, 1>, k_occ<OP, 2>, k_occ<OP, 4>, k_occ<OP, 8>};
  const int chains[4] = {1, 2, 4, 8};
  std::vector<unsigned long long> cyc(cus * 8);
  for (int ci = 0; ci < 4; ++ci) {
    for (int wps : {1, 2, 4, 6, 8}) {  // waves per SIMD = blocks per CU (4 waves per block)
      const int blocks = cus * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(fns[ci], dim3(blocks), dim3(256), 0, 0, d_cyc, d_sink, 7u + rep);
        CHK(hipDeviceSynchronize());
      }
      CHK(hipMemcpy(cyc.data(), d_cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
      std::sort(cyc.begin(), cyc.begin() + blocks);
      const double med = (double)cyc[blocks / 2];
      // each wave issued kIters * 32 instructions; wps waves share the SIMD over `med` cycles
      const double cpi = med / ((double)kIters * 32.0 * wps);
      printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cyc_per_insn_per_simd\": %.3f}\n", name,
             chains[ci], wps, cpi);
    }
  }
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  unsigned long long* d_cyc;
  uint32_t* d_sink;
  CHK(hipMalloc(&d_cyc, sizeof(unsigned long long) * cus * 8));
  CHK(hipMalloc(&d_sink, 64));
  run_op<0>("v_add_u32", cus, d_cyc, d_sink);
  run_op<4>("v_xor_b32", cus, d_cyc, d_sink);
  run_op<1>("v_alignbit_b32", cus, d_cyc, d_sink);
  run_op<2>("v_mul_lo_u32", cus, d_cyc, d_sink);
  run_op<3>("v_mad_u64_u32", cus, d_cyc, d_sink);
  run_op<5>("v_add_f64", cus, d_cyc, d_sink);
  return 0;
}
