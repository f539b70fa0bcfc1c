// Does a raw buffer load of 16 bytes at an arbitrary byte offset return those 16 bytes on gfx950
// (SH_MEM_CONFIG unaligned mode)?  And out-of-range bytes: zero?  Checks every offset 0..4095 of a
// buffer of i & 255 bytes, with the descriptor's size cut at 4000 bytes.  Measured on MI355X
// (round 4): every byte of a dword wholly in range is right; out-of-range bytes read 0; and a dword
// that straddles the end reads 0 WHOLE (24 in-range bytes lost at t = 3985..3999) -- the range
// check is per dword, so the kernels read a key within 16 bytes of the heap end word by word.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(const uint8_t* buf, uint32_t size, uint32_t* bad, uint32_t* oob_bad) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 4096) return;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(buf), 0, (int)size, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)t, 0, 0);
  for (int i = 0; i < 16; ++i) {
    const uint8_t got = (uint8_t)(v[i / 4] >> (8 * (i % 4)));
    const uint32_t at = t + i;
    const uint32_t dw_end = t + 4 * (i / 4) + 4;  // end of the dword this byte arrives in
    if (dw_end <= size) {
      if (got != (uint8_t)(at & 255)) atomicAdd(bad, 1u);
    } else if (at < size) {
      // straddling dword: zero (reported, not an error)
    } else if (got != 0) {
      atomicAdd(oob_bad, 1u);
    }
  }
}

int main() {
  uint8_t* d;
  uint32_t* c;
  uint8_t h[8192];
  for (int i = 0; i < 8192; ++i) h[i] = (uint8_t)i;
  hipMalloc(&d, 8192);
  hipMalloc(&c, 8);
  hipMemcpy(d, h, 8192, hipMemcpyHostToDevice);
  hipMemset(c, 0, 8);
  probe<<<16, 256>>>(d, 4000, c, c + 1);
  uint32_t r[2];
  hipMemcpy(r, c, 8, hipMemcpyDeviceToHost);
  std::printf("unaligned b128 buffer loads: mismatches in whole in-range dwords %u, nonzero out of range %u\n", r[0], r[1]);
  return r[0] != 0;
}
