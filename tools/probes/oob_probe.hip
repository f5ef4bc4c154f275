// oob_probe.hip -- how a raw buffer dwordx4 load that straddles num_records is range-checked on
// gfx950: per dword (the in-range dwords come back) or per instruction (all four are zero)?
// Buffer of 64 bytes = 0x01.., resource with 20 records; loads at offsets 0, 4, 8, 12, 16, 20.
// Tuning probe, not product code.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t* buf, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, 20, 0x00020000);
  const int t = threadIdx.x;
  if (t < 6) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * t, 0, 0);
    out[4 * t + 0] = v.x;
    out[4 * t + 1] = v.y;
    out[4 * t + 2] = v.z;
    out[4 * t + 3] = v.w;
  }
}

int main() {
  uint8_t h[64];
  for (int i = 0; i < 64; i++) h[i] = (uint8_t)(i + 1);
  uint8_t* d;
  uint32_t* o;
  if (hipMalloc(&d, 64) != hipSuccess || hipMalloc(&o, 96) != hipSuccess) return 1;
  (void)hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(d, o);
  uint32_t r[24];
  if (hipMemcpy(r, o, 96, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int t = 0; t < 6; t++)
    printf("offset %2d: %08x %08x %08x %08x\n", 4 * t, r[4 * t], r[4 * t + 1], r[4 * t + 2], r[4 * t + 3]);
  return 0;
}
