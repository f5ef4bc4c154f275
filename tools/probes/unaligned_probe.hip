// unaligned_probe.hip -- do unaligned global loads of 8 and 16 bytes return the bytes at their address?
// (correctness probe for the parse walk's frame-head load; not product code)
//
// Over a 64 MB buffer of known bytes, every thread loads at offset 17 * tid + (tid % 61) (every
// alignment, crossing 64-B, 128-B and 4-KB boundaries) with global_load_dwordx2, global_load_dwordx4
// and buffer_load_dwordx4 (raw buffer, unaligned offset), and compares each with byte loads.
// Prints the number of mismatching loads per kind and the first few; exits non-zero on any.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1), aligned(1))) uint64_t g_u64_a1;
typedef const __attribute__((address_space(1), aligned(1))) u32x4 g_u32x4_a1;

__global__ void probe(const uint8_t* buf, uint64_t nbytes, uint32_t n, uint32_t* bad, uint32_t* first) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t off = (uint64_t)t * 17 + t % 61;
  if (off + 16 > nbytes) return;
  const uint8_t* q = buf + off;
  uint8_t ref[16];
  for (int k = 0; k < 16; k++) ref[k] = *(const volatile uint8_t*)(q + k);
  const uint64_t w = *(g_u64_a1*)q;
  const u32x4 v = *(g_u32x4_a1*)q;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, 0x7FFFFFF0, 0x00020000);
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  bool ok8 = true, ok16 = true, okb = true;
  for (int k = 0; k < 16; k++) {
    const uint32_t vk = (k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w) >> (8 * (k & 3)) & 0xFF;
    const uint32_t bk = (k < 4 ? b.x : k < 8 ? b.y : k < 12 ? b.z : b.w) >> (8 * (k & 3)) & 0xFF;
    if (k < 8 && ((w >> (8 * k)) & 0xFF) != ref[k]) ok8 = false;
    if (vk != ref[k]) ok16 = false;
    if (bk != ref[k]) okb = false;
  }
  if (!ok8 && atomicAdd(&bad[0], 1u) < 4) atomicExch(&first[0 + (bad[0] & 3)], (uint32_t)off);
  if (!ok16 && atomicAdd(&bad[1], 1u) < 4) atomicExch(&first[4 + (bad[1] & 3)], (uint32_t)off);
  if (!okb && atomicAdd(&bad[2], 1u) < 4) atomicExch(&first[8 + (bad[2] & 3)], (uint32_t)off);
}

__global__ void fill(uint8_t* buf, uint64_t nbytes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nbytes) buf[i] = (uint8_t)((i * 2654435761u) >> 13);
}

int main() {
  const uint64_t nbytes = 64ull << 20;
  const uint32_t n = (uint32_t)(nbytes / 17) - 8;
  uint8_t* buf;
  uint32_t *bad, *first;
  if (hipMalloc(&buf, nbytes) != hipSuccess || hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 64) != hipSuccess)
    return 1;
  (void)hipMemset(bad, 0, 16);
  (void)hipMemset(first, 0, 64);
  hipLaunchKernelGGL(fill, dim3((unsigned)((nbytes + 255) / 256)), dim3(256), 0, 0, buf, nbytes);
  hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, buf, nbytes, n, bad, first);
  uint32_t hb[4], hf[16];
  if (hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hf, first, 64, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  printf("loads %u: mismatches global dwordx2 %u, global dwordx4 %u, buffer dwordx4 %u\n", n, hb[0], hb[1], hb[2]);
  for (int k = 0; k < 3; k++)
    if (hb[k]) printf("  kind %d: e.g. offsets %u %u %u %u (mod 16: %u %u %u %u)\n", k, hf[4 * k], hf[4 * k + 1],
                      hf[4 * k + 2], hf[4 * k + 3], hf[4 * k] % 16, hf[4 * k + 1] % 16, hf[4 * k + 2] % 16, hf[4 * k + 3] % 16);
  return (hb[0] || hb[1] || hb[2]) ? 1 : 0;
}
