// struct_buf_probe.hip -- range checking of structured buffer loads on gfx950 (tuning probe, not
// product code): a resource with stride 128 and num_records N; loads with index i and voffset v
// (v larger than the stride, and indices past N and "negative" ones; every case addresses memory
// inside the allocation even if it were not range-checked).  Prints, per case, whether the
// load returned the bytes at base + i * 128 + v or zeros.
// Build: hipcc -O3 --offload-arch=gfx950 -o struct_buf_probe struct_buf_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 sbl(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.ptr.buffer.load.v4i32");

__global__ void probe(const uint32_t* base, const int* idx, const int* off, uint32_t* out, int n, int nrec) {
  const int t = threadIdx.x;
  if (t >= n) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 128, nrec, 0x00020000);
  const u32x4 v = sbl(rs, idx[t], off[t], 0, 0);
  out[t] = v.x;
}

int main() {
  const int words = 1 << 22;  // 16 MB of words w[i] = i
  std::vector<uint32_t> h(words);
  for (int i = 0; i < words; i++) h[i] = (uint32_t)i;
  const int nrec = 1000;
  const int cases[][2] = {{0, 0},        {1, 0},     {5, 16},    {0, 200},   {3, 1000},   {10, 65536}, {999, 0},
                          {999, 4096},   {1000, 0},  {1001, 0},  {-1, 128},  {-1, 4096},  {-12, 65536}, {2, 1 << 20},
                          {0, 0x7FFFF0}, {-2, 256}};
  const int n = sizeof(cases) / sizeof(cases[0]);
  std::vector<int> hi(n), ho(n);
  for (int i = 0; i < n; i++) hi[i] = cases[i][0], ho[i] = cases[i][1];
  uint32_t *d, *o;
  int *di, *dof;
  if (hipMalloc(&d, words * 4) || hipMalloc(&o, n * 4) || hipMalloc(&di, n * 4) || hipMalloc(&dof, n * 4)) return 1;
  (void)hipMemcpy(d, h.data(), words * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(di, hi.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dof, ho.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, di, dof, o, n, nrec);
  std::vector<uint32_t> r(n);
  if (hipMemcpy(r.data(), o, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int i = 0; i < n; i++) {
    const int64_t byte = (int64_t)hi[i] * 128 + ho[i];
    const uint32_t expect = (byte >= 0 && byte / 4 < words) ? (uint32_t)(byte / 4) : 0xDEADu;
    printf("index %6d voffset %8d -> %10u (%s)\n", hi[i], ho[i], r[i],
           r[i] == expect ? "data" : (r[i] == 0 ? "zero" : "other"));
  }
  return 0;
}
