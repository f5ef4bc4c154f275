// Memory probe 2 (not product code): non-temporal loads; byte-unaligned dwordx4 correctness/speed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <int FPW, int NI, int NBUF, bool NT>
__global__ __launch_bounds__(1024) void probe(const uint8_t* __restrict__ base, size_t stride, int shift, int nframes, uint32_t* out) {
  constexpr int LPF = 64 / FPW;
  const int lane = threadIdx.x & 63, col = lane % LPF, grp = lane / LPF;
  const int W = gridDim.x * (blockDim.x >> 6);
  const int w0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint32_t acc = 0;
  uint4 buf[NBUF][NI];
  auto load = [&](int wf, uint4 (&x)[NI]) {
    int f = min(wf * FPW + grp, nframes - 1);
    const uint8_t* fb = base + (size_t)f * stride + shift;
    #pragma unroll
    for (int j = 0; j < NI; j++) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4* p = (const u32x4*)(fb + 1024 / FPW * j + 16 * col);
      u32x4 v = NT ? __builtin_nontemporal_load(p) : *p;
      x[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  int wf = w0;
  #pragma unroll
  for (int b = 0; b < NBUF - 1; b++) load(wf + b * W, buf[b]);
  for (; wf * FPW < nframes; wf += NBUF * W) {
    #pragma unroll
    for (int b = 0; b < NBUF; b++) {
      load(wf + (b + NBUF - 1) * W, buf[(b + NBUF - 1) % NBUF]);
      #pragma unroll
      for (int j = 0; j < NI; j++) acc ^= buf[b][j].x ^ buf[b][j].y ^ buf[b][j].z ^ buf[b][j].w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void unaligned_check(const uint8_t* p, uint4* out) {
  int t = threadIdx.x;  // t = byte offset 0..63
  out[t] = *(const uint4*)(p + t);
}

int main() {
  const size_t BYTES = 1600ull * 1000000 + (1 << 20);
  uint8_t* d; CK(hipMalloc(&d, BYTES)); CK(hipMemset(d, 1, BYTES));
  uint32_t* o; CK(hipMalloc(&o, 1 << 24));
  // unaligned correctness
  std::vector<uint8_t> h(256); for (int i = 0; i < 256; i++) h[i] = (uint8_t)(i * 7 + 3);
  CK(hipMemcpy(d, h.data(), 256, hipMemcpyHostToDevice));
  unaligned_check<<<1, 64>>>(d, (uint4*)o); CK(hipDeviceSynchronize());
  std::vector<uint8_t> r(64 * 16); CK(hipMemcpy(r.data(), o, r.size(), hipMemcpyDeviceToHost));
  int bad = 0; for (int t = 0; t < 64; t++) for (int k = 0; k < 16; k++) if (r[t * 16 + k] != h[t + k]) bad++;
  printf("unaligned dwordx4 byte mismatches: %d\n", bad);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* nm, auto kern, size_t stride, int shift, int nframes, double bytes) {
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
    kern<<<256, 1024, 163840>>>(d, stride, shift, nframes, o); CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 15; r++) { CK(hipEventRecord(e0)); kern<<<256, 1024, 163840>>>(d, stride, shift, nframes, o); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms); }
    std::sort(ts.begin(), ts.end());
    printf("%-52s median %.3f ms  %.1f GB/s\n", nm, ts[7], bytes / ts[7] / 1e6); fflush(stdout);
  };
  const int N = 1000000;
  run("FPW4 NI6 s1500 nb2", probe<4, 6, 2, false>, 1500, 0, N, 1500.0 * N);
  run("FPW4 NI6 s1500 nb2 NT", probe<4, 6, 2, true>, 1500, 0, N, 1500.0 * N);
  run("FPW4 NI6 s1500 nb3 NT", probe<4, 6, 3, true>, 1500, 0, N, 1500.0 * N);
  run("FPW4 NI6 s1500 shift1 nb2", probe<4, 6, 2, false>, 1500, 1, N, 1500.0 * N);
  run("FPW4 NI6 s1500 shift2 nb2", probe<4, 6, 2, false>, 1500, 2, N, 1500.0 * N);
  run("FPW4 NI6 s1501 shift3 nb2", probe<4, 6, 2, false>, 1501, 3, N, 1501.0 * N);
  run("FPW4 NI6 s1500 shift1 nb2 NT", probe<4, 6, 2, true>, 1500, 1, N, 1500.0 * N);
  printf("done\n");
}
