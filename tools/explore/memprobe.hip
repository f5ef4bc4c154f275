// Memory-pattern probe (not product code): loads-only kernels shaped like the CRC kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// FPW frames per wave; each lane group (64/FPW lanes) reads RUN = 1024/FPW contiguous bytes per
// instruction from its frame; NI instructions per frame; frame f at base + f*stride + shift.
template <int FPW, int NI, int NBUF>
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
    for (int j = 0; j < NI; j++) x[j] = *(const uint4*)(fb + 1024 / FPW * j + 16 * col);
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

int main() {
  const size_t BYTES = 1600ull * 1000000 + (1 << 20);
  uint8_t* d; CK(hipMalloc(&d, BYTES)); CK(hipMemset(d, 1, BYTES));
  uint32_t* o; CK(hipMalloc(&o, 1 << 24));
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
  // W4-shaped: 4 frames/wave, 256-B runs, 6 instr/frame
  run("FPW4 NI6 stride1500 shift0 nb2", probe<4, 6, 2>, 1500, 0, N, 1536.0 * N);
  run("FPW4 NI6 stride1500 shift0 nb3", probe<4, 6, 3>, 1500, 0, N, 1536.0 * N);
  run("FPW4 NI6 stride1536 shift0 nb2 (aligned)", probe<4, 6, 2>, 1536, 0, N, 1536.0 * N);
  run("FPW4 NI6 stride1536 shift4 nb2", probe<4, 6, 2>, 1536, 4, N, 1536.0 * N);
  run("FPW4 NI6 stride1536 shift64 nb2", probe<4, 6, 2>, 1536, 64, N, 1536.0 * N);
  run("FPW2 NI3 stride1500 nb2 (512-B runs)", probe<2, 3, 2>, 1500, 0, N, 1536.0 * N);
  run("FPW2 NI3 stride1536 nb2 (512-B runs aligned)", probe<2, 3, 2>, 1536, 0, N, 1536.0 * N);
  run("FPW1 NI2 stride1500 nb2 (1KiB runs, 2048/frame)", probe<1, 2, 2>, 1500, 0, N, 2048.0 * N);
  run("FPW1 NI2 stride2048 nb2 (1KiB aligned)", probe<1, 2, 2>, 2048, 0, N * 3 / 4, 2048.0 * N * 3 / 4);
  run("FPW4 NI6 stride1500 nb4", probe<4, 6, 4>, 1500, 0, N, 1536.0 * N);
  run("FPW8 NI12 stride1500 nb2 (128-B runs)", probe<8, 12, 2>, 1500, 0, N, 1536.0 * N);
  printf("done\n");
}
