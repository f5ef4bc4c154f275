// scatterprobe.hip -- can the seal's 1M trailer writes leave the read stream? (tuning probe for the
// seal; not product code)
//
// Times, on config 2's 1M x 1500-B buffer:
//   A  the stream read alone (sealprobe's loads-only shape, crc words to a 4-MB array);
//   B  a scatter kernel alone: one thread per frame writes crc[i] (BE) at its trailer;
//   A+B back to back on one stream (the two-kernel seal), and the in-loop seal shape (sealprobe
//   mode 1) for comparison.
// Build: hipcc -O3 --offload-arch=gfx950 -o scatterprobe scatterprobe.hip ; run: ./scatterprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <functional>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

constexpr int L = 1500, J = 6, PAD = J * 256 - L;

template <bool SEAL_IN_LOOP>
__global__ __launch_bounds__(512) void stream(uint8_t* buf, uint32_t nframes, uint32_t* crc) {
  const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nsets = nframes / 4;
  const uint32_t lo = (uint64_t)nsets * blockIdx.x / gridDim.x, hi = (uint64_t)nsets * (blockIdx.x + 1) / gridDim.x;
  auto load = [&](uint32_t q, u32x4 (&x)[J]) {
    const uint32_t qc = q < hi ? q : (hi > lo ? hi - 1 : lo);
    int64_t off = (int64_t)(4 * (uint64_t)qc + grp) * L + 16 * col - PAD;
    off = off < 0 ? 0 : off;
#pragma unroll
    for (int j = 0; j < J; j++) x[j] = __builtin_nontemporal_load((g_u32x4*)(buf + off + 256 * j));
  };
  u32x4 A[J], B[J];
  uint32_t q = lo + wid;
  load(q, A);
  auto body = [&](uint32_t qq, u32x4 (&cur)[J], u32x4 (&nxt)[J]) {
    load(qq + 8, nxt);
    __builtin_amdgcn_sched_barrier(0);
    if (qq < hi) {
      uint32_t f = 0;
#pragma unroll
      for (int j = 0; j < J; j++) f ^= cur[j].x ^ cur[j].y ^ cur[j].z ^ cur[j].w;
      const uint64_t frame = 4 * (uint64_t)qq + grp;
      if (col == 15) {
        if (SEAL_IN_LOOP)
          *(uint32_t*)(buf + frame * L + L - 4) = f;
        else
          crc[frame] = f;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (; q < hi; q += 16) {
    body(q, A, B);
    body(q + 8, B, A);
  }
}

template <int POL>
__global__ __launch_bounds__(256) void scatter(uint8_t* buf, uint32_t nframes, const uint32_t* crc) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nframes) return;
  const uint32_t v = __builtin_bswap32(crc[i]);
  uint32_t* t = (uint32_t*)(buf + (uint64_t)i * L + L - 4);
  if (POL == 0) *t = v;
  if (POL == 1) __builtin_nontemporal_store(v, t);
}

int main() {
  const uint32_t n = 1000000;
  uint8_t* buf;
  uint32_t* crc;
  if (hipMalloc(&buf, (size_t)n * L + 4096) != hipSuccess || hipMalloc(&crc, (size_t)n * 4) != hipSuccess) return 1;
  hipMemset(buf, 0x5A, (size_t)n * L);
  hipMemset(crc, 0, (size_t)n * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned sg = (n + 255) / 256;
  auto A = [&] { hipLaunchKernelGGL(stream<false>, dim3(256), dim3(512), 0, 0, buf, n, crc); };
  auto S = [&] { hipLaunchKernelGGL(stream<true>, dim3(256), dim3(512), 0, 0, buf, n, crc); };
  auto B0 = [&] { hipLaunchKernelGGL(scatter<0>, dim3(sg), dim3(256), 0, 0, buf, n, crc); };
  auto B1 = [&] { hipLaunchKernelGGL(scatter<1>, dim3(sg), dim3(256), 0, 0, buf, n, crc); };
  struct V { const char* name; std::vector<std::function<void()>> ks; };
  std::vector<V> vs = {{"A: stream, crc to array", {A}},
                       {"B: scatter default", {B0}},
                       {"B: scatter nt", {B1}},
                       {"A+B default", {A, B0}},
                       {"A+B nt", {A, B1}},
                       {"in-loop seal", {S}}};
  for (int round = 0; round < 2; round++) {
    for (auto& v : vs) {
      for (int w = 0; w < 20; w++)
        for (auto& k : v.ks) k();
      std::vector<float> t;
      for (int r = 0; r < 30; r++) {
        hipEventRecord(e0, 0);
        for (auto& k : v.ks) k();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("round %d  %-26s median %.4f ms  min %.4f ms\n", round, v.name, t[t.size() / 2], t[0]);
    }
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
