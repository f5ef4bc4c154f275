// sealprobe.hip -- what does writing each frame's 4-byte trailer cost next to a 1.5 GB stream read?
// (tuning probe for the seal kernel; not product code)
//
// The lean kernel's access pattern (4 frames of 1500 B per wave step, 16 lanes per frame, six
// 16-B non-temporal loads per lane, 2 sets in flight, 8 waves per CU, static interleaved sets),
// the data XOR-folded, plus one write variant per frame at its trailer address:
//   0 none; 1 the 4-B trailer (dword); 2 the 32-B aligned sector holding it (2 lanes x 16 B);
//   3 the 64-B aligned segment (4 lanes); 4 the 128-B line (8 lanes);
//   5 = 1 but every store after the loop (the round-1 seal kernel's shape).
// Build: hipcc -O3 --offload-arch=gfx950 -o sealprobe sealprobe.hip ; run: ./sealprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

constexpr int L = 1500, J = 6, PAD = J * 256 - L;

template <int POL>
__device__ __forceinline__ void st4(uint8_t* a, uint32_t v) {
  if (POL == 0) asm volatile("global_store_dword %0, %1, off" ::"v"(a), "v"(v));
  if (POL == 1) asm volatile("global_store_dword %0, %1, off nt" ::"v"(a), "v"(v));
  if (POL == 2) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(a), "v"(v));
  if (POL == 3) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(a), "v"(v));
  if (POL == 4) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(a), "v"(v));
  if (POL == 5) asm volatile("global_store_dword %0, %1, off sc0" ::"v"(a), "v"(v));
}
__device__ __forceinline__ void st16(uint8_t* a, uint32_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(a), "v"((u32x4){v, v, v, v}));
}

template <int MODE, int POL, bool NTLOAD>
__global__ __launch_bounds__(512) void probe(uint8_t* buf, uint32_t nframes, uint32_t* out) {
  const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nsets = nframes / 4;
  const uint32_t lo = (uint64_t)nsets * blockIdx.x / gridDim.x, hi = (uint64_t)nsets * (blockIdx.x + 1) / gridDim.x;
  uint32_t acc = 0;
  uint8_t* pend[64];
  uint32_t npend = 0;
  auto load = [&](uint32_t q, u32x4 (&x)[J]) {
    const uint32_t qc = q < hi ? q : (hi > lo ? hi - 1 : lo);
    int64_t off = (int64_t)(4 * (uint64_t)qc + grp) * L + 16 * col - PAD;
    off = off < 0 ? 0 : off;
#pragma unroll
    for (int j = 0; j < J; j++)
      x[j] = NTLOAD ? __builtin_nontemporal_load((g_u32x4*)(buf + off + 256 * j)) : *(g_u32x4*)(buf + off + 256 * j);
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
      acc ^= f;
      const uint64_t frame = 4 * (uint64_t)qq + grp;
      uint8_t* tr = buf + frame * L + L - 4;  // the trailer
      if (MODE == 1 && col == 15) st4<POL>(tr, f);
      if (MODE == 5 && col == 15 && npend < 64) pend[npend++] = tr;
      if (MODE >= 2 && MODE <= 4) {
        const int span = MODE == 2 ? 32 : MODE == 3 ? 64 : 128;
        uint8_t* s = (uint8_t*)((uintptr_t)tr & ~(uintptr_t)(span - 1));
        if (col < span / 16) st16(s + 16 * col, f);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (; q < hi; q += 16) {
    body(q, A, B);
    body(q + 8, B, A);
  }
  if (MODE == 5)
    for (uint32_t i = 0; i < npend; i++) st4<POL>(pend[i], acc);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint32_t n = 1000000;
  uint8_t* buf;
  uint32_t* out;
  if (hipMalloc(&buf, (size_t)n * L + 4096) != hipSuccess || hipMalloc(&out, 256 * 512 * 4) != hipSuccess) return 1;
  hipMemset(buf, 0x5A, (size_t)n * L);
  struct V { void (*k)(uint8_t*, uint32_t, uint32_t*); const char* name; };
  V vs[] = {{probe<0, 0, true>, "loads only (nt)"},
            {probe<0, 0, false>, "loads only (default)"},
            {probe<1, 0, true>, "4B in loop, store default"},
            {probe<1, 1, true>, "4B in loop, store nt"},
            {probe<1, 2, true>, "4B in loop, store sc0 sc1"},
            {probe<1, 3, true>, "4B in loop, store sc1"},
            {probe<1, 4, true>, "4B in loop, store sc0sc1nt"},
            {probe<1, 5, true>, "4B in loop, store sc0"},
            {probe<1, 0, false>, "4B in loop, dflt ld+st"},
            {probe<1, 1, false>, "4B in loop, dflt ld, nt st"},
            {probe<3, 0, true>, "64B in loop"},
            {probe<5, 0, true>, "4B after loop"},
            {probe<5, 1, true>, "4B after loop, nt"},
            {probe<5, 2, true>, "4B after loop, sc0 sc1"}};
  const int NV = sizeof(vs) / sizeof(vs[0]);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int round = 0; round < 2; round++) {
    for (int m = 0; m < NV; m++) {
      for (int w = 0; w < 20; w++) hipLaunchKernelGGL(vs[m].k, dim3(256), dim3(512), 0, 0, buf, n, out);
      std::vector<float> t;
      for (int r = 0; r < 30; r++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(vs[m].k, dim3(256), dim3(512), 0, 0, buf, n, out);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("round %d  %-28s median %.4f ms  min %.4f ms\n", round, vs[m].name, t[t.size() / 2], t[0]);
    }
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
