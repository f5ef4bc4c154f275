// bsprobe.hip -- loads-only probe of byte-stream access patterns for config 3 (7.82 GB):
// each wave splits its contiguous byte range into G sub-ranges, one per lane group of 64/G lanes;
// per step a group reads 16 B per lane (1024/G contiguous, aligned bytes) of its own sub-range.
// G = 1 is the plain stream.  D steps in flight, WAVES waves per CU, one workgroup per CU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int G, int D, int WAVES, bool NT>
__global__ __launch_bounds__(WAVES * 64) void groups(const uint8_t* bytes, uint64_t nbytes, uint32_t* out) {
  constexpr int LPG = 64 / G;
  constexpr uint64_t STEP = 16 * LPG;
  const uint32_t lane = threadIdx.x & 63, g = lane / LPG, gl = lane % LPG;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t W = (uint64_t)gridDim.x * WAVES * G;
  const uint64_t w = ((uint64_t)blockIdx.x * WAVES + wid) * G + g;
  const uint64_t nsteps = nbytes / STEP;
  const uint64_t lo = nsteps * w / W, hi = nsteps * (w + 1) / W;
  const uint64_t nmax = (nsteps + W - 1) / W;  // wave-uniform loop count
  uint32_t acc = 0;
  u32x4 data[D];
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  const uint64_t lo0 = __builtin_amdgcn_readfirstlane((uint32_t)0);
  (void)lo0;
  for (uint64_t k = 0; k < nmax; k += D) {
#pragma unroll
    for (int s = 0; s < D; s++) {
      uint64_t kk = lo + k + s;
      kk = kk < hi ? kk : hi - 1;
      const u32x4* p = (const u32x4*)(bytes + kk * STEP + 16 * gl);
      const u32x4 v = NT ? __builtin_nontemporal_load(p) : *p;
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
    }
  }
  for (int i = 0; i < D; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint64_t total = 7816000000ull;
  uint8_t* bytes;
  uint32_t* out;
  if (hipMalloc(&bytes, total + 65536) != hipSuccess || hipMalloc(&out, 256 * 1024 * 4) != hipSuccess) return 1;
  (void)hipMemset(bytes, 0x3C, total + 65536);
  struct V {
    const char* name;
    void (*launch)(const uint8_t*, uint64_t, uint32_t*);
  };
#define GV(G_, D_, W_, NT_)                                                                    \
  {"G=" #G_ " D=" #D_ " waves=" #W_ " nt=" #NT_, [](const uint8_t* b, uint64_t t, uint32_t* o) { \
     hipLaunchKernelGGL((groups<G_, D_, W_, NT_>), dim3(256), dim3(W_ * 64), 0, 0, b, t, o);     \
   }}
  V vs[] = {GV(1, 4, 8, true),  GV(1, 4, 8, false), GV(2, 4, 8, true),  GV(4, 4, 8, true),  GV(4, 4, 8, false),
            GV(4, 2, 8, true),  GV(4, 3, 8, true),  GV(4, 6, 8, true),  GV(4, 4, 12, true), GV(4, 2, 12, true),
            GV(4, 4, 16, true), GV(4, 2, 16, true), GV(8, 4, 8, true),  GV(8, 2, 12, true), GV(2, 2, 12, true),
            GV(4, 3, 12, true)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 3; w++) v.launch(bytes, total, out);
      std::vector<float> t;
      for (int r = 0; r < 9; r++) {
        (void)hipEventRecord(e0, 0);
        v.launch(bytes, total, out);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
          printf("%s failed\n", v.name);
          return 1;
        }
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("round %d  %-30s median %.4f ms  %.2f TB/s\n", round, v.name, t[t.size() / 2],
             total / t[t.size() / 2] / 1e9);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
