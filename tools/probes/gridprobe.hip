// gridprobe.hip -- loads-only probe for a block-grid streaming layout of the variable-length gate
// (config 3: 10M frames of U[64,1500] B, 7.8 GB, CSR).  Tuning probe, not product code.
//
// Pattern "gstream<G, P, D, WAVES, AUX>": the batch's bytes are cut at the global 256-byte grid
// into one contiguous block range per G-lane group of the grid (64 / G groups per wave).  A group
// reads its range in order, one 256-byte block per step: lane c loads the 16 bytes at
// 16 c + 16 G h for h < P (G * P * 16 = 256).  So every load instruction reads 64 / G whole
// 256-byte blocks (every byte once, no refetch) from 64 / G independent streams.  D steps in flight.
// Pattern "stream": the same bytes as one contiguous stream per wave (1 KB per instruction).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;

template <int G, int P, int D, int WAVES, int AUX>
__global__ __launch_bounds__(WAVES * 64) void gstream(const uint8_t* bytes, uint64_t nbytes, uint32_t* out) {
  static_assert(G * P * 16 == 256, "one 256-byte block per group step");
  constexpr int NGW = 64 / G;
  __shared__ char pad_lds[160 * 1024];  // one workgroup per CU, as the real kernel
  const uint32_t lane = threadIdx.x & 63, c = lane % G, g = lane / G;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t W = (uint64_t)gridDim.x * WAVES, w = (uint64_t)blockIdx.x * WAVES + wid;
  const uint64_t NG = W * NGW, gi = w * NGW + g;
  const uint64_t nblk = nbytes / 256;
  const uint64_t lo = nblk * gi / NG, hi = nblk * (gi + 1) / NG;
  const uint64_t wlo = nblk * (w * NGW) / NG;  // the wave's first block (resource base)
  const uint32_t nb = (uint32_t)(hi - lo), rel0 = (uint32_t)(lo - wlo) * 256u + 16u * c;
  const uint32_t nmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)((nblk * (w * NGW + NGW) / NG - wlo + NGW - 1) / NGW + 1));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + wlo * 256), 0, 0x7FFFFFF0, 0x00020000);
  uint32_t acc = pad_lds[threadIdx.x];
  u32x4 data[D][P];
#pragma unroll
  for (int i = 0; i < D; i++)
#pragma unroll
    for (int h = 0; h < P; h++) data[i][h] = (u32x4){0, 0, 0, 0};
  for (uint32_t k = 0; k < nmax; k += D) {
#pragma unroll
    for (int s = 0; s < D; s++) {
      const uint32_t kk = k + s;
      const uint32_t vo = kk < nb ? rel0 + 256u * kk : kOob;
#pragma unroll
      for (int h = 0; h < P; h++) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vo + 16u * G * h), 0, AUX);
        acc ^= data[s][h].x ^ data[s][h].y ^ data[s][h].z ^ data[s][h].w;
        data[s][h] = v;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < D; i++)
#pragma unroll
    for (int h = 0; h < P; h++) acc ^= data[i][h].x ^ data[i][h].y ^ data[i][h].z ^ data[i][h].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int D, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void stream(const uint8_t* bytes, uint64_t nbytes, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint64_t nchunks = nbytes / 1024;  // 1 KB per wave step
  const uint64_t lo = nchunks * w / W, hi = nchunks * (w + 1) / W;
  uint32_t acc = 0;
  u32x4 data[D];
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  for (uint64_t k = lo; k < hi; k += D) {
#pragma unroll
    for (int s = 0; s < D; s++) {
      const uint64_t kk = min(k + s, hi - 1);
      const u32x4 v = __builtin_nontemporal_load((const u32x4*)(bytes + kk * 1024 + 16 * lane));
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
    }
  }
  for (int i = 0; i < D; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint32_t n = 10000000;
  std::vector<uint64_t> off(n + 1, 0);
  uint64_t x = 0x5EED0002;
  for (uint32_t i = 0; i < n; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    off[i + 1] = off[i] + 64 + (x >> 33) % 1437;
  }
  const uint64_t total = off[n];
  uint8_t* bytes;
  uint32_t* out;
  if (hipMalloc(&bytes, total + 8192) != hipSuccess || hipMalloc(&out, 256 * 1024 * 4) != hipSuccess) return 1;
  (void)hipMemset(bytes, 0x3C, total + 8192);
  printf("grid probe: %.3f GB\n", total / 1e9);
  struct V {
    const char* name;
    int waves;
    void (*launch)(const uint8_t*, uint64_t, uint32_t*);
  };
#define GS(G_, P_, D_, W_, A_) {"gstream G=" #G_ " P=" #P_ " D=" #D_ " waves=" #W_ " aux=" #A_, W_, \
    [](const uint8_t* b, uint64_t nb, uint32_t* ou) { \
      hipLaunchKernelGGL((gstream<G_, P_, D_, W_, A_>), dim3(256), dim3(W_ * 64), 0, 0, b, nb, ou); }}
#define SV(D_, W_) {"stream D=" #D_ " waves=" #W_, W_, \
    [](const uint8_t* b, uint64_t nb, uint32_t* ou) { \
      hipLaunchKernelGGL((stream<D_, W_>), dim3(256), dim3(W_ * 64), 0, 0, b, nb, ou); }}
  V vs[] = {SV(4, 8),
            GS(16, 1, 4, 8, 0), GS(16, 1, 8, 8, 0), GS(16, 1, 4, 12, 0), GS(16, 1, 4, 8, 2),
            GS(8, 2, 2, 8, 0), GS(8, 2, 4, 8, 0), GS(8, 2, 2, 12, 0), GS(8, 2, 3, 12, 0), GS(8, 2, 2, 16, 0),
            GS(8, 2, 4, 8, 2), GS(8, 2, 2, 12, 2),
            GS(4, 4, 2, 8, 0), GS(4, 4, 2, 12, 0)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 5; w++) v.launch(bytes, total, out);
      std::vector<float> t;
      for (int r = 0; r < 15; r++) {
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
      printf("round %d  %-44s median %.4f ms  %.2f TB/s\n", round, v.name, t[t.size() / 2], total / t[t.size() / 2] / 1e9);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
