// setorder.hip -- loads-only probe: does the ORDER in which a workgroup's waves take the sorted sets
// change what the variable-length gate's access pattern streams at?  Config 3's 10M frames of
// U[64,1500] B; each run of 64 consecutive frames is ordered by piece count on the host (as the
// kernel's in-kernel sort does) and cut into 8 sets of 8 frames; a set is read as 8 frames x 128-byte
// pieces per step (8 lanes per frame, 16 B per lane), right-aligned 4-byte windows, max P steps per
// set.  Records (window start, piece count) come precomputed, so only the order and the loads differ:
//   order 0 -- a workgroup owns a contiguous range of runs, wave w takes whole runs w, w + WAVES, ...
//              (the product kernel's shape: a CU's waves stream 12 runs ~600 KB apart);
//   order 2 -- wave w takes a contiguous range of the workgroup's runs (12 streams ~1/12 of the
//              workgroup's range apart);
//   order 1 -- the workgroup's waves take consecutive SETS: wave w takes sets w, w + WAVES, ... so
//              the 8 sets of a run are read at the same time by 8 waves (neighbouring frames' shared
//              lines close in time, the CU's reads within ~1.5 runs).
// Tuning probe, not product code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;

// rec[s * 8 + g] = (window start relative to the buffer | P << 28) of frame g of set s (P <= 15).
template <int D, int WAVES, int ORDER, int AUX>
__global__ __launch_bounds__(WAVES * 64) void sets(const uint8_t* bytes, const uint64_t* rec, uint32_t nsets,
                                                   uint32_t* out) {
  __shared__ char pad_lds[160 * 1024];
  const uint32_t lane = threadIdx.x & 63, c = lane & 7, g = lane >> 3;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nruns = nsets / 8;
  const uint32_t R0 = (uint64_t)nruns * blockIdx.x / gridDim.x, R1 = (uint64_t)nruns * (blockIdx.x + 1) / gridDim.x;
  const uint32_t S0 = R0 * 8, S1 = R1 * 8;
  // this wave's k-th set
  auto set_of = [&](uint32_t k) -> uint32_t {
    if (ORDER == 0) {
      const uint32_t run = R0 + wid + WAVES * (k / 8);
      return run < R1 ? run * 8 + (k & 7) : 0xFFFFFFFFu;
    }
    if (ORDER == 2) {  // wave-contiguous run ranges inside the workgroup's range
      const uint32_t a = R0 + (uint32_t)((uint64_t)(R1 - R0) * wid / WAVES);
      const uint32_t b = R0 + (uint32_t)((uint64_t)(R1 - R0) * (wid + 1) / WAVES);
      const uint32_t run = a + k / 8;
      return run < b ? run * 8 + (k & 7) : 0xFFFFFFFFu;
    }
    const uint32_t s = S0 + wid + WAVES * k;
    return s < S1 ? s : 0xFFFFFFFFu;
  };
  uint32_t acc = pad_lds[threadIdx.x];
  uint32_t k = 0, s = set_of(0), j = 0, P = 0, ws = 0, Pg = 0;
  bool live = s != 0xFFFFFFFFu;
  auto take = [&]() {
    const uint64_t r = live ? rec[(uint64_t)s * 8 + g] : 0;
    ws = (uint32_t)r;
    Pg = (uint32_t)(r >> 32);
    uint32_t mx = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) mx = max(mx, (uint32_t)__builtin_amdgcn_readlane((int)Pg, 8 * q));
    P = mx ? mx : 1;
  };
  if (live) take();
  u32x4 data[D];
#pragma unroll
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)bytes, 0, 0x7FFFFFF0, 0x00020000);
  while (__builtin_amdgcn_readfirstlane((int)live)) {
#pragma unroll
    for (int st = 0; st < D; st++) {
      if (j >= P) {
        j = 0;
        k++;
        s = set_of(k);
        live = s != 0xFFFFFFFFu;
        if (live) take();
      }
      const uint32_t voff = (live && j < Pg) ? ws + 128u * j + 16u * c : kOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs0, (int)voff, 0, AUX);
      acc ^= data[st].x ^ data[st].y ^ data[st].z ^ data[st].w;
      data[st] = v;
      j++;
    }
  }
#pragma unroll
  for (int i = 0; i < D; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint32_t n = 10000000;  // (< 2 GB of frames: 32-bit window starts)
  std::vector<uint64_t> off(n + 1, 0);
  uint64_t x = 0x5EED0002;
  for (uint32_t i = 0; i < n; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    off[i + 1] = off[i] + 64 + (x >> 33) % 1437;
  }
  const uint64_t total = off[n];
  // The first 2^31 - 4096 bytes' runs only (32-bit relative window starts).
  uint32_t nruns = 0;
  while ((uint64_t)(nruns + 1) * 64 <= n && off[(nruns + 1) * 64] < (1ull << 31) - 4096) nruns++;
  std::vector<uint64_t> rec((size_t)nruns * 64);
  for (uint32_t r = 0; r < nruns; r++) {
    uint32_t idx[64], P[64], ws[64];
    for (uint32_t i = 0; i < 64; i++) {
      const uint64_t a = off[r * 64 + i] + 4096, b = off[r * 64 + i + 1] + 4096;  // (4 KB in front)
      const uint64_t we = (b + 3) & ~3ull;
      const uint64_t w0 = we - ((we - (a - 4) + 127) & ~127ull);
      ws[i] = (uint32_t)w0;
      P[i] = (uint32_t)((we - w0) / 128);
      idx[i] = i;
    }
    std::stable_sort(idx, idx + 64, [&](uint32_t p, uint32_t q) { return P[p] < P[q]; });
    for (uint32_t i = 0; i < 64; i++) rec[(size_t)r * 64 + i] = (uint64_t)ws[idx[i]] | ((uint64_t)P[idx[i]] << 32);
  }
  const uint64_t used = off[nruns * 64];
  uint8_t* bytes;
  uint64_t* drec;
  uint32_t* out;
  if (hipMalloc(&bytes, used + 8192 + 4096) != hipSuccess || hipMalloc(&drec, rec.size() * 8) != hipSuccess ||
      hipMalloc(&out, 256 * 1024 * 4) != hipSuccess)
    return 1;
  (void)hipMemset(bytes, 0x3C, used + 8192 + 4096);
  (void)hipMemcpy(drec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice);
  const uint32_t nsets = nruns * 8;
  printf("set-order probe: %u runs, %.3f GB of frames\n", nruns, used / 1e9);
  struct V {
    const char* name;
    void (*launch)(const uint8_t*, const uint64_t*, uint32_t, uint32_t*);
  };
#define SV(D_, W_, O_, A_) {"sets D=" #D_ " waves=" #W_ " order=" #O_ " aux=" #A_, \
    [](const uint8_t* b, const uint64_t* r, uint32_t ns, uint32_t* ou) { \
      hipLaunchKernelGGL((sets<D_, W_, O_, A_>), dim3(256), dim3(W_ * 64), 0, 0, b, r, ns, ou); }}
  V vs[] = {SV(6, 12, 0, 0), SV(6, 12, 2, 0), SV(6, 12, 1, 0), SV(8, 8, 0, 0), SV(8, 8, 2, 0), SV(4, 12, 2, 0),
            SV(6, 12, 2, 2)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 3; w++) v.launch(bytes, drec, nsets, out);
      std::vector<float> t;
      for (int r = 0; r < 9; r++) {
        (void)hipEventRecord(e0, 0);
        v.launch(bytes, drec, nsets, out);
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
      printf("round %d  %-36s median %.4f ms  %.2f TB/s\n", round, v.name, t[t.size() / 2], used / t[t.size() / 2] / 1e9);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
