// v8probe.hip -- loads-only probe of the 8-lanes-per-frame variable-length access pattern (config 3:
// 10M frames of U[64,1500] B, 7.8 GB) with right-aligned 4-byte-aligned windows (the product
// varlen8 kernel's) against 128-byte-aligned windows, sorted or unsorted sets.  A wave owns a
// contiguous frame range, walks it in runs of 64 frames (optionally ordered by piece count P, ballot
// ranks), sets of 8 frames, 8 lanes per frame, one 16-B load per lane per step = one 128-B piece of
// each of the set's frames; a set takes max P steps (pieces past a frame's own P load nothing).
// D steps in flight.  Tuning probe, not product code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;

template <int D, int WAVES, bool SORT, bool ALIGN, int AUX>
__global__ __launch_bounds__(WAVES * 64) void v8(const uint8_t* bytes, const uint64_t* offsets, uint32_t nframes,
                                                 uint32_t* out) {
  __shared__ char pad_lds[160 * 1024];
  const uint32_t lane = threadIdx.x & 63, c = lane & 7, g = lane >> 3;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint32_t F0 = (uint64_t)nframes * w / W, F1 = (uint64_t)nframes * (w + 1) / W;
  const uint64_t b0 = offsets[F0] & ~127ull;
  const uint8_t* base = bytes + b0 - 256;
  auto rel = [&](uint64_t x) -> uint32_t { return (uint32_t)(x - b0 + 256); };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
  uint32_t acc = pad_lds[threadIdx.x];
  uint32_t win = F0 - 64, k = 8, j = 0, P = 0;
  uint32_t s_ws = 0, s_P = 0, ws_g = 0, Pg = 0, live = 1;
  u32x4 data[D];
#pragma unroll
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  bool done = false;
  while (!done) {
#pragma unroll
    for (int s = 0; s < D; s++) {
      if (j >= P) {
        k++;
        j = 0;
        if (k >= 8) {  // next run of 64 frames
          win += 64;
          k = 0;
          const uint32_t nwin = win < F1 ? min(64u, F1 - win) : 0u;
          const uint32_t a = rel(offsets[min(win + lane, F1)]), b = rel(offsets[min(win + lane + 1, F1)]);
          uint32_t ws, we;
          if (ALIGN) {
            ws = (a - 4) & ~127u;
            we = (b + 127) & ~127u;
          } else {
            we = (b + 3) & ~3u;
            ws = we - ((we - (a - 4) + 127) & ~127u);
          }
          const uint32_t Pl = (we - ws) / 128;
          const uint32_t key = lane < nwin ? min(Pl, 15u) : 16u;
          uint32_t rank = lane;
          if (SORT) {
            uint32_t below = 0, rank_in = 0;
            for (uint32_t kk = 0; kk <= 16; kk++) {
              const uint64_t m = __builtin_amdgcn_ballot_w64(key == kk);
              below += (kk < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
              const uint32_t r = __builtin_popcountll(m & ((1ull << lane) - 1));
              rank_in = (kk == key) ? r : rank_in;
            }
            rank = below + rank_in;
          }
          s_ws = __builtin_amdgcn_ds_permute(rank * 4, (int)ws);
          s_P = __builtin_amdgcn_ds_permute(rank * 4, (int)(key == 16 ? 0u : Pl));
          if (nwin == 0) live = 0;
        }
        ws_g = __builtin_amdgcn_ds_bpermute((8 * k + g) * 4, (int)s_ws);
        Pg = __builtin_amdgcn_ds_bpermute((8 * k + g) * 4, (int)s_P);
        uint32_t mx = 0;
        for (int q = 0; q < 8; q++) mx = max(mx, (uint32_t)__builtin_amdgcn_readlane(s_P, 8 * k + q));
        P = mx ? mx : 1;
      }
      const uint32_t voff = (live && j < Pg) ? ws_g + 128 * j + 16 * c : kOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, AUX);
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
      j++;
    }
    done = !live;
  }
#pragma unroll
  for (int i = 0; i < D; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int D, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void stream(const uint8_t* bytes, uint64_t nbytes, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint64_t nchunks = nbytes / 1024;
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

uint64_t g_total = 0;

int main() {
  const uint32_t n = 10000000;
  std::vector<uint64_t> off(n + 1, 0);
  uint64_t x = 0x5EED0002;
  for (uint32_t i = 0; i < n; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    off[i + 1] = off[i] + 64 + (x >> 33) % 1437;
  }
  const uint64_t total = off[n];
  uint8_t *alloc, *bytes;
  uint64_t* doff;
  uint32_t* out;
  if (hipMalloc(&alloc, total + 8192) != hipSuccess || hipMalloc(&doff, 8 * (n + 1)) != hipSuccess ||
      hipMalloc(&out, 256 * 1024 * 4) != hipSuccess)
    return 1;
  (void)hipMemset(alloc, 0x3C, total + 8192);
  bytes = alloc + 4096;
  (void)hipMemcpy(doff, off.data(), 8 * (n + 1), hipMemcpyHostToDevice);
  g_total = total;
  printf("config 3 probe: %u frames, %.3f GB\n", n, total / 1e9);
  struct V {
    const char* name;
    void (*launch)(const uint8_t*, const uint64_t*, uint32_t, uint32_t*);
  };
#define PV(D_, W_, S_, A_, X_)                                                                                  \
  {"v8 D=" #D_ " waves=" #W_ " sort=" #S_ " align=" #A_ " aux=" #X_,                                          \
   [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) {                                        \
     hipLaunchKernelGGL((v8<D_, W_, S_, A_, X_>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou);               \
   }}
#define SV(D_, W_)                                                                                              \
  {"stream D=" #D_ " waves=" #W_, [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) {         \
     (void)o;                                                                                                   \
     (void)nn;                                                                                                  \
     hipLaunchKernelGGL((stream<D_, W_>), dim3(256), dim3(W_ * 64), 0, 0, b, g_total, ou);                      \
   }}
  V vs[] = {SV(4, 8),
            PV(4, 12, true, false, 0), PV(4, 12, true, true, 0), PV(4, 12, false, false, 0), PV(4, 12, false, true, 0),
            PV(4, 12, true, true, 2), PV(4, 12, false, true, 2), PV(6, 12, true, true, 0), PV(6, 8, true, true, 0),
            PV(4, 8, false, true, 2), PV(8, 8, false, true, 2), PV(6, 12, false, true, 2)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 3; w++) v.launch(bytes, doff, n, out);
      std::vector<float> t;
      for (int r = 0; r < 9; r++) {
        (void)hipEventRecord(e0, 0);
        v.launch(bytes, doff, n, out);
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
      printf("round %d  %-40s median %.4f ms  %.2f TB/s\n", round, v.name, t[t.size() / 2], total / t[t.size() / 2] / 1e9);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
