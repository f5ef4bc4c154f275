// lanes_probe.hip -- loads-only probe (tuning, not product code): config 3's batch (10M frames of
// U[64,1500] B, 7.8 GB, CSR) read in the variable-length kernel's access pattern with 8 lanes per
// frame (8-frame sets, 128-byte pieces: the product's varlen8 layout) against 16 lanes per frame
// (4-frame sets, 256-byte pieces: the fixed kernel's layout), runs of 64 frames ordered by block
// count (ballot ranks) or not, windows right-aligned to the frame end rounded up to 4 B, pieces wholly
// before the frame out of range (no request), default cache policy, DEPTH sets in flight per wave, one
// workgroup per CU.  Question (round 4, first): does the 16-lane layout's access pattern (3 lines per
// 256-B piece instead of 2 per 128-B piece) stream faster?  (Second, "full6"): what do the out-of-range
// load instructions cost that the product kernel issues for the blocks past a set's own (it issues 6
// blocks' loads for every set)?  Prints one line per variant (median of 9 launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;

// LANES lanes per frame, 64 / LANES frames per set, piece = 16 * LANES bytes, JM blocks of 256 B max.
template <int LANES, int D, int WAVES, bool SORT, bool FULL = false>
__global__ __launch_bounds__(WAVES * 64) void vl(const uint8_t* bytes, const uint64_t* offsets, uint32_t nframes,
                                                 uint32_t* out) {
  __shared__ char pad_lds[160 * 1024];  // one workgroup per CU, as the kernels
  constexpr uint32_t FPS = 64 / LANES;  // frames per set
  constexpr uint32_t PIECE = 16 * LANES;
  constexpr uint32_t SETS = 64 / FPS;  // sets per run of 64 frames
  const uint32_t lane = threadIdx.x & 63, c = lane % LANES, g = lane / LANES;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint32_t F0 = (uint64_t)nframes * w / W, F1 = (uint64_t)nframes * (w + 1) / W;
  const uint64_t b0 = offsets[F0] & ~127ull;
  const uint8_t* base = bytes + b0 - 512;
  auto rel = [&](uint64_t x) -> uint32_t { return (uint32_t)(x - b0 + 512); };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
  uint32_t acc = pad_lds[threadIdx.x];
  uint32_t win = F0 - 64, k = SETS, j = 0, P = 0;
  uint32_t s_ws = 0, s_fr = 0, s_P = 0, ws_g = 0, fr_g = 0, Pg = 0, live = 1;
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
        if (k >= SETS) {  // next run of 64 frames: one frame per lane
          win += 64;
          k = 0;
          const uint32_t nwin = win < F1 ? min(64u, F1 - win) : 0u;
          const uint32_t a = rel(offsets[min(win + lane, F1)]), b = rel(offsets[min(win + lane + 1, F1)]);
          const uint32_t we = (b + 3) & ~3u;                       // window end: frame end up to 4 B
          const uint32_t J = (we - a + 4 + 255) / 256;             // blocks (G before the frame)
          const uint32_t ws = we - 256 * J;                        // window start
          const uint32_t Pl = J * (256 / PIECE);                   // pieces
          const uint32_t key = lane < nwin ? min(J, 15u) : 16u;
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
          s_fr = __builtin_amdgcn_ds_permute(rank * 4, (int)(a - ws));
          s_P = __builtin_amdgcn_ds_permute(rank * 4, (int)(key == 16 ? 0u : Pl));
          if (nwin == 0) live = 0;
        }
        ws_g = __builtin_amdgcn_ds_bpermute((FPS * k + g) * 4, (int)s_ws);
        fr_g = __builtin_amdgcn_ds_bpermute((FPS * k + g) * 4, (int)s_fr);
        Pg = __builtin_amdgcn_ds_bpermute((FPS * k + g) * 4, (int)s_P);
        uint32_t mx = 0;
        for (uint32_t q = 0; q < FPS; q++) mx = max(mx, (uint32_t)__builtin_amdgcn_readlane(s_P, FPS * k + q));
        P = FULL ? 6u * (256 / PIECE) : (mx ? mx : 1);  // FULL: every set issues 6 blocks' loads (out of range past its own)
      }
      const uint32_t wst = ws_g, front = fr_g;  // window start, bytes before the frame
      const uint32_t o = PIECE * j + 16 * c;
      const bool before = o + 16 <= front;  // the piece is wholly before the frame
      const uint32_t voff = (live && j < Pg && !before) ? wst + o : kOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 0);
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

__global__ __launch_bounds__(512) void stream(const uint8_t* bytes, uint64_t nbytes, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * 8, w = blockIdx.x * 8 + wid;
  const uint64_t nchunks = nbytes / 1024;
  const uint64_t lo = nchunks * w / W, hi = nchunks * (w + 1) / W;
  uint32_t acc = 0;
  u32x4 data[4];
  for (int i = 0; i < 4; i++) data[i] = (u32x4){0, 0, 0, 0};
  for (uint64_t k = lo; k < hi; k += 4) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint64_t kk = min(k + s, hi - 1);
      const u32x4 v = __builtin_nontemporal_load((const u32x4*)(bytes + kk * 1024 + 16 * lane));
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
    }
  }
  for (int i = 0; i < 4; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
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
  printf("lanes probe: %u frames, %.3f GB\n", n, total / 1e9);
  struct V {
    const char* name;
    void (*launch)(const uint8_t*, const uint64_t*, uint32_t, uint32_t*);
  };
#define PV(L_, D_, W_, S_)                                                                         \
  {"lanes=" #L_ " D=" #D_ " waves=" #W_ " sort=" #S_, [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
     hipLaunchKernelGGL((vl<L_, D_, W_, S_>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou);       \
   }}
#define PVF(L_, D_, W_, S_)                                                                        \
  {"lanes=" #L_ " D=" #D_ " waves=" #W_ " sort=" #S_ " full6", [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
     hipLaunchKernelGGL((vl<L_, D_, W_, S_, true>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou); \
   }}
  V vs[] = {{"stream", [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) {
               (void)o;
               (void)nn;
               hipLaunchKernelGGL(stream, dim3(256), dim3(512), 0, 0, b, g_total, ou);
             }},
            PV(8, 4, 12, true), PVF(8, 4, 12, true), PV(8, 8, 12, true), PVF(8, 8, 12, true), PV(8, 12, 12, true),
            PVF(8, 12, 12, true)};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // settle: clocks ramp up from idle over ~1 s
  for (int i = 0; i < 400; i++) vs[0].launch(bytes, doff, n, out);
  (void)hipDeviceSynchronize();
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
      printf("round %d  %-36s median %.4f ms  %.2f TB/s\n", round, v.name, t[t.size() / 2], total / t[t.size() / 2] / 1e9);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
