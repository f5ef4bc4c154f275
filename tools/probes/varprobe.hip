// varprobe.hip -- loads-only probe of candidate access patterns for the variable-length gate
// (config 3: 10M frames of U[64,1500] B, 7.8 GB).  Tuning probe, not product code.
//
// Pattern "groups": a wave owns a contiguous frame range; its 64/G groups of G lanes each hold one
// frame and walk it in B = 16 G byte blocks (one 16-B load per lane per step), right-aligned to the
// frame end and realigned to 4 bytes.  A group that finishes its frame takes the next unassigned
// frame of the wave's range (in order, ballot + popcount ranks), reading its offsets from a per-wave
// LDS ring that the wave refills from `offsets` with one coalesced load per D steps.  D steps of
// loads are in flight per wave.  The data is XOR-folded (no CRC).
// Pattern "stream": the same bytes read as one contiguous stream (16 B per lane, D in flight): the
// ceiling for 7.8 GB.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOob = 0x80000000u;
uint64_t g_total = 0;

template <int G, int D, int WAVES, bool PADSKIP = false>
__global__ __launch_bounds__(WAVES * 64) void groups(const uint8_t* bytes, const uint64_t* offsets, uint32_t nframes,
                                                     uint32_t* out) {
  constexpr int B = 16 * G;
  __shared__ uint32_t ring[WAVES][256];
  __shared__ char pad_lds[160 * 1024 - WAVES * 1024];  // one workgroup per CU, as the real kernel
  const uint32_t lane = threadIdx.x & 63, c = lane % G, g = lane / G;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint32_t F0 = (uint64_t)nframes * w / W, F1 = (uint64_t)nframes * (w + 1) / W;
  const uint32_t nf = F1 - F0;
  const uint64_t b0 = offsets[F0] & ~3ull;
  const uint8_t* base = bytes + b0 - 256;
  auto rel = [&](uint64_t x) -> uint32_t { return (uint32_t)(x - b0 + 256); };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
  uint32_t* rg = ring[wid];
  // prologue: frames [0, 256) of the range
  for (int k = 0; k < 4; k++) rg[64 * k + lane] = rel(offsets[F0 + min(64u * k + lane, nf)]);
  __syncthreads();
  uint32_t fp = 256, cp = 0;
  uint32_t refill = rg[192 + lane];
  uint32_t a = 0, e = 0, J = 0, blk = 0, live = 1;
  uint32_t acc = pad_lds[threadIdx.x];
  u32x4 data[D];
#pragma unroll
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  bool done = false;
  while (!done) {
    // ring refill: one coalesced load per iteration, written one iteration later
    rg[(fp - 64 + lane) & 255] = refill;  // (the first time rewrites frames [192, 256): the same values)
    {
      const uint32_t f = (fp - cp < 192) ? fp : fp - 64;
      refill = rel(offsets[F0 + min(f + lane, nf)]);
      fp = f + 64;
    }
#pragma unroll
    for (int s = 0; s < D; s++) {
      const bool need = live && blk >= J;
      const uint64_t m = __builtin_amdgcn_ballot_w64(need && c == 0);
      if (m) {
        const uint32_t rank = __builtin_popcountll(m & ((1ull << (g * G)) - 1));
        if (need) {
          const uint32_t idx = cp + rank;
          if (idx < nf) {
            a = rg[idx & 255];
            e = rg[(idx + 1) & 255];
            J = (e - a + 4 + B - 1) / B;
            blk = 0;
          } else {
            live = 0;
          }
        }
        cp += __builtin_popcountll(m);
      }
      const uint32_t ws = e - B * J;                 // window start (relative)
      const bool padlane = PADSKIP && blk == 0 && 16 * c + 16 <= B * J - (e - a);
      const uint32_t voff = (live && !padlane) ? ((ws + 3) & ~3u) + B * blk + 16 * c : kOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 2);
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
      blk++;
    }
    done = __builtin_amdgcn_ballot_w64(live) == 0;
  }
#pragma unroll
  for (int i = 0; i < D; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}


// Pattern "sorted": the wave walks its range in windows of 64 frames; each window's frames are
// sorted by block count J (ballot ranks, ds_permute into sorted lanes), sets of 4 consecutive
// sorted frames share J (up to the bin edges), and the wave issues one 1-KB block load per step:
// block j of the 4 frames of the load cursor's set (exactly J loads per set).  D steps in flight;
// the next window's offsets are prefetched one unrolled iteration (D steps) ahead.
template <int D, int WAVES, int SORTW, bool PADSKIP>
__global__ __launch_bounds__(WAVES * 64) void sorted(const uint8_t* bytes, const uint64_t* offsets, uint32_t nframes,
                                                     uint32_t* out) {
  __shared__ char pad_lds[160 * 1024];
  const uint32_t lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint32_t F0 = (uint64_t)nframes * w / W, F1 = (uint64_t)nframes * (w + 1) / W;
  const uint64_t b0 = offsets[F0] & ~3ull;
  const uint8_t* base = bytes + b0 - 256;
  auto rel = [&](uint64_t x) -> uint32_t { return (uint32_t)(x - b0 + 256); };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
  uint32_t acc = pad_lds[threadIdx.x];
  // window state (load cursor side)
  uint32_t win = F0;                       // first frame of the current window
  uint32_t s_ws = 0, s_J = 0;              // sorted lanes: window start (rel) and J of sorted frame `lane`
  uint32_t k = 16, j = 0, J = 0;           // set in window, block in set, set's J (k = 16: window exhausted)
  uint32_t ws_g = 0, Jg = 0, pad_g = 0;    // this group's frame window start, J and pad for the current set
  uint32_t s_pad = 0;
  uint32_t live = 1;
  auto fetch = [&](uint32_t wf, uint32_t& pa, uint32_t& pb) {
    pa = rel(offsets[min(wf + lane, F1)]);
    pb = rel(offsets[min(wf + lane + 1, F1)]);
  };
  uint32_t pa, pb, qa, qb, tp, tq;  // prefetched offsets of window tp (usable) and tq (in flight)
  fetch(F0, qa, qb);
  tq = F0;
  win = F0 - 64;
  u32x4 data[D];
#pragma unroll
  for (int i = 0; i < D; i++) data[i] = (u32x4){0, 0, 0, 0};
  bool done = false;
  while (!done) {
    pa = qa;  // the prefetch issued one iteration (D steps) ago
    pb = qb;
    tp = tq;
    tq = win + 64 == tp ? win + 128 : win + 64;
    fetch(tq, qa, qb);
#pragma unroll
    for (int s = 0; s < D; s++) {
      if (j >= J) {  // next set
        k++;
        j = 0;
        if (k >= 16) {  // next window: sort it
          win += 64;
          k = 0;
          uint32_t a = pa, b = pb;
          if (tp != win) fetch(win, a, b);  // (not prefetched: rare)
          const uint32_t nwin = win < F1 ? min(64u, F1 - win) : 0u;
          const uint32_t len = b - a;
          uint32_t Jl = (len + 4 + 255) / 256;
          uint32_t key = lane < nwin ? min(Jl, 7u) : 8u;
          uint32_t rank = lane;
          if (SORTW > 1) {  // sort by J within aligned windows of SORTW lanes
            const uint64_t qmask = (SORTW == 64) ? ~0ull : (((1ull << SORTW) - 1) << (lane & ~(SORTW - 1)));
            uint32_t below = 0, rank_in = 0;
#pragma unroll
            for (uint32_t kk = 1; kk <= 8; kk++) {
              const uint64_t m = __builtin_amdgcn_ballot_w64(key == kk) & qmask;
              below += (kk < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
              const uint32_t r = __builtin_popcountll(m & ((1ull << lane) - 1));
              rank_in = (kk == key) ? r : rank_in;
            }
            rank = (lane & ~(SORTW - 1)) + below + rank_in;
          }
          s_ws = __builtin_amdgcn_ds_permute(rank * 4, (int)(b - 256 * Jl));
          s_J = __builtin_amdgcn_ds_permute(rank * 4, (int)(key == 8 ? 0u : Jl));
          s_pad = __builtin_amdgcn_ds_permute(rank * 4, (int)(256 * Jl - len));
          if (nwin == 0) live = 0;
        }
        ws_g = __builtin_amdgcn_ds_bpermute((4 * k + g) * 4, (int)s_ws);
        Jg = __builtin_amdgcn_ds_bpermute((4 * k + g) * 4, (int)s_J);
        pad_g = __builtin_amdgcn_ds_bpermute((4 * k + g) * 4, (int)s_pad);
        J = max(max(__builtin_amdgcn_readlane(s_J, 4 * k), __builtin_amdgcn_readlane(s_J, 4 * k + 1)),
                max(__builtin_amdgcn_readlane(s_J, 4 * k + 2), __builtin_amdgcn_readlane(s_J, 4 * k + 3)));
        if (J == 0) { J = 1; }
      }
      const bool padlane = PADSKIP && j == 0 && 16 * c + 16 <= pad_g;
      const uint32_t voff = (live && j < Jg && !padlane) ? ((ws_g + 3) & ~3u) + 256 * j + 16 * c : kOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 2);
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
  uint64_t* doff;
  uint32_t* out;
  uint8_t* alloc;
  if (hipMalloc(&alloc, total + 8192) != hipSuccess || hipMalloc(&doff, 8 * (n + 1)) != hipSuccess ||
      hipMalloc(&out, 256 * 1024 * 4) != hipSuccess)
    return 1;
  (void)hipMemset(alloc, 0x3C, total + 8192);
  bytes = alloc + 4096;  // the first frames' windows start up to 67 B before the batch
  (void)hipMemcpy(doff, off.data(), 8 * (n + 1), hipMemcpyHostToDevice);
  printf("config 3 probe: %u frames, %.3f GB\n", n, total / 1e9);
  struct V {
    const char* name;
    void (*launch)(const uint8_t*, const uint64_t*, uint32_t, uint32_t*);
  };
#define GV(G_, D_, W_) {"groups G=" #G_ " (B=" #G_ "*16) D=" #D_ " waves=" #W_, \
    [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
      hipLaunchKernelGGL((groups<G_, D_, W_>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou); }}
#define SO(D_, W_, S_, P_) {"sorted" #S_ " blockstream D=" #D_ " waves=" #W_ " padskip=" #P_, \
    [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
      hipLaunchKernelGGL((sorted<D_, W_, S_, P_>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou); }}
#define GP(G_, D_, W_) {"groups G=" #G_ " D=" #D_ " waves=" #W_ " padskip", \
    [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
      hipLaunchKernelGGL((groups<G_, D_, W_, true>), dim3(256), dim3(W_ * 64), 0, 0, b, o, nn, ou); }}
#define SV(D_, W_) {"stream D=" #D_ " waves=" #W_, \
    [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
      (void)o; (void)nn; \
      hipLaunchKernelGGL((stream<D_, W_>), dim3(256), dim3(W_ * 64), 0, 0, b, g_total, ou); }}
  V vs[] = {SV(4, 8), SO(12, 8, 16, true), SO(8, 16, 16, true), SO(6, 16, 16, true), SO(4, 16, 16, true), SO(8, 8, 16, true), SO(16, 8, 16, true), SO(12, 8, 32, true)};
  g_total = total;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 5; w++) v.launch(bytes, doff, n, out);
      std::vector<float> t;
      for (int r = 0; r < 15; r++) {
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
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
