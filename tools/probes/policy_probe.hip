// policy_probe.hip -- loads-only probe (round 5, not product code): config 3's batch (10M frames of
// U[64,1500] B, 7.8 GB, CSR) read in the variable-length kernel's access pattern (8 lanes per frame,
// 8-frame sets, runs of 64 frames sorted by block count, windows right-aligned to the frame end rounded
// up to 4 B), with the cache policy chosen per lane: POL 0 default everywhere (the product), 1 non-temporal
// for the lanes whose 16 bytes touch neither the frame's first nor its last 128-byte line (those lines are
// shared with the neighbouring frames, which the sort puts in other sets), default for the rest -- two load
// instructions per piece, each lane in range in one of them; 2 the same two instructions, both default
// (what the extra instructions cost); 3 non-temporal everywhere.  Question: does keeping the interior of
// every frame out of the caches let the shared lines survive and the stream run faster?
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;

// LANES lanes per frame, 64 / LANES frames per set, piece = 16 * LANES bytes, JM blocks of 256 B max.
template <int LANES, int D, int WAVES, bool SORT, bool FULL = false, int POL = 0, bool ALIGNED = false>
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
          uint32_t ws, Pl;
          if (ALIGNED) {  // window from the 128-byte line holding G's first byte to the frame's last line
            ws = (a - 4) & ~127u;
            Pl = (b - ws + 127) / 128;
          } else {
            const uint32_t we = (b + 3) & ~3u;                     // window end: frame end up to 4 B
            const uint32_t J = (we - a + 4 + 255) / 256;           // blocks (G before the frame)
            ws = we - 256 * J;                                     // window start
            Pl = J * (256 / PIECE);                                // pieces
          }
          const uint32_t J = Pl;
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
      u32x4 v;
      if constexpr (POL == 0) {
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 0);
      } else if constexpr (POL == 3) {
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, 2);
      } else {
        // absolute lines: the frame's first (fs) and last (fl), this lane's 16 bytes (la, lb)
        const uintptr_t ab = (uintptr_t)base;
        const uintptr_t fs = (ab + wst + front) >> 7, fl = (ab + wst + PIECE * Pg - 1) >> 7;
        const uintptr_t la = (ab + wst + o) >> 7, lb = (ab + wst + o + 15) >> 7;
        const bool interior = la > fs && lb < fl;
        const uint32_t vn = interior ? voff : kOob, vd = interior ? kOob : voff;
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vd, 0, 0);
        const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vn, 0, POL == 1 ? 2 : 0);
        v = a | b;
      }
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


// Set-shaped variant (the planned kernel's loads): runs of 64 frames sorted by 128-byte piece count P
// (windows from the line holding G's first byte), sets of 8 frames, SL = 13 load slots per set issued
// together, 2 sets in flight per wave.  SLOTS 0: slot k = piece k, default policy.  1: slot 0 = piece 0
// and slot 1 = the frame's last piece (its shared lines) with default policy, slots 2.. = pieces 1..P-2
// non-temporal.  2: that slot order, every slot default.  3: right-aligned 256-byte blocks (the
// product's windows), 12 slots, default.
template <int SLOTS>
__global__ __launch_bounds__(768) void vset(const uint8_t* bytes, const uint64_t* offsets, uint32_t nframes,
                                            uint32_t* out) {
  __shared__ char pad_lds[160 * 1024];
  constexpr int SL = 13;
  const uint32_t lane = threadIdx.x & 63, c = lane & 7, g = lane >> 3;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * 12, w = blockIdx.x * 12 + wid;
  const uint32_t F0 = (uint64_t)nframes * w / W, F1 = (uint64_t)nframes * (w + 1) / W;
  const uint64_t b0 = offsets[F0] & ~127ull;
  const uint8_t* base = bytes + b0 - 512;
  auto rel = [&](uint64_t x) -> uint32_t { return (uint32_t)(x - b0 + 512); };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFF0, 0x00020000);
  uint32_t acc = pad_lds[threadIdx.x];
  uint32_t s_ws = 0, s_fr = 0, s_P = 0;
  uint32_t win = F0, k = 8;
  bool live = true;
  // the next set's per-lane (window start, bytes before the frame, pieces); false past the range
  auto next_set = [&](uint32_t& ws_g, uint32_t& fr_g, uint32_t& P_g) -> bool {
    if (k >= 8) {
      k = 0;
      if (win >= F1) return false;
      const uint32_t nwin = min(64u, F1 - win);
      const uint32_t a = rel(offsets[min(win + lane, F1)]), b = rel(offsets[min(win + lane + 1, F1)]);
      uint32_t ws, Pl;
      if (SLOTS == 3) {
        const uint32_t we = (b + 3) & ~3u;
        const uint32_t J = (we - a + 4 + 255) / 256;
        ws = we - 256 * J;
        Pl = 2 * J;
      } else {
        ws = (a - 4) & ~127u;
        Pl = (b - ws + 127) / 128;
      }
      const uint32_t key = lane < nwin ? min(Pl, 15u) : 16u;
      uint32_t below = 0, rank_in = 0;
      for (uint32_t kk = 0; kk <= 16; kk++) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(key == kk);
        below += (kk < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
        const uint32_t r = __builtin_popcountll(m & ((1ull << lane) - 1));
        rank_in = (kk == key) ? r : rank_in;
      }
      const uint32_t rank = below + rank_in;
      s_ws = __builtin_amdgcn_ds_permute(rank * 4, (int)ws);
      s_fr = __builtin_amdgcn_ds_permute(rank * 4, (int)(a - ws));
      s_P = __builtin_amdgcn_ds_permute(rank * 4, (int)(key == 16 ? 0u : Pl));
      win += 64;
    }
    ws_g = __builtin_amdgcn_ds_bpermute((8 * k + g) * 4, (int)s_ws);
    fr_g = __builtin_amdgcn_ds_bpermute((8 * k + g) * 4, (int)s_fr);
    P_g = __builtin_amdgcn_ds_bpermute((8 * k + g) * 4, (int)s_P);
    k++;
    return true;
  };
  auto issue = [&](bool ok, uint32_t ws, uint32_t fr, uint32_t P, u32x4 (&x)[SL]) {
    const uint32_t o0 = ok ? ws + 16 * c : kOob;
    const bool before0 = 16 * c + 16 <= fr;  // the lane's 16 bytes of piece 0 lie before the frame
#pragma unroll
    for (int s = 0; s < SL; s++) {
      uint32_t piece, vo;
      int aux = 0;
      if (SLOTS == 0 || SLOTS == 3) {
        piece = s;
        vo = (piece < P && !(s == 0 && before0) && !(SLOTS == 3 && s == 1 && 128 + 16 * c + 16 <= fr)) ? o0 + 128 * s : kOob;
        if (SLOTS == 3 && s >= 12) vo = kOob;
      } else {
        if (s == 0) {
          vo = before0 ? kOob : o0;
        } else if (s == 1) {
          vo = P >= 2 ? o0 + 128 * (P - 1) : kOob;
        } else {
          vo = (uint32_t)(s - 1) < P - 1 && P >= 2 ? o0 + 128 * (s - 1) : kOob;
          aux = SLOTS == 1 ? 2 : 0;
        }
      }
      if (aux == 2)
        x[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, 2);
      else
        x[s] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, 0);
    }
  };
  u32x4 A[SL], B[SL];
  uint32_t ws, fr, P;
  bool okA = next_set(ws, fr, P);
  issue(okA, ws, fr, P, A);
  while (okA) {
    bool okB = next_set(ws, fr, P);
    issue(okB, ws, fr, P, B);
#pragma unroll
    for (int s = 0; s < SL; s++) acc ^= A[s].x ^ A[s].y ^ A[s].z ^ A[s].w;
    if (!okB) break;
    okA = next_set(ws, fr, P);
    issue(okA, ws, fr, P, A);
#pragma unroll
    for (int s = 0; s < SL; s++) acc ^= B[s].x ^ B[s].y ^ B[s].z ^ B[s].w;
  }
#pragma unroll
  for (int s = 0; s < SL; s++) acc ^= A[s].x ^ B[s].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  (void)live;
}

// Round 6: the product's load schedule without its compute.  One set buffer of 13 slots per wave (slot 0 =
// line 0, slot k >= 1 = line k - 13 + P, the last line default policy, the lines between non-temporal),
// software-pipelined as the product: slot k of the next set is issued as soon as the current set has
// consumed slot k.  The sets (8 frames each, sorted by line count within runs of 64 on the host) come as
// one 16-byte record per frame, read two sets ahead.  STEPS: each consumed slot also runs the product's
// chain step (4 perm + 4 ds_read_b32 + 2 xor3 per word from LDS; the values are not a CRC).  Question: is
// the one-buffer schedule itself, or the compute on it, what holds config 3's gate above the 2-buffer
// probe's 1.18 ms?
struct SetRec {
  uint32_t ws, fr, P, wsh;  // window start (low, high 32 bits of the offset in the allocation)
};
template <int WAVES, bool STEPS>
__global__ __launch_bounds__(WAVES * 64) void vpipe(const uint8_t* bytes, const SetRec* recs, uint32_t nsets,
                                                    uint32_t* out) {
  __shared__ char lds[160 * 1024];
  constexpr int SL = 13;
  const uint32_t lane = threadIdx.x & 63, c = lane & 7, g = lane >> 3;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * WAVES, w = blockIdx.x * WAVES + wid;
  const uint32_t S0 = (uint64_t)nsets * w / W, S1 = (uint64_t)nsets * (w + 1) / W;
  // (the wave's base: its first window start - 512; window starts relative to it fit 32 bits)
  // (read as a vector load and made uniform with readfirstlane: a scalar load of the two words was
  // combined with a sign-extending s_bfe_i64 of the low word, a wrong base past 2 GB -- round 6's fault)
  const u32x4 r0v = *(const u32x4*)(recs + (uint64_t)S0 * 8);
  const uint64_t wbase = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r0v.x) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r0v.w) << 32);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + wbase - 512), 0, 0x7FFFFFF0, 0x00020000);
  for (uint32_t i = threadIdx.x; i < 160 * 1024 / 4; i += WAVES * 64) ((uint32_t*)lds)[i] = i * 0x9E3779B1u;
  __syncthreads();
  const uint32_t K = ((lane & 31u) * 4u) | (((lane & 31u) * 4u + 128u) << 8) | (1u << 24);
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, acc = 0;
  auto step = [&](uint32_t v, uint32_t x) -> uint32_t {
    const char* t = lds + 32768;
    const uint32_t r0 = *(const uint32_t*)(t + __builtin_amdgcn_perm(v, K, 0x0C020400u));
    const uint32_t r1 = *(const uint32_t*)(t + __builtin_amdgcn_perm(v, K, 0x0C020501u));
    const uint32_t r2 = *(const uint32_t*)(t + __builtin_amdgcn_perm(v, K, 0x0C030600u));
    const uint32_t r3 = *(const uint32_t*)(t + __builtin_amdgcn_perm(v, K, 0x0C030701u));
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(r0, r1, r2, 0x96), r3, x, 0x96);
  };
  auto rec = [&](uint32_t si) -> SetRec {  // (unconditional: the array holds 2 padding sets past the last)
    const u32x4 v = *(const u32x4*)(recs + (uint64_t)si * 8 + g);
    return SetRec{(uint32_t)(((uint64_t)v.w << 32 | v.x) - wbase + 512u), v.y, v.z, 0u};
  };
  // dep: the value the consuming step has just produced; the load is tied after it (as the product's
  // load_slot), so the loads go out in slot order and the waits stay counted
  auto load = [&](int s, const SetRec& r, uint32_t dep, bool live = true) -> u32x4 {
    const uint32_t o0 = live && r.P > 0 ? r.ws + 16 * c : kOob;
    uint32_t vo;
    if (s == 0) {
      vo = 16 * c + 16 <= r.fr ? kOob : o0;
    } else {
      const int line = s - 13 + (int)r.P;
      vo = line >= 1 ? o0 + 128u * (uint32_t)line : kOob;
    }
    asm("" : "+v"(vo) : "v"(dep));
    if (s == 0 || s == 12) return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, 0);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, 2);
  };
  u32x4 A[SL];
  {
    const SetRec r0 = rec(S0);
#pragma unroll
    for (int s = 0; s < SL; s++) A[s] = load(s, r0, 0u);
  }
  // records of sets si + 1 and si + 2 in two registers used in turn (no copy of a pending load's result)
  SetRec ra = rec(S0 + 1), rb = rec(S0 + 2);
  auto body = [&](const SetRec& rn, bool live) {
#pragma unroll
    for (int s = 0; s < SL; s++) {
      const u32x4 x = A[s];
      if (STEPS) {
        c0 = step(c0, x.x);
        c1 = step(c1, x.y);
        c2 = step(c2, x.z);
        c3 = step(c3, x.w);
      } else {
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
      }
      A[s] = load(s, rn, STEPS ? (c0 ^ c3) : acc, live);
      asm volatile("" ::: "memory");  // (one slot at a time, as the product's position blocks)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (uint32_t si = S0; si < S1; si += 2) {
    body(ra, si + 1 < S1);
    ra = rec(si + 3);
    if (si + 1 >= S1) break;
    body(rb, si + 2 < S1);
    rb = rec(si + 4);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ c0 ^ c1 ^ c2 ^ c3;
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
SetRec* g_recs = nullptr;
uint32_t g_nsets = 0;
uint8_t* g_alloc = nullptr;

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
  {  // vpipe's set records: runs of 64 frames sorted by line count (stable), 8 frames per set
    const uint32_t nsets = (n + 7) / 8;
    std::vector<SetRec> recs((size_t)(nsets + 4) * 8, SetRec{0, 0, 0, 0});  // (+ padding sets, P = 0)
    const uint64_t ab = (uint64_t)(bytes - alloc);
    for (uint32_t r0 = 0; r0 < n; r0 += 64) {
      std::vector<std::pair<uint32_t, uint32_t>> kf;
      for (uint32_t i = r0; i < std::min(n, r0 + 64); i++) {
        const uint64_t a = off[i] + ab, b = off[i + 1] + ab;  // (offsets within the allocation)
        const uint64_t ws = (a - 4) & ~127ull;
        kf.push_back({(uint32_t)((b - ws + 127) / 128), i});
      }
      std::stable_sort(kf.begin(), kf.end(), [](auto& x, auto& y) { return x.first < y.first; });
      for (size_t j = 0; j < kf.size(); j++) {
        const uint32_t i = kf[j].second;
        const uint64_t a = off[i] + ab, ws = (a - 4) & ~127ull;
        recs[(size_t)(r0 / 8 + j / 8) * 8 + j % 8] = SetRec{(uint32_t)ws, (uint32_t)(a - ws), kf[j].first, (uint32_t)(ws >> 32)};
      }
    }
    if (hipMalloc(&g_recs, recs.size() * sizeof(SetRec)) != hipSuccess) return 1;
    (void)hipMemcpy(g_recs, recs.data(), recs.size() * sizeof(SetRec), hipMemcpyHostToDevice);
    g_nsets = nsets;
    g_alloc = alloc;
  }
  printf("policy probe: %u frames, %.3f GB\n", n, total / 1e9);
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
#define PP(D_, P_, A_)                                                                              \
  {"D=" #D_ " pol=" #P_ " aligned=" #A_, [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
     hipLaunchKernelGGL((vl<8, D_, 12, true, false, P_, A_>), dim3(256), dim3(12 * 64), 0, 0, b, o, nn, ou); \
   }}
  V vs[] = {{"stream", [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) {
               (void)o;
               (void)nn;
               hipLaunchKernelGGL(stream, dim3(256), dim3(512), 0, 0, b, g_total, ou);
             }},
            PP(12, 0, false), PP(12, 1, true),
#define PS(S_) {"set slots=" #S_, [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
     hipLaunchKernelGGL((vset<S_>), dim3(256), dim3(768), 0, 0, b, o, nn, ou); }}
            PS(1),
#define PQ(W_, S_) {"pipe waves=" #W_ " steps=" #S_, [](const uint8_t* b, const uint64_t* o, uint32_t nn, uint32_t* ou) { \
     (void)b; (void)o; (void)nn; \
     hipLaunchKernelGGL((vpipe<W_, S_>), dim3(256), dim3(W_ * 64), 0, 0, g_alloc, g_recs, g_nsets, ou); }}
            PQ(16, false), PQ(16, true), PQ(12, false), PQ(12, true)};
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
