// frame_crc_varlen2.hip -- the variable-length frame-CRC kernel (CSR offsets or (start, end) pairs)
// for MI355X / gfx950: BASELINE.json config 3 (10M frames of U[64,1500] B) and the receive path.
//
// The batched CRC gate of Frame::read (src/frame/serial/mod.rs:675-690) and the frame seal
// (serial/mod.rs:463-470, build.rs:151-159) for frame i = bytes[offsets[i] .. offsets[i+1]).
// Same math, LDS tables and 16-lanes-per-frame layout as the fixed kernels (frame_crc_dev.hpp);
// what differs is how mixed lengths are scheduled (probes: tools/probes/varprobe.hip):
//   * Sorted sets.  A wave walks its contiguous frame range in super-windows of 64 frames.  Each
//     super-window's frames are sorted by block count J inside aligned windows of 16 (ballot ranks,
//     ds_permute into sorted lanes); a set = 4 consecutive sorted frames (one per 16-lane group), so
//     a set's frames mostly share J: a set costs max J blocks, 4.0 on average for config 3 against
//     5.2 for 4 consecutive unsorted frames.  (Sorting over 64 frames would save more compute but
//     costs the memory system locality: loads-only 5.7 vs 5.9 TB/s.)
//   * A block stream.  One 1-KB wave load per step: block j of the 4 frames of the load cursor's
//     set, so a set issues exactly max J loads; kV2Depth steps are in flight per wave.  Lanes whose
//     16 bytes lie wholly before their frame (the right-aligned window's pad) and blocks past a
//     frame's own J load nothing (an out-of-range buffer offset).  The compute cursor consumes the
//     ring in the same order; per-step geometry travels with the data (a per-lane VGPR and a
//     wave-uniform SGPR word per ring slot).
//   * Uniform control.  Block 0 of a set (front fix: zeros / G before the frame, no table lookups),
//     block 1 (the word that may straddle G), the chain steps, the frozen chains of a mixed set and
//     the set's finish are uniform branches.
//   * Results of a super-window collect in one register per lane (lane l = frame l of the window)
//     and leave as one coalesced store per super-window (hidden from hipcc's wait counts).
//   * Slow frames -- shorter than 4 B or longer than 6 blocks, a window that starts before the buffer
//     or ends within 3 bytes of its end -- stay out of the sets and run byte-wise, four at a time,
//     when their super-window's results are flushed (rare: the batch's first and last frames).
//   * Everything rare (sorting the next super-window, flushing the previous one, slow frames) runs
//     once per kV2Depth steps, outside the unrolled steps, which stay small.
#include <type_traits>

#include "frame_crc_dev.hpp"

namespace ufc_dev {

namespace {

constexpr int kV2Waves = kVarlen2Threads / 64;  // 16: four waves per SIMD hide each other's issue
constexpr int kV2Depth = 8;             // block steps in flight per wave (= the unrolled loop's length)
constexpr uint32_t kV2Oob = 0x80000000u;  // out-of-range buffer offset: loads zeros, no memory request
constexpr uint32_t kV2Bias = 512;        // relative offsets: x - (first byte of the wave, 4-aligned down) + bias
constexpr int kV2Blocks = 6;             // fast path: frames of 4..1532 B
#ifndef UFC_V2_AUX
#define UFC_V2_AUX 2
#endif
constexpr int kV2Aux = UFC_V2_AUX;         // cache policy of the block loads

// Per-lane frame geometry (one VGPR): pad [0,9), J [9,12), dl [12,14), len >= 5 [14], live [15],
// [16,22): the frame's index in its super-window (sorting, the slow path) or, in a ring entry, the
// set's index in its super-window (uniform).
__device__ __forceinline__ uint32_t g_pad(uint32_t g) { return g & 511u; }
__device__ __forceinline__ uint32_t g_J(uint32_t g) { return (g >> 9) & 7u; }
__device__ __forceinline__ uint32_t g_dl(uint32_t g) { return (g >> 12) & 3u; }
__device__ __forceinline__ bool g_len5(uint32_t g) { return (g >> 14) & 1u; }
__device__ __forceinline__ bool g_live(uint32_t g) { return (g >> 15) & 1u; }
__device__ __forceinline__ uint32_t g_idx(uint32_t g) { return (g >> 16) & 63u; }
__device__ __forceinline__ uint32_t g_set(uint32_t g) { return (g >> 16) & 15u; }

// Step word (wave-uniform, in bits [22,32) of the ring's geometry word): j [0,3), Jset [3,6),
// valid [6], the first step of a super-window [7], mixed J in the set [8], a frame of the set has
// G in block 1 (pad > 252) [9].  A valid step with Jset = 0 is a marker (a super-window without a
// set of fast frames: only the compute cursor's crossing).
constexpr uint32_t kStValid = 1u << 6, kStFirst = 1u << 7, kStMixed = 1u << 8, kStG1 = 1u << 9;
constexpr int kStShift = 22;

// Stores written as inline asm (see frame_crc_dev.hpp st_u32_hidden).
__device__ __forceinline__ void st_u8_hidden_v2(uint8_t* a, uint32_t v) {
  asm volatile("global_store_byte %0, %1, off" : : "v"(a), "v"(v));
}

}  // namespace

template <bool SEAL, bool PAIRS>
__global__ __launch_bounds__(kV2Waves * 64) void frame_crc_varlen2_kernel(const KernelParams p) {
  constexpr int D = kV2Depth;
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const StageSet<kV2Waves * 64> sr = stage_load<kV2Waves * 64>(p);
  Lane L;
  init_lane(L, lds, p.G);
  const uint32_t lane = (uint32_t)L.lane, col = (uint32_t)L.col, grp = (uint32_t)L.grp;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t W = gridDim.x * kV2Waves, w = blockIdx.x * kV2Waves + wid;
  const uint64_t nfr = p.nframes;
  const uint64_t F0 = nfr * w / W, F1 = nfr * (w + 1) / W;
  const uint32_t nf = (uint32_t)(F1 - F0);  // frames of this wave (< 2^31: host-chunked)

  // Frame bounds (absolute byte offsets into p.bytes) and the wave's relative addressing.
  auto bounds = [&](uint64_t f, uint64_t& a, uint64_t& b) {
    if (PAIRS) {
      a = *as_global<g_u64>(p.offsets + 2 * f);
      b = *as_global<g_u64>(p.offsets + 2 * f + 1);
    } else {
      a = *as_global<g_u64>(p.offsets + f);
      b = *as_global<g_u64>(p.offsets + f + 1);
    }
  };
  uint64_t b0 = 0;  // pairs: addresses relative to the buffer itself (host: bytes_len < 2^31 - 1024)
  if (!PAIRS && nf) {
    const uint64_t v = *as_global<g_u64>(p.offsets + F0);
    b0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
  }
  b0 &= ~3ull;
  const uint8_t* base = p.bytes + b0 - kV2Bias;
  const uint64_t buf_end = PAIRS ? p.frame_len : *as_global<g_u64>(p.offsets + nfr);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)0x7FFFFFF0, 0x00020000);
  // bounds of frame sw + lane of super-window sw (clamped to the range)
  auto fetch = [&](uint32_t sw, uint64_t& a, uint64_t& b) { bounds(F0 + min(sw + lane, nf - 1), a, b); };

  // Sort a super-window (bounds a, b of frame sw + lane): sorted records (lane l = l-th frame in
  // sorted order) and the mask of its slow frames (bit = frame index in the window).
  auto sort_window = [&](uint32_t sw, uint64_t a, uint64_t b, uint32_t& o_ws, uint32_t& o_geo, uint64_t& o_slow,
                         uint32_t& o_rank) {
    const bool live = sw + lane < nf;
    const uint64_t len64 = b >= a ? b - a : 0;
    const uint32_t len = (uint32_t)min(len64, (uint64_t)0x7FFFFFFF);
    const uint32_t J = (len + 4u + 255u) >> 8;  // (len >= 4: E = len)
    const uint32_t pad = (J * 256u - len) & 511u;
    const uint64_t wsabs = b - 256u * (uint64_t)J;  // window start, absolute
    const uint32_t dl = (0u - ((uint32_t)(uintptr_t)p.bytes + (uint32_t)wsabs)) & 3u;
    const uint64_t wsrel = wsabs - b0 + kV2Bias;
    const bool fast = len >= 4u && J <= (uint32_t)kV2Blocks && a >= pad && b + 3 <= buf_end && b >= b0 &&
                      wsrel + 256u * J + 16u < 0x7FFFFFF0u;
    o_slow = __builtin_amdgcn_ballot_w64(live && !fast);
    const uint32_t key = (live && fast) ? J : 8u;  // slow and dead frames sort last, out of the sets
    const uint64_t qmask = 0xFFFFull << (lane & 48u);  // ranks inside aligned windows of 16 lanes
    uint32_t below = 0, rank_in = 0;
#pragma unroll
    for (uint32_t kk = 1; kk <= 6; kk++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(key == kk) & qmask;
      below += (kk < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
      const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      rank_in = (kk == key) ? r : rank_in;
    }
    if (key == 8u) {  // after the quarter's fast frames
      const uint64_t m = __builtin_amdgcn_ballot_w64(key == 8u) & qmask;
      rank_in = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    const uint32_t rank = (lane & 48u) + below + rank_in;
    o_rank = rank;
    const uint32_t geo = pad | ((key != 8u ? J : 0u) << 9) | (dl << 12) | ((len >= 5u ? 1u : 0u) << 14) |
                         ((key != 8u ? 1u : 0u) << 15) | (lane << 16);
    o_ws = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank * 4), (int)(uint32_t)wsrel);
    o_geo = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank * 4), (int)geo);
  };

  // ---- load cursor: sorted records of its super-window (cur) and the next one (nxt) ----
  uint32_t cur_ws = 0, cur_geo = 0, nxt_ws = 0, nxt_geo = 0;
  bool nxt_ready = false;
  uint32_t sw_load = 0;                    // first frame (relative to F0) of the load cursor's super-window
  int set_k = -1;
  uint32_t set_j = 0, set_J = 0, set_flags = 0;
  uint32_t ws_g = 0, geo_g = 0;            // this group's frame in the current set
  uint32_t ld_off = 0, ld_lo = 0, ld_n = 0;  // its loads: offset of block 0, blocks [ld_lo, ld_lo + ld_n)
  bool ended = nf == 0;
  uint64_t qa = 0, qb = 0;                 // prefetched bounds of super-window q_target
  uint32_t q_target = 0xFFFFFFFFu;
  // Slow-frame masks of the super-windows the compute cursor has not reached yet (FIFO).
  // With them, each frame's sorted position (lane l: frame l of the window).
  uint64_t smq0 = 0, smq1 = 0;
  uint32_t rq0 = 0, rq1 = 0;
  uint32_t smq_n = 0;
  auto smq_push = [&](uint64_t m, uint32_t rk) {
    if (smq_n == 0) {
      smq0 = m;
      rq0 = rk;
    } else {
      smq1 = m;
      rq1 = rk;
    }
    smq_n++;
  };
  auto smq_pop = [&](uint32_t& rk) -> uint64_t {
    const uint64_t m = smq0;
    rk = rq0;
    smq0 = smq1;
    rq0 = rq1;
    smq_n--;
    return m;
  };
  if (nf) {  // super-window 0, sorted now; the next one's bounds prefetched
    uint64_t a, b, sm;
    uint32_t rk;
    fetch(0, a, b);
    sort_window(0, a, b, cur_ws, cur_geo, sm, rk);
    smq_push(sm, rk);
    if (64 < nf) {
      fetch(64, qa, qb);
      q_target = 64;
    }
  }

  // Advance the load cursor by one set (straight-line: a set without fast frames costs one empty
  // step; the first set of a super-window is always a valid step, a marker when empty, so the
  // compute cursor sees every crossing).
  auto next_set = [&]() {
    set_j = 0;
    set_J = 0;
    set_flags = 0;
    if (++set_k >= 16) {
      if (sw_load + 64 >= nf) {
        ended = true;
        return;
      }
      if (!nxt_ready) {  // (only after super-windows shorter than kV2Depth steps): an empty step
        set_k = 15;
        return;
      }
      cur_ws = nxt_ws;
      cur_geo = nxt_geo;
      nxt_ready = false;
      sw_load += 64;
      set_k = 0;
    }
    const int src = (4 * set_k + (int)grp) * 4;
    ws_g = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cur_ws);
    geo_g = ((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cur_geo) & ~(63u << 16)) | ((uint32_t)set_k << 16);
    // J of the four frames (0 for slow and dead frames, which sort last)
    const uint32_t j0 = g_J((uint32_t)__builtin_amdgcn_readlane((int)geo_g, 0));
    const uint32_t j1 = g_J((uint32_t)__builtin_amdgcn_readlane((int)geo_g, 16));
    const uint32_t j2 = g_J((uint32_t)__builtin_amdgcn_readlane((int)geo_g, 32));
    const uint32_t j3 = g_J((uint32_t)__builtin_amdgcn_readlane((int)geo_g, 48));
    const uint32_t jmax = max(max(j0, j1), max(j2, j3));
    const uint32_t jmin = min(min(j0, j1), min(j2, j3));
    const bool g1 = __builtin_amdgcn_ballot_w64(g_pad(geo_g) > 256u) != 0;
    {  // this lane's loads: block j at ld_off + 256 j for j in [ld_lo, ld_lo + ld_n)
      const uint32_t Jg = g_J(geo_g), dl = g_dl(geo_g);
      ld_off = ws_g + dl + 16u * col;
      ld_lo = (16u * (col + 1) + dl <= g_pad(geo_g)) ? 1u : 0u;  // 16 bytes wholly before the frame
      ld_n = Jg > ld_lo ? Jg - ld_lo : 0u;
    }
    set_J = jmax;
    set_flags = (set_k == 0 || jmax != 0 ? kStValid : 0u) | (set_k == 0 ? kStFirst : 0u) |
                (jmin != jmax ? kStMixed : 0u) | (g1 ? kStG1 : 0u);
  };

  // ---- compute cursor ----
  Chains ch{0u, 0u, 0u, 0u, 0u};
  uint32_t rp = 0;  // lane 15's last loaded word of the previous block (realignment of lane 0)
  uint32_t acc_crc = 0, acc_ok = 0, prev_crc = 0, prev_ok = 0;  // results: lane l = frame l of the window
  uint32_t cw_rank = 0;                    // sorted position of frame `lane` of the compute cursor's window
  uint32_t cs_sel = 0;                     // the current set's realignment selector (per lane)
  uint32_t cw = 0u - 64u;                  // the compute cursor's super-window
  uint64_t sm_cur = 0, sm_prev = 0;        // their slow frames
  bool flush_pending = false;
  uint32_t fw = 0;                         // the super-window to flush
  // Record results of a set (lane 16 g holds frame g's geometry and results) into acc.
  auto record = [&](uint32_t geo, uint32_t crc, uint32_t ok, uint32_t& acrc, uint32_t& aok) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const uint32_t gg = (uint32_t)__builtin_amdgcn_readlane((int)geo, 16 * g);
      const uint32_t cg = (uint32_t)__builtin_amdgcn_readlane((int)crc, 16 * g);
      const uint32_t og = (uint32_t)__builtin_amdgcn_readlane((int)ok, 16 * g);
      const bool hit = g_live(gg) && lane == g_idx(gg);
      acrc = hit ? cg : acrc;
      aok = hit ? og : aok;
    }
  };
  // Record a set's results (group g's in all its lanes): frame l of the window takes group
  // (rank & 3)'s if it sits in this set.
  auto record_set = [&](uint32_t k, uint32_t crc, uint32_t ok) {
    const int src = (int)(64u * (cw_rank & 3u));  // lane 16 g, byte address
    const uint32_t c = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)crc);
    const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)ok);
    const bool hit = (cw_rank >> 2) == k;
    acc_crc = hit ? c : acc_crc;
    acc_ok = hit ? o : acc_ok;
  };
  // Finish super-window fw: its slow frames byte-wise (four at a time, one per group), then the
  // coalesced result stores.  Runs once per kV2Depth steps at most (outside the unrolled steps).
  auto finish_window = [&]() {
    uint64_t m = sm_prev;
    while (m) {
      uint32_t idx[4];
      uint32_t cnt = 0;
#pragma unroll
      for (int g = 0; g < 4; g++) {
        idx[g] = m ? (uint32_t)__builtin_ctzll(m) : 64u;
        if (m) {
          m &= m - 1;
          cnt++;
        }
      }
      const uint32_t li = idx[grp];
      const bool mine = li < 64u;
      uint64_t a, b;
      bounds(F0 + min(fw + (mine ? li : 0u), nf - 1), a, b);
      const FrameDesc d = make_desc(a, b >= a ? b - a : 0);
      const int nb = max(max(__builtin_amdgcn_readlane(d.J, 0), __builtin_amdgcn_readlane(d.J, 16)),
                         max(__builtin_amdgcn_readlane(d.J, 32), __builtin_amdgcn_readlane(d.J, 48)));
      Chains ce{0u, 0u, 0u, 0u, 0u};
#pragma unroll 1
      for (int blk = 0; blk < nb; blk++) {
        const int bl = min(blk, d.J - 1);
        uint32_t wv[4];
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
          const int o = 256 * bl + 16 * L.col + 4 * bb - d.pad;
          uint32_t v = 0;
#pragma unroll 1
          for (int k = 0; k < 4; k++) {
            const int ob = o + k;
            if (ob >= 0 && ob < (int)d.len) v |= (uint32_t)*as_global<g_u8>(p.bytes + d.start + (uint64_t)ob) << (8 * k);
          }
          wv[bb] = v;
        }
        process_block<true>(L, d, blk, make_uint4(wv[0], wv[1], wv[2], wv[3]), ce);
      }
      const uint32_t crc = ~group_lin(L, ce);
      const uint32_t tr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ce.tr, 0x15F, 0xF, 0xF, false);  // lane 15's
      const uint32_t ok = (d.len >= 5u && __builtin_bswap32(tr) == crc) ? 1u : 0u;
      if (SEAL && mine && L.col == 15 && d.len >= 4u) {
        g_u8w* wp = as_global<g_u8w>(p.wbytes + d.start + d.n);
        wp[0] = (uint8_t)(crc >> 24);
        wp[1] = (uint8_t)(crc >> 16);
        wp[2] = (uint8_t)(crc >> 8);
        wp[3] = (uint8_t)crc;
      }
      const uint32_t geo = (mine ? (1u << 15) : 0u) | (li << 16);  // live + frame index, for record
      record(geo, crc, ok, prev_crc, prev_ok);
      (void)cnt;
    }
    if (sm_prev) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no visible load or store stays pending
    if (fw + lane < nf) {
      const uint64_t f = F0 + fw + lane;
      if (p.crc_out) st_u32_hidden(p.crc_out + f, prev_crc);
      if (!SEAL && p.valid_out) st_u8_hidden_v2(p.valid_out + f, prev_ok);
    }
  };

  // One compute step on a ring entry (data v, per-lane geometry geo, step word st; seal: the frame's
  // window start ws).
  auto compute = [&](const u32x4 v, const uint32_t geo, const uint32_t ws) {
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)geo) >> kStShift;
    if (!(st & kStValid)) return;
    if (st & kStFirst) {  // a new super-window: the previous one is flushed at the next round's start
      if ((int)cw >= 0) {
        flush_pending = true;
        fw = cw;
        sm_prev = sm_cur;
        prev_crc = acc_crc;
        prev_ok = acc_ok;
      }
      cw += 64;
      sm_cur = smq_pop(cw_rank);
      acc_crc = 0;
      acc_ok = 0;
    }
    const uint32_t j = st & 7u, Jset = (st >> 3) & 7u;
    if (Jset == 0) return;  // a marker
#ifdef UFC_V2_LOADS_ONLY  // tuning experiment: the memory side alone
    acc_crc ^= v.x ^ v.y ^ v.z ^ v.w;
    return;
#endif
    uint4 x;
    if (j == 0) cs_sel = 0x03020100u + (4u - g_dl(geo)) * 0x01010101u;
    {  // realign the 4-byte-aligned loads to the frame's right-aligned window
      const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w, 0x121, 0xF, 0xF, false);  // row_ror:1
      const uint32_t prev = (col == 0) ? rp : r1;
      rp = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w, 0x15F, 0xF, 0xF, false);  // row_newbcast:15
      const uint32_t sel = cs_sel;
      x = make_uint4(perm(v.x, prev, sel), perm(v.y, v.x, sel), perm(v.z, v.y, sel), perm(v.w, v.z, sel));
    }
    const uint32_t Jg = g_J(geo);
    if (st & kStMixed) {  // the frame's last block: lane 15's last word is the trailer, CRC'd as zero
      const bool t = col == 15 && j + 1 == Jg;
      ch.tr = t ? x.w : ch.tr;
      x.w = t ? 0u : x.w;
    } else if (j + 1 == Jset) {
      ch.tr = col == 15 ? x.w : ch.tr;
      x.w = col == 15 ? 0u : x.w;
    }
    if (j == 0) {  // block 0: front fix (zeros, then G, before the frame), no table lookups
      const uint4 f = front_fix(x, (int)g_pad(geo) - (int)(16u * col), L.G);
      ch.v0 = f.x;
      ch.v1 = f.y;
      ch.v2 = f.z;
      ch.v3 = f.w;
    } else {
      if (j == 1 && (st & kStG1)) x.x = fix_word(x.x, 256 + (int)(16u * col) - (int)g_pad(geo), L.G);
      const uint32_t n0 = chain_step(L.lds, ch.v0, L.K, x.x);
      const uint32_t n1 = chain_step(L.lds, ch.v1, L.K, x.y);
      const uint32_t n2 = chain_step(L.lds, ch.v2, L.K, x.z);
      const uint32_t n3 = chain_step(L.lds, ch.v3, L.K, x.w);
      if (st & kStMixed) {  // frames whose own blocks are done keep their chains
        const bool act = j < Jg;
        ch.v0 = act ? n0 : ch.v0;
        ch.v1 = act ? n1 : ch.v1;
        ch.v2 = act ? n2 : ch.v2;
        ch.v3 = act ? n3 : ch.v3;
      } else {
        ch.v0 = n0;
        ch.v1 = n1;
        ch.v2 = n2;
        ch.v3 = n3;
      }
    }
    if (j + 1 == Jset) {  // the set's last block: finish its four frames
      const uint32_t crc = ~group_lin(L, ch);
      const uint32_t tr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ch.tr, 0x15F, 0xF, 0xF, false);
      const uint32_t ok = (g_len5(geo) && __builtin_bswap32(tr) == crc) ? 1u : 0u;
      if (SEAL && col >= 12 && g_live(geo)) {  // the BE32 trailer at frame end - 4 + k, one byte per lane
        const uint32_t k = col - 12u;
        st_u8_hidden_v2((uint8_t*)p.wbytes + (base - p.bytes) + (ws + 256u * Jg - 4u + k), crc >> (24 - 8 * k));
      }
      record_set(g_set(geo), crc, ok);
    }
  };

  // ---- rings: slot r holds the load issued D steps ago and its geometry (+ the step word) ----
  u32x4 ring[D];
  uint32_t rgeo[D], rws[SEAL ? D : 1];
#pragma unroll
  for (int i = 0; i < D; i++) {
    ring[i] = (u32x4){0, 0, 0, 0};
    rgeo[i] = 0;
    if (SEAL) rws[i] = 0;
  }
  // One load-cursor step into ring slot r: the next block of the current set (or nothing).
  auto issue = [&](int r) {
    uint32_t gw = 0, voff = kV2Oob;
    if (!ended && set_j >= set_J) next_set();
    if (!ended) {
      const uint32_t j = set_j;
      const uint32_t st = j | (set_J << 3) | (j == 0 ? set_flags : (set_flags & ~kStFirst));
      if (j < set_J) {
        voff = (j - ld_lo < ld_n) ? ld_off + 256u * j : kV2Oob;
#ifdef UFC_V2_NO_LOADS  // tuning experiment: the compute side alone
        voff = kV2Oob;
#endif
      }
      gw = geo_g | (st << kStShift);
      set_j++;
    }
    ring[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff, 0, kV2Aux);
    rgeo[r] = gw;
    if (SEAL) rws[r] = ws_g;
  };
  // Once per round (D steps), outside the unrolled steps: flush the compute cursor's previous
  // super-window, sort the load cursor's next one (bounds prefetched a round ago), prefetch the
  // bounds of the one after.
  auto round_start = [&]() {
    if (flush_pending) {
      finish_window();
      flush_pending = false;
    }
    if (!nxt_ready && q_target == sw_load + 64) {
      uint64_t sm;
      uint32_t rk;
      sort_window(q_target, qa, qb, nxt_ws, nxt_geo, sm, rk);
      smq_push(sm, rk);
      nxt_ready = true;
    }
    const uint32_t t = nxt_ready ? sw_load + 128 : sw_load + 64;
    if (t < nf && t != q_target) {
      fetch(t, qa, qb);
      q_target = t;
    }
  };

  // ---- prologue: the first D steps' loads, then the tables (HBM busy from the start) ----
#pragma unroll
  for (int r = 0; r < D; r++) issue(r);
  stage_store<kV2Waves * 64>(sr, lds);
  // ---- main loop: per step, slot r's load (issued D steps ago) is computed while the load cursor
  // refills the slot; once the cursor has ended, one more round drains the ring ----
  bool drained = false;
  while (!drained) {
    const bool was_ended = ended;
    round_start();
#pragma unroll
    for (int r = 0; r < D; r++) {
      const u32x4 v = ring[r];
      const uint32_t geo = rgeo[r], ws = SEAL ? rws[r] : 0u;
      issue(r);
      compute(v, geo, ws);
    }
    drained = was_ended;
  }
  if (flush_pending) finish_window();
  if ((int)cw >= 0) {  // the last super-window
    flush_pending = true;
    fw = cw;
    sm_prev = sm_cur;
    prev_crc = acc_crc;
    prev_ok = acc_ok;
    finish_window();
  }
}

#define UFC_V2_INST(SEAL, PAIRS) template __global__ void frame_crc_varlen2_kernel<SEAL, PAIRS>(const KernelParams);
UFC_V2_INST(false, false) UFC_V2_INST(true, false) UFC_V2_INST(false, true)
#undef UFC_V2_INST

const void* varlen2_kernel_symbol(bool seal, bool pairs) {
  if (pairs) return seal ? nullptr : (const void*)frame_crc_varlen2_kernel<false, true>;
  return seal ? (const void*)frame_crc_varlen2_kernel<true, false> : (const void*)frame_crc_varlen2_kernel<false, false>;
}

}  // namespace ufc_dev
