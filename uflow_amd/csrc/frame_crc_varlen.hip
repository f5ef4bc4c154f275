// frame_crc_varlen.hip -- lean variable-length frame-CRC kernel for MI355X / gfx950.
//
// The batched CRC gate of Frame::read (src/frame/serial/mod.rs:675-690) and the frame seal
// (src/frame/serial/mod.rs:463-470, src/frame/serial/build.rs:151-159) over a CSR batch: frame i
// is bytes[offsets[i] .. offsets[i+1]).  This is how received datagrams arrive (uflow frames are
// 5..1472 B, src/lib.rs:294) and BASELINE.json config 3 (10M frames of U[64,1500] B).
//
// Same math, LDS tables and wave layout as the fixed-length kernels (frame_crc_dev.hpp); the
// schedule is the lean fixed kernel's with per-frame geometry:
//   * A set is 4 consecutive frames, one per 16-lane group, so neighbouring frames' shared
//     boundary lines are read by one wave within a few instructions.
//   * Frame g loads exactly its J_g 256-byte blocks [start - pad, start + len).  A set always
//     issues 6 block loads, so hipcc's wait counts stay static whatever the mix of lengths: they
//     are raw buffer loads on a per-set resource (scalar base = the set's first frame - 512), and
//     blocks past J_g get an out-of-range offset, which returns zeros without a memory request.
//     (Re-reading a block instead costs its full bytes again: non-temporal lines are not kept.)
//   * Loads are 4-byte aligned: a frame's window [start - pad, start + len) starts anywhere, and a
//     misaligned dwordx4 costs the load path ~15 % (measured).  The window is loaded from its
//     start rounded up to 4 bytes (dl = 0..3 bytes later) and each word is rebuilt with one
//     v_perm_b32 from the loaded word and its predecessor: the lane's previous word, the previous
//     lane's last word (DPP row_ror:1), or for lane 0 the previous block's lane-15 word.  The
//     window's first dl bytes are pad (synthesised anyway); its last dl loaded bytes lie past the
//     frame, so frames ending within 3 bytes of the batch end take the byte path.
//   * The set computes max_g J_g blocks (a uniform branch per block); frame g freezes its chains
//     after block J_g - 1, whose lane-15 last word is its trailer.
//   * Offsets: lane (g, col) loads offsets[4q + g + (col & 1)] (one dwordx2) and swaps with its
//     quad neighbour (DPP), so every lane holds its frame's [start, end).  Scalar loads would be
//     one instruction per set, but they share lgkmcnt with LDS, so every table lookup of the
//     compute would wait for them.  Per step k: read the claim for set k+4, issue the next claim,
//     issue set k+4's offsets, turn set k+2's offsets (issued in step k-2, before set k's data,
//     so this wait never covers set k's data) into its geometry, issue its 6 block loads,
//     compute set k.
//   * Results leave once per run of 16 sets through global stores written as inline asm.  hipcc
//     never sees them, so its wait-count model keeps counting loads only; a store it could see
//     would make every later load wait vmcnt(0), since loads and stores share vmcnt and may
//     complete out of order.  Hidden stores can only make a counted wait stricter (loads return
//     in order), never looser.
//   * Sets the fast path cannot take -- a frame shorter than 4 B or longer than 6 blocks, pad
//     bytes before the buffer, the partial last set -- run byte-wise in the loop (rare: the loads
//     and waits of that branch only drain this wave's pipeline).
#include <type_traits>

#include "frame_crc_dev.hpp"

namespace ufc_dev {


// Per-lane pick between two uniform values by a constant lane mask (v_cndmask_b32).  Written as
// asm: hipcc turns a select chain over the lane's group into an indexed scratch-memory table.
__device__ __forceinline__ uint32_t lane_pick32(uint64_t mask, uint32_t t, uint32_t f) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mask));
  return r;
}
__device__ __forceinline__ uint64_t lane_pick64(uint64_t mask, uint64_t t, uint64_t f) {
  return (uint64_t)lane_pick32(mask, (uint32_t)t, (uint32_t)f) |
         ((uint64_t)lane_pick32(mask, (uint32_t)(t >> 32), (uint32_t)(f >> 32)) << 32);
}
constexpr uint64_t kOddLanes = 0xAAAAAAAAAAAAAAAAull;

// Packed per-lane geometry of one set: pad (bits 0..8), J (bits 9..12), len >= 5 (bit 13),
// realignment dl (bits 14..15).
__device__ __forceinline__ int vl_pad(uint32_t g) { return (int)(g & 511u); }
__device__ __forceinline__ int vl_J(uint32_t g) { return (int)((g >> 9) & 15u); }
// v_perm_b32 selector taking the 4 bytes that start dl bytes before word `hi` of {hi, lo}.
__device__ __forceinline__ uint32_t vl_sel(uint32_t g) { return 0x03020100u + (4u - ((g >> 14) & 3u)) * 0x01010101u; }

// Front fix of a word of block 0 (or word 0 of block 1): d = bytes of the word that precede the
// frame.  Bytes at frame offsets [-4, 0) are G's, below -4 zeros: x' = (x & dm) | pre.
__device__ __forceinline__ uint32_t vl_fix(uint32_t x, int d, uint32_t G) {
  const uint32_t dm = d <= 0 ? 0xFFFFFFFFu : (d < 4 ? (0xFFFFFFFFu << ((uint32_t)(8 * d) & 31u)) : 0u);
  const uint32_t pre = (d > 0 && d < 8) ? (uint32_t)(((uint64_t)G << 32) >> ((64 - 8 * d) & 63)) : 0u;
  return __builtin_amdgcn_bitop3_b32(x, dm, pre, 0xEA);  // (x & dm) | pre
}

struct SetMeta {   // uniform part of a set's geometry
  int Jset;        // max_g J_g
  bool slow;       // byte path
};

constexpr int kVlBlocks = 6;      // fast-path blocks per frame (frames of 4..1532 B)
constexpr uint32_t kVlBias = 512;  // lane offsets are relative to (start of frame 0) - 512
// Raw buffer resource of a set: num_records far above any fast-path offset (< 2^20 + 2^11);
// kVlOob is out of range (the load returns zeros and makes no memory request).
constexpr uint32_t kVlRecords = 0x7FFFFFF0u;
constexpr uint32_t kVlOob = 0x80000000u;
constexpr int kRsrcWord3 = 0x00020000;  // gfx9-family raw buffer descriptor word 3
#ifndef UFC_VL_AUX
#define UFC_VL_AUX 2
#endif
constexpr int kAuxNT = UFC_VL_AUX;      // cache policy bits of the loads: 2 = nt (streaming)
// Sorted sets take default-policy loads: a frame's first and last lines are shared with its
// neighbours, which sorting puts in other sets; nt lines are not kept for them (config 3 FETCH_SIZE:
// 10.0 GB with nt against 8.2 GB for 7.82 GB of frames).

// ABL (tuning builds only; results meaningless): bit 0 = loads + XOR fold, no CRC; bit 1 = CRC of
// register data, no block loads (offsets and geometry kept).
// PAIRS: frame i = bytes[pairs[2i] .. pairs[2i+1]) (p.offsets holds the 2n pairs, p.frame_len the
// buffer's byte length): any gapped layout, e.g. datagrams received into fixed-size slots.
// SCHED: kSchedClaim (sets handed out by a per-workgroup counter) or kSchedBlocked (static: wave
// w takes the 16-set runs w, w + WAVES, w + 2 WAVES, ... of its workgroup's range, so every run of
// results is 64 consecutive frames and leaves with coalesced stores).  WAVES: 8 or 16.
// SORTED: p.offsets holds run-sorted records (sort_runs_kernel): set q takes records 4q..4q+3,
// whose frames share a block count; results go to frame 64 (q / 16) + (record's index in run).
template <bool SEAL, bool PAIRS, int ABL, int SCHED, int WAVES, bool SORTED>
__global__ __launch_bounds__(WAVES * 64) void frame_crc_varlen_kernel(const KernelParams p) {
  constexpr bool DYN = SCHED == kSchedClaim;
  constexpr int kAux = SORTED ? 0 : kAuxNT;
  using OffT = typename std::conditional<SORTED, uint4, uint64_t>::type;
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const StageSet<WAVES * 64> sr = stage_load<WAVES * 64>(p);
  Lane L;
  init_lane(L, lds, p.G);
  constexpr int JM = kVlBlocks;
  const uint64_t nfr = p.nframes;
  // < 2^30 (host chunks launches); sorted: every run's 16 sets, the last run padded
  const uint32_t nsets = SORTED ? (uint32_t)((nfr + kRunFrames - 1) / kRunFrames) * (kRunFrames / 4)
                                : (uint32_t)((nfr + 3) >> 2);
  const uint32_t wpb = WAVES;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q_lo = (uint32_t)((uint64_t)nsets * blockIdx.x / gridDim.x);
  const uint32_t q_end = (uint32_t)((uint64_t)nsets * (blockIdx.x + 1) / gridDim.x);
  uint32_t* ctr = DYN ? p.ctr + blockIdx.x * kCtrWordsPerBlock : nullptr;
  auto claim_issue = [&]() -> uint32_t {
    uint32_t v = 0;
    if (DYN && L.lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  // Claimed: sets 0..3 of each wave are static (lo + wpb*i + wid); the rest are claimed.
  auto claim_set = [&](uint32_t v) -> uint32_t { return q_lo + 4 * wpb + __builtin_amdgcn_readfirstlane(v); };
  // Blocked: the set after q in this wave's sequence (runs of kSetsPerRun consecutive sets).
  auto next_set = [&](uint32_t q) -> uint32_t {
    return ((q - q_lo) % kSetsPerRun == kSetsPerRun - 1) ? q + 1 + (wpb - 1) * kSetsPerRun : q + 1;
  };
  // offsets[4q + g + (col & 1)] (clamped), or pairs[2(4q + g) + (col & 1)]: even lanes get the
  // frame's start, odd lanes its end.
  auto load_off = [&](uint32_t q) -> OffT {
    if constexpr (SORTED) {  // this group's record (the same 16 bytes in its 16 lanes)
      const u32x4 r = *as_global<g_u32x4>((const uint32_t*)p.offsets + 4 * (4 * (uint64_t)min(q, nsets - 1) + L.grp));
      return make_uint4(r.x, r.y, r.z, r.w);
    } else if (PAIRS) {
      const uint64_t f = min(4 * (uint64_t)min(q, nsets - 1) + (uint64_t)L.grp, nfr - 1);
      return *as_global<g_u64>(p.offsets + 2 * f + (uint64_t)(L.col & 1));
    } else {
      const uint64_t i = 4 * (uint64_t)min(q, nsets - 1) + (uint64_t)L.grp + (uint64_t)(L.col & 1);
      return *as_global<g_u64>(p.offsets + (i < nfr ? i : nfr));
    }
  };
  auto frame_bounds = [&](uint64_t f, uint64_t& a, uint64_t& b) {
    a = PAIRS ? p.offsets[2 * f] : p.offsets[f];
    b = PAIRS ? p.offsets[2 * f + 1] : p.offsets[f + 1];
  };
  const uint32_t lane16 = 16u * (uint32_t)L.col;
  // end of the batch's bytes (CSR: the last offset; pairs: the buffer length)
  const uint64_t buf_end =
      PAIRS ? p.frame_len : *as_global<g_u64>((SORTED ? p.offsets_csr : p.offsets) + nfr);

  // Geometry of set q from its offsets: lane offset of block 0 (voff0), packed per-lane geometry,
  // the set's scalar base and uniform meta.  A set that is not live (past the range, or slow)
  // loads nothing (voff0 out of range).
  // (sorted: also the record's index in its run, bits 16..21)
  auto geometry = [&](uint32_t q, OffT mine, const uint8_t*& sbase, uint32_t& voff0, SetMeta& m) -> uint32_t {
    uint64_t a, b, a0;
    bool dead = false;
    uint32_t orig = 0;
    auto lane_u64 = [](uint64_t v, int l) -> uint64_t {
      return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
    };
    if constexpr (SORTED) {
      a = (uint64_t)mine.x | ((uint64_t)mine.y << 32);
      b = a + mine.z;
      dead = (mine.w >> 31) != 0;
      orig = mine.w & 63u;
      // the set's frames are anywhere in their run: base on the lowest start
      a0 = min(min(lane_u64(a, 0), lane_u64(a, 16)), min(lane_u64(a, 32), lane_u64(a, 48)));
    } else {
      const uint32_t lo = (uint32_t)mine, hi = (uint32_t)(mine >> 32);
      const uint32_t plo = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
      const uint32_t phi = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0xB1, 0xF, 0xF, false);
      const uint64_t other = (uint64_t)plo | ((uint64_t)phi << 32);
      a = lane_pick64(kOddLanes, other, mine);
      b = lane_pick64(kOddLanes, mine, other);
      a0 = lane_u64(a, 0);
    }
    const uint64_t len = b - a, rel = a - a0;
    const uint32_t l32 = (uint32_t)min(len, (uint64_t)0x40000000u);
    const uint32_t n = l32 >= 4u ? l32 - 4u : l32;
    const uint32_t J = min((n + 8u + 255u) >> 8, 15u);
    const uint32_t pad = (J * 256u - (n + 4u)) & 511u;
#ifdef UFC_VL_UNALIGNED  // tuning experiment: byte-exact (unaligned) block loads, no realignment
    const uint32_t dl = 0;
#else
    const uint32_t dl = (0u - ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a - pad)) & 3u;
#endif
    const bool bad = dead || l32 < 4u || J > (uint32_t)JM || a < (uint64_t)pad || rel > (1u << 20) || b + 3 > buf_end;
    m.slow = __builtin_amdgcn_ballot_w64(bad) != 0;
    m.Jset = max(max(__builtin_amdgcn_readlane((int)J, 0), __builtin_amdgcn_readlane((int)J, 16)),
                 max(__builtin_amdgcn_readlane((int)J, 32), __builtin_amdgcn_readlane((int)J, 48)));
    const bool live = q < q_end && !m.slow;
    sbase = p.bytes + a0 - kVlBias;
    voff0 = live ? (uint32_t)rel + kVlBias - pad + dl + lane16 : kVlOob;
    return pad | (J << 9) | ((l32 >= 5u ? 1u : 0u) << 13) | (dl << 14) | (orig << 16);
  };
  // Frame index of this lane's group in set q (results are recorded by frame, not by set).
  auto frame_of = [&](uint32_t q, uint32_t geo) -> uint32_t {
    return SORTED ? (q / (kRunFrames / 4)) * kRunFrames + ((geo >> 16) & 63u) : q;
  };
  // The 6 block loads of a set: blocks past the frame's J (and every block of a set that is not
  // live) are out of range.
  auto load_set6 = [&](const uint8_t* sbase, uint32_t voff0, uint32_t geo, ItemBuf<JM>& buf) {
    const int J = vl_J(geo);
    if (ABL & 2) {  // register data derived from the geometry instead of loads
#pragma unroll
      for (int j = 0; j < JM; j++) buf.x[j] = make_uint4(voff0 + j, geo, voff0 ^ geo, (uint32_t)j * J);
      return;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sbase, 0, (int)kVlRecords, kRsrcWord3);
    {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)voff0, 0, kAux);
      buf.x[0] = make_uint4(v.x, v.y, v.z, v.w);
    }
    // Every slot issues its 16-byte load, used or not: a uniform branch around a load makes
    // hipcc's wait counts assume it may be missing (and it then turned the stand-in 4-byte loads
    // tried here into dependent loads behind vmcnt(0)).  Each wave-level load costs the CU ~28
    // cycles of issue even when every lane is out of range (measured).
#pragma unroll
    for (int j = 1; j < JM; j++) {
      const uint32_t vo = (j < J) ? voff0 + 256u * j : kVlOob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, kAux);
      buf.x[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };

  // ---- results: lane (g, col = t) holds frame g of the run's t-th set; qv = q | slow << 30 |
  // valid << 31.  A full run leaves through hidden stores. ----
  uint32_t acc_crc = 0, acc_qv = 0;
  uint32_t t = 0;  // sets in the current run (uniform)
  auto store_run = [&](int cnt) {
    // (sorted: qv holds the frame index; else the set index)
    const uint64_t f = SORTED ? (uint64_t)(acc_qv & 0x3FFFFFFFu) : (uint64_t)(acc_qv & 0x3FFFFFFFu) * 4 + (uint64_t)L.grp;
    if (L.col < cnt && f < nfr && !(acc_qv & 0x40000000u)) {
      if (p.crc_out) st_u32_hidden(p.crc_out + f, acc_crc);
      if (!SEAL && p.valid_out) st_u8_hidden(p.valid_out + f, acc_qv >> 31);
    }
  };
  auto record = [&](uint32_t crc, uint32_t qv) {
    acc_crc = (L.col == (int)t) ? crc : acc_crc;
    acc_qv = (L.col == (int)t) ? qv : acc_qv;
    if (++t == kSetsPerRun) {
      store_run(kSetsPerRun);
      t = 0;
    }
  };
  // Seal: lanes 12..15 of each group write the BE32 CRC into the frame's last 4 bytes (hidden
  // byte stores; the frame's trailer address = sbase + voff0 - dl - 16 col + 256 J - 4).
  auto seal_trailer = [&](const uint8_t* sbase, uint32_t voff0, uint32_t geo, uint32_t crc) {
    if (L.col >= 12) {
      const uint32_t k = (uint32_t)L.col - 12u;
      const uint32_t dl = (geo >> 14) & 3u;
      uint8_t* a = (uint8_t*)p.wbytes + (sbase - p.bytes) + (voff0 - dl - lane16 + 256u * (uint32_t)vl_J(geo) - 4u + k);
      st_u8_hidden(a, crc >> (24 - 8 * k));
    }
  };

  // Fast set: Jset blocks, frame g frozen after its own J_g.
  auto compute = [&](uint32_t geo, int Jset, const ItemBuf<JM>& b) -> uint2 {
    if (ABL & 1) {
      uint32_t f = geo;
#pragma unroll
      for (int j = 0; j < JM; j++) f ^= b.x[j].x ^ b.x[j].y ^ b.x[j].z ^ b.x[j].w;
      return make_uint2(f, f & 1u);
    }
    const int J = vl_J(geo);
    const int d0 = vl_pad(geo) - 16 * L.col;
    const uint32_t sel = vl_sel(geo);
    // Realigned block j: words rebuilt from the loaded words (see the header comment); rp = the
    // previous lane's last loaded word of block j - 1 (row_ror:1), for lane 0.
    uint32_t rp = 0;
    auto realign = [&](const uint4& w) -> uint4 {
#ifdef UFC_VL_UNALIGNED
      return w;
#endif
      const uint32_t r = (uint32_t)__builtin_amdgcn_mov_dpp((int)w.w, 0x121, 0xF, 0xF, false);  // row_ror:1
      const uint32_t prev = (L.col == 0) ? rp : r;
      rp = r;
      return make_uint4(perm(w.x, prev, sel), perm(w.y, w.x, sel), perm(w.z, w.y, sel), perm(w.w, w.z, sel));
    };
    Chains c;
    {
      uint4 x = realign(b.x[0]);
      const bool last = (J == 1);
      c.tr = x.w;
      x.w = (last && L.col == 15) ? 0u : x.w;
      c.v0 = vl_fix(x.x, d0, L.G);
      c.v1 = vl_fix(x.y, d0 - 4, L.G);
      c.v2 = vl_fix(x.z, d0 - 8, L.G);
      c.v3 = vl_fix(x.w, d0 - 12, L.G);
    }
#pragma unroll
    for (int j = 1; j < JM; j++) {
      if (j < Jset) {
        uint4 x = realign(b.x[j]);
        const bool last = (j == J - 1);
        c.tr = last ? x.w : c.tr;
        x.w = (last && L.col == 15) ? 0u : x.w;
        if (j == 1) x.x = vl_fix(x.x, d0 - 256, L.G);
        const uint32_t n0 = chain_step(L.lds, c.v0, L.K, x.x);
        const uint32_t n1 = chain_step(L.lds, c.v1, L.K, x.y);
        const uint32_t n2 = chain_step(L.lds, c.v2, L.K, x.z);
        const uint32_t n3 = chain_step(L.lds, c.v3, L.K, x.w);
        const bool act = j < J;
        c.v0 = act ? n0 : c.v0;
        c.v1 = act ? n1 : c.v1;
        c.v2 = act ? n2 : c.v2;
        c.v3 = act ? n3 : c.v3;
      }
    }
    const uint32_t crc = ~group_lin(L, c);
    const uint32_t tr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c.tr, 0x15F, 0xF, 0xF, false);
    const uint32_t ok = (((geo >> 13) & 1u) && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    return make_uint2(crc, ok);
  };

  // Byte path for set q: loads restricted to each frame, any length; results stored at once,
  // followed by vmcnt(0) so that no visible store stays pending.
  auto slow_set = [&](uint32_t q) {
    uint64_t fr, a, b;
    bool store_ok;
    if constexpr (SORTED) {  // the record again (its ring slot has been reused by now)
      const u32x4 r = *as_global<g_u32x4>((const uint32_t*)p.offsets + 4 * (4 * (uint64_t)q + L.grp));
      a = (uint64_t)r.x | ((uint64_t)r.y << 32);
      b = a + r.z;
      fr = (uint64_t)(q / (kRunFrames / 4)) * kRunFrames + (r.w & 63u);
      store_ok = (r.w >> 31) == 0;
    } else {
      fr = 4 * (uint64_t)q + (uint64_t)L.grp;
      const uint64_t f = fr < nfr ? fr : nfr - 1;
      frame_bounds(f, a, b);
      store_ok = fr < nfr;
    }
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
    const uint32_t ok = (d.len >= 5u && __builtin_bswap32(ce.tr) == crc) ? 1u : 0u;
    if (L.col == 15 && store_ok) {
      if (p.crc_out) *as_global<g_u32w>(p.crc_out + fr) = crc;
      if (!SEAL && p.valid_out) *as_global<g_u8w>(p.valid_out + fr) = (uint8_t)ok;
      if (SEAL && d.len >= 4u) {
        g_u8w* w = as_global<g_u8w>(p.wbytes + d.start + d.n);
        w[0] = (uint8_t)(crc >> 24);
        w[1] = (uint8_t)(crc >> 16);
        w[2] = (uint8_t)(crc >> 8);
        w[3] = (uint8_t)crc;
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  };

  // ---- prologue: static sets 0..3, claims for sets 4 and 5, data of sets 0 and 1 ----
  uint32_t S0, S1, S2, S3, S4 = 0;
  if (DYN) {
    S0 = q_lo + wid;
    S1 = q_lo + wpb + wid;
    S2 = q_lo + 2 * wpb + wid;
    S3 = q_lo + 3 * wpb + wid;
  } else {
    S0 = q_lo + wid * kSetsPerRun;
    S1 = next_set(S0);
    S2 = next_set(S1);
    S3 = next_set(S2);
  }
  uint32_t cX = 0, cY = 0, cZ = 0;
  cY = claim_issue();  // read in step 0 -> set 4 (claimed schedule)
  cZ = claim_issue();  // read in step 1 -> set 5
  ItemBuf<JM> A, B, C;          // data ring: set m in slot m % 3
  OffT O0, O1, O2;              // offsets (sorted: record) ring: set m in slot m % 3
  uint32_t g0, g1, g2;          // per-lane geometry ring
  SetMeta m0, m1, m2;           // uniform meta ring
  uint32_t v0 = 0, v1 = 0, v2 = 0;                               // seal: voff0 ring
  const uint8_t *b0 = p.bytes, *b1 = p.bytes, *b2 = p.bytes;  // seal: scalar base ring
  {
    const OffT o0 = load_off(S0), o1 = load_off(S1);
    O2 = load_off(S2);
    O0 = load_off(S3);
    uint32_t vo;
    const uint8_t* sb;
    g0 = geometry(S0, o0, sb, vo, m0);
    load_set6(sb, vo, g0, A);
    if (SEAL) { b0 = sb; v0 = vo; }
    g1 = geometry(S1, o1, sb, vo, m1);
    load_set6(sb, vo, g1, B);
    if (SEAL) { b1 = sb; v1 = vo; }
  }
  stage_store(sr, lds);

  // One step (see the header comment).  cur/gc/mc: set S0; ro/fill/gf/mf: set S2; wo: set S4.
  auto step = [&](ItemBuf<JM>& cur, uint32_t& gc, SetMeta& mc, const uint8_t*& bc, uint32_t& vc, OffT& ro,
                  OffT& wo, ItemBuf<JM>& fill, uint32_t& gf, SetMeta& mf, const uint8_t*& bf, uint32_t& vf,
                  uint32_t& c_issue, uint32_t& c_read) {
    if (DYN) {
      S4 = claim_set(c_read);
      c_issue = claim_issue();
    } else {
      S4 = next_set(S3);
    }
    wo = load_off(S4);
    {
      const uint8_t* sb;
      uint32_t vo;
      gf = geometry(S2, ro, sb, vo, mf);
      load_set6(sb, vo, gf, fill);
      if (SEAL) { bf = sb; vf = vo; }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (S0 < q_end) {
      if (!mc.slow) {
        const uint2 r = compute(gc, mc.Jset, cur);
        if (SEAL) seal_trailer(bc, vc, gc, r.x);
        record(r.x, frame_of(S0, gc) | (r.y << 31));
      } else {
        slow_set(S0);
        record(0u, S0 | 0x40000000u);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    S0 = S1;
    S1 = S2;
    S2 = S3;
    S3 = S4;
  };
  // O(S_m) sits in slot m % 3: step k reads slot (k+2) % 3 and writes slot (k+4) % 3.
  while (S0 < q_end) {
    step(A, g0, m0, b0, v0, O2, O1, C, g2, m2, b2, v2, cX, cY);
    step(B, g1, m1, b1, v1, O0, O2, A, g0, m0, b0, v0, cY, cZ);
    step(C, g2, m2, b2, v2, O1, O0, B, g1, m1, b1, v1, cZ, cX);
  }
  if (t > 0) store_run((int)t);

  if (DYN) {  // the workgroup's last wave resets the claim counters for the next launch
    // Every claim of this wave has returned (so has been performed) before `done` is counted.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    uint32_t done = 0;
    if (L.lane == 0) done = __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(done) == wpb - 1 && L.lane == 0) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

#define UFC_VL_INST(SC, WV, SO)                                                                    \
  template __global__ void frame_crc_varlen_kernel<false, false, 0, SC, WV, SO>(const KernelParams); \
  template __global__ void frame_crc_varlen_kernel<true, false, 0, SC, WV, SO>(const KernelParams);  \
  template __global__ void frame_crc_varlen_kernel<false, true, 0, SC, WV, SO>(const KernelParams);  \
  template __global__ void frame_crc_varlen_kernel<true, true, 0, SC, WV, SO>(const KernelParams);
#ifdef UFC_TUNING  // round-1 kernels, measured slower than frame_crc_varlen8.hip: A/B builds only
UFC_VL_INST(kSchedClaim, 16, true)
UFC_VL_INST(kSchedClaim, 16, false)
UFC_VL_INST(kSchedBlocked, 8, false)
#endif

const void* varlen_kernel_symbol(bool seal, bool pairs, int abl, int sched, int waves, bool sorted) {
#ifdef UFC_TUNING
  if (!seal && !pairs && (abl == 1 || abl == 2) && !sorted && waves != 12) {
    // A/B: ablations for the schedule/waves pairs (instantiated by taking their addresses)
    const bool blk = sched == kSchedBlocked;
    if (waves == 8)
      return abl == 1 ? (blk ? (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedBlocked, 8, false>
                             : (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedClaim, 8, false>)
                      : (blk ? (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedBlocked, 8, false>
                             : (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedClaim, 8, false>);
    return abl == 1 ? (blk ? (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedBlocked, 16, false>
                           : (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedClaim, 16, false>)
                    : (blk ? (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedBlocked, 16, false>
                           : (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedClaim, 16, false>);
  }
  if (!seal && !pairs && (abl == 1 || abl == 2) && sorted && sched == kSchedClaim && waves == 16)
    return abl == 1 ? (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedClaim, 16, true>
                    : (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedClaim, 16, true>;
  if (!seal && !pairs && (abl == 1 || abl == 2) && !sorted && sched == kSchedClaim && waves == 12)
    return abl == 1 ? (const void*)frame_crc_varlen_kernel<false, false, 1, kSchedClaim, 12, false>
                    : (const void*)frame_crc_varlen_kernel<false, false, 2, kSchedClaim, 12, false>;
  if (!seal && !pairs && abl == 0 && !sorted) {
    if (sched == kSchedClaim && waves == 12) return (const void*)frame_crc_varlen_kernel<false, false, 0, kSchedClaim, 12, false>;
    if (sched == kSchedClaim && waves == 8) return (const void*)frame_crc_varlen_kernel<false, false, 0, kSchedClaim, 8, false>;
    if (sched == kSchedBlocked && waves == 16) return (const void*)frame_crc_varlen_kernel<false, false, 0, kSchedBlocked, 16, false>;
  }
  if (abl != 0) return nullptr;
#define UFC_VL_PICK(SC, WV, SO)                                                          \
  if (sched == SC && waves == WV && sorted == SO) {                                      \
    if (pairs)                                                                           \
      return seal ? (const void*)frame_crc_varlen_kernel<true, true, 0, SC, WV, SO>      \
                  : (const void*)frame_crc_varlen_kernel<false, true, 0, SC, WV, SO>;    \
    return seal ? (const void*)frame_crc_varlen_kernel<true, false, 0, SC, WV, SO>       \
                : (const void*)frame_crc_varlen_kernel<false, false, 0, SC, WV, SO>;     \
  }
  UFC_VL_PICK(kSchedClaim, 16, true)
  UFC_VL_PICK(kSchedClaim, 16, false)
  UFC_VL_PICK(kSchedBlocked, 8, false)
#undef UFC_VL_PICK
#endif  // UFC_TUNING
  return nullptr;
}

// ---- sorted mode pre-pass: one wave per run of 64 frames ----
// Key = the frame's block count J (1..6); 7 = a frame the fast path cannot take (shorter than
// 4 B, longer than 6 blocks); 8 = past the end of the batch.  Stable counting sort by ballots.
template <bool PAIRS>
__global__ __launch_bounds__(256) void sort_runs_kernel(const uint64_t* offsets, uint64_t nframes, uint4* rec) {
  const uint64_t run = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nruns = (nframes + kRunFrames - 1) / kRunFrames;
  if (run >= nruns) return;  // (whole waves)
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t f = run * kRunFrames + lane;
  const bool live = f < nframes;
  uint64_t a = 0, b = 0;
  if (live) {
    a = PAIRS ? offsets[2 * f] : offsets[f];
    b = PAIRS ? offsets[2 * f + 1] : offsets[f + 1];
  }
  const uint64_t len = b >= a ? b - a : 0;
  const uint64_t n4 = len >= 4 ? len - 4 : len;
  const uint64_t J = (n4 + 8 + 255) >> 8;
  const uint32_t key = !live ? 8u : ((len >= 4 && len < 0x40000000ull && J <= (uint64_t)kVlBlocks) ? (uint32_t)J : 7u);
  uint32_t below = 0, rank_in = 0;
#pragma unroll
  for (uint32_t k = 1; k <= 8; k++) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(key == k);
    const uint32_t c = (uint32_t)__builtin_popcountll(m);
    below += (k < key) ? c : 0u;
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    rank_in = (k == key) ? r : rank_in;
  }
  const uint32_t rank = below + rank_in;
  rec[run * kRunFrames + rank] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)min(len, (uint64_t)0xFFFFFFFFu),
                                            lane | (live ? 0u : 0x80000000u));
}

__global__ __launch_bounds__(256) void slots_to_pairs_kernel(const uint32_t* lens, uint64_t stride, uint64_t n,
                                                              uint64_t* pairs) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const uint64_t a = i * stride;
    pairs[2 * i] = a;
    pairs[2 * i + 1] = a + lens[i];
  }
}

int slots_to_pairs(const uint32_t* d_lens, uint64_t stride, uint64_t n, uint64_t* d_pairs, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(slots_to_pairs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     d_lens, stride, n, d_pairs);
  return (int)hipGetLastError();
}

int sort_runs(const uint64_t* offsets, bool pairs, uint64_t nframes, void* records, void* stream) {
  const uint64_t nruns = (nframes + kRunFrames - 1) / kRunFrames;
  if (nruns == 0) return 0;
  const unsigned blocks = (unsigned)((nruns + 3) / 4);
  if (pairs)
    hipLaunchKernelGGL(sort_runs_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, offsets, nframes,
                       (uint4*)records);
  else
    hipLaunchKernelGGL(sort_runs_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, offsets, nframes,
                       (uint4*)records);
  return (int)hipGetLastError();
}

}  // namespace ufc_dev
