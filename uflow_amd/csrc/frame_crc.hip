// frame_crc.hip -- batched frame CRC-32 (uflow, polynomial 0x132c00699) for MI355X / gfx950:
// the generic kernel (any fixed length, CSR fallback) and the lean fixed-length kernel.
// Algorithm, layouts and shared helpers: frame_crc_dev.hpp.
#include "frame_crc_dev.hpp"

namespace ufc_dev {

// Per-run output accumulators: lane i holds the results of frame i of the run.
struct RunAcc {
  uint32_t crc;
  uint32_t valid;
};

// Slot constants + 16-lane XOR -> the frame's CRC (in every lane of its group); validity from the
// trailer (lane 15 of the group); results written into the run accumulators at lanes 4t + g.
// Seal mode writes the trailer here.
template <bool SEAL>
__device__ __forceinline__ void finish_set(const Lane& L, const KernelParams& p, const FrameDesc& d, const Chains& c,
                                           uint64_t set, int t, RunAcc& acc) {
  const uint32_t X0 = L.odd ? c.v2 : c.v0, X1 = L.odd ? c.v3 : c.v1;
  const uint32_t X2 = L.odd ? c.v0 : c.v2, X3 = L.odd ? c.v1 : c.v3;
  uint32_t lin = xor3(nib_mul<0>(L.lds, X0, L.K2), nib_mul<1>(L.lds, X1, L.K2), nib_mul<2>(L.lds, X2, L.K2)) ^
                 nib_mul<3>(L.lds, X3, L.K2);
  lin = row_xor16(lin);
  const uint32_t crc = ~lin;
  if (SEAL) {
    const uint64_t f = set * 4 + (uint64_t)L.grp;
    if (L.col == 15 && f < p.nframes && d.len >= 4u) {
      uint8_t* a = p.wbytes + d.start + d.n;
      if (((uintptr_t)a & 3u) == 0) {
        *as_global<g_u32w>((uint32_t*)a) = __builtin_bswap32(crc);
      } else {
        g_u8w* w = as_global<g_u8w>(a);
        w[0] = (uint8_t)(crc >> 24);
        w[1] = (uint8_t)(crc >> 16);
        w[2] = (uint8_t)(crc >> 8);
        w[3] = (uint8_t)crc;
      }
    }
  }
  const uint32_t ok = (d.len >= 5u && __builtin_bswap32(c.tr) == crc) ? 1u : 0u;
  // gather: frame g of this set -> lane 4t + g of the run accumulators
  const int dst = L.lane - 4 * t;  // in [0, 4) for the 4 lanes receiving this set's results
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const uint32_t cg = __builtin_amdgcn_readlane(crc, 16 * g);
    acc.crc = (dst == g) ? cg : acc.crc;
    if (!SEAL) {
      const uint32_t vg = __builtin_amdgcn_readlane(ok, 16 * g + 15);
      acc.valid = (dst == g) ? vg : acc.valid;
    }
  }
}

// Store a run's results (frames run_first .. run_first + 63, clipped to nframes): one coalesced
// dword store of CRC words and one coalesced byte store of valid flags per wave.
template <bool SEAL>
__device__ __forceinline__ void store_run(const Lane& L, const KernelParams& p, uint64_t run_first, const RunAcc& acc) {
  const uint64_t f = run_first + (uint64_t)L.lane;
  if (f < p.nframes) {
    if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = acc.crc;
    if (!SEAL && p.valid_out) *as_global<g_u8w>(p.valid_out + f) = (uint8_t)acc.valid;
  }
}

// Slow path for one set (edge/tail sets: frames whose fast loads could leave the buffer).  Byte
// loads restricted to [0, len) of the frame, one block at a time, not unrolled, so that it adds no
// register pressure to the fast path.
template <bool SEAL>
__device__ __forceinline__ void slow_set(const Lane& L, const KernelParams& p, const FrameDesc& d, int nblocks,
                                         uint64_t set, int t, RunAcc& acc) {
  Chains c{0u, 0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int blk = 0; blk < nblocks; blk++) {
    const int bl = min(blk, d.J - 1);
    uint32_t w[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int o = 256 * bl + 16 * L.col + 4 * b - d.pad;  // frame offset of the word
      uint32_t a = 0;
#pragma unroll 1
      for (int k = 0; k < 4; k++) {
        const int ob = o + k;
        if (ob >= 0 && ob < (int)d.len) a |= (uint32_t)*as_global<g_u8>(p.bytes + d.start + (uint64_t)ob) << (8 * k);
      }
      w[b] = a;
    }
    process_block<true>(L, d, blk, make_uint4(w[0], w[1], w[2], w[3]), c);
  }
  finish_set<SEAL>(L, p, d, c, set, t, acc);
}


template <int JC>
__device__ __forceinline__ void load_item(const uint8_t* lane_base, int part, ItemBuf<JC>& b) {
  const uint8_t* q = lane_base + (int64_t)part * (JC * 256);
#pragma unroll
  for (int j = 0; j < JC; j++) {
    const u32x4 v = __builtin_nontemporal_load(as_global<g_u32x4>(q + 256 * j));
    b.x[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <int JC, bool FREEZE, bool PART0>
__device__ __forceinline__ void compute_item(const Lane& L, const FrameDesc& d, int part, const ItemBuf<JC>& b,
                                             Chains& c) {
#pragma unroll
  for (int j = 0; j < JC; j++) process_block<FREEZE>(L, d, PART0 ? j : part * JC + j, b.x[j], c);
}

template <int JC, int MODE>
__global__ __launch_bounds__(1024) void frame_crc_kernel(const KernelParams p) {
  constexpr bool VARLEN = (MODE & kModeVarlen) != 0;
  constexpr bool SEAL = (MODE & kModeSeal) != 0;
  constexpr bool FREEZE = VARLEN || (MODE & kModeFreeze) != 0;  // blocks past J may occur in a part
  // Fixed-length frames without freeze: the host picks JC == J, so every set is one part.
  constexpr bool SINGLE = !VARLEN && (MODE & kModeFreeze) == 0;
  // Static LDS (all 160 KiB): its base is the constant 0, so a perm result IS the LDS address (a
  // dynamic-LDS base would cost one v_add per table lookup).
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  stage_tables(p, lds);

  Lane L;
  init_lane(L, lds, p.G);
  const uint64_t nsets = (p.nframes + 3) >> 2;  // 4 frames per set (one per 16-lane group)
  const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
  // Wave-uniform counters, provably uniform (SGPR) so that loop control compiles to scalar
  // branches and no load sits behind an exec mask.
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  // Set sequence of this wave: runs r = w0, w0 + W, ...; run r covers sets [r*R, r*R + R).
  constexpr int R = kSetsPerRun;
  uint64_t run = w0;
  int t = 0;  // set index inside the run
  if (run * R >= nsets) return;
  auto set_of = [&](uint64_t r, int tt) -> uint64_t { return r * R + (uint64_t)tt; };
  // next set in this wave's sequence: advance t, or jump to the next run
  auto next_pos = [&](uint64_t r, int tt, uint64_t& r2, int& t2) {
    if (tt + 1 < R && set_of(r, tt + 1) < nsets) {
      r2 = r;
      t2 = tt + 1;
    } else {
      r2 = r + W;
      t2 = 0;
    }
  };
  const uint64_t buf_end =
      VARLEN ? *as_global<g_u64>(p.offsets + p.nframes) : (p.nframes - 1) * p.stride + p.frame_len;

  auto frame_index = [&](uint64_t set) -> uint64_t {
    const uint64_t f = set * 4 + (uint64_t)L.grp;
    return f < p.nframes ? f : p.nframes - 1;
  };
  auto desc_now = [&](uint64_t set) -> FrameDesc {
    const uint64_t f = frame_index(set);
    if (VARLEN) {
      const uint64_t a = *as_global<g_u64>(p.offsets + f), b = *as_global<g_u64>(p.offsets + f + 1);
      return make_desc(a, b - a);
    }
    return make_desc(f * p.stride, p.frame_len);
  };
  auto wave_max = [&](int v) -> int {
    int m = __builtin_amdgcn_readlane(v, 0);
    m = max(m, __builtin_amdgcn_readlane(v, 16));
    m = max(m, __builtin_amdgcn_readlane(v, 32));
    m = max(m, __builtin_amdgcn_readlane(v, 48));
    return m;
  };
  auto set_parts = [&](const FrameDesc& dd) -> int { return (wave_max(dd.J) + JC - 1) / JC; };
  // Fast loads read [start - pad, start - pad + 256*JC*parts) of every frame: stay in the buffer.
  auto set_slow = [&](const FrameDesc& dd, int parts) -> bool {
    const int bad =
        (dd.start < (uint64_t)dd.pad || dd.start - dd.pad + (uint64_t)(256 * JC) * parts > buf_end) ? 1 : 0;
    return wave_max(bad) != 0;
  };

  RunAcc acc{0u, 0u};
  // After set (r, tt): store the run's results when the run ends.
  auto after_set = [&](uint64_t r, int tt) {
    uint64_t r2;
    int t2;
    next_pos(r, tt, r2, t2);
    if (r2 != r) store_run<SEAL>(L, p, set_of(r, 0) * 4, acc);
  };

  FrameDesc d = desc_now(set_of(run, t));
  int parts = set_parts(d);
  // Edge sets (first sets of the batch) through the slow path.
  while (set_slow(d, parts)) {
    slow_set<SEAL>(L, p, d, parts * JC, set_of(run, t), t, acc);
    after_set(run, t);
    next_pos(run, t, run, t);
    if (set_of(run, t) >= nsets) return;
    d = desc_now(set_of(run, t));
    parts = set_parts(d);
  }

  // ---- fast path: items (set, part) in a 3-deep software pipeline ----
  // Cursor of one item.  valid/slow are wave-uniform.
  struct Cursor {
    uint64_t run;
    int t, part, parts;
    bool valid, slow;
    FrameDesc d;
  };
  // Varlen: offsets of the set after the leading cursor's set, loaded one set ahead.
  uint64_t pre_a = 0, pre_b = 0;
  auto prefetch_offsets = [&](uint64_t r2, int t2) {
    if (VARLEN) {
      const uint64_t s2 = set_of(r2, t2);
      const uint64_t f = frame_index(s2 < nsets ? s2 : 0);
      pre_a = *as_global<g_u64>(p.offsets + f);
      pre_b = *as_global<g_u64>(p.offsets + f + 1);
    }
  };
  // Advance the leading cursor to the next item of the wave's sequence.
  auto advance = [&](Cursor& c) {
    if (!c.valid || c.slow) {
      c.valid = false;
      return;
    }
    if (!SINGLE && c.part + 1 < c.parts) {
      c.part++;
      return;
    }
    uint64_t r2;
    int t2;
    next_pos(c.run, c.t, r2, t2);
    c.run = r2;
    c.t = t2;
    c.part = 0;
    if (set_of(r2, t2) >= nsets) {
      c.valid = false;
      return;
    }
    c.d = VARLEN ? make_desc(pre_a, pre_b - pre_a) : make_desc(frame_index(set_of(r2, t2)) * p.stride, p.frame_len);
    {
      uint64_t r3;
      int t3;
      next_pos(r2, t2, r3, t3);
      prefetch_offsets(r3, t3);
    }
    c.parts = set_parts(c.d);
    c.slow = set_slow(c.d, c.parts);
  };
  auto lane_base = [&](const Cursor& c) -> const uint8_t* { return p.bytes + c.d.start - c.d.pad + 16 * L.col; };

  Cursor C0{run, t, 0, parts, true, false, d};
  {
    uint64_t r2;
    int t2;
    next_pos(run, t, r2, t2);
    prefetch_offsets(r2, t2);
  }
  Cursor C1 = C0;
  advance(C1);
  Cursor C2 = C1;
  advance(C2);
  // A fast load of a cursor that is not a fast item re-reads C0's first part (harmless, in bounds).
  auto load_cursor = [&](const Cursor& c, ItemBuf<JC>& b) {
    const bool ok = c.valid && !c.slow;
    load_item<JC>(ok ? lane_base(c) : lane_base(C0), ok ? c.part : 0, b);
  };

  Chains c{0u, 0u, 0u, 0u, 0u};
  bool go_slow = false;  // the sequence continues with a slow (tail) set
  uint64_t slow_run = 0;
  int slow_t = 0;
  // One pipeline step: issue the loads of C2 into `nxt2` (the buffer of the item computed last
  // step), compute C0 from `cur`, shift the cursors.  Loads are unconditional: a load behind a
  // branch makes the waitcnt pass assume it was skipped and wait for the whole prefetch.
  auto step = [&](ItemBuf<JC>& cur, ItemBuf<JC>& nxt2) -> bool {
    {
      // The prefetch of C2 is spread over the compute of C0, one block load per block of compute,
      // pinned by sched_barrier: a wave that issued all its loads up front would stall at VMEM issue
      // behind the other waves' bursts instead of computing.
      const bool ok = C2.valid && !C2.slow;
      const uint8_t* q = (ok ? lane_base(C2) : lane_base(C0)) + (int64_t)(ok ? C2.part : 0) * (JC * 256);
      const bool p0 = SINGLE || C0.part == 0;
      if (!p0) __builtin_assume(C0.part >= 1);
#pragma unroll
      for (int j = 0; j < JC; j++) {
        const u32x4 v = __builtin_nontemporal_load(as_global<g_u32x4>(q + 256 * j));
        nxt2.x[j] = make_uint4(v.x, v.y, v.z, v.w);
        __builtin_amdgcn_sched_barrier(0);
        if (p0)
          process_block<FREEZE>(L, C0.d, j, cur.x[j], c);
        else
          process_block<FREEZE>(L, C0.d, C0.part * JC + j, cur.x[j], c);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (SINGLE || C0.part + 1 == C0.parts) {
      finish_set<SEAL>(L, p, C0.d, c, set_of(C0.run, C0.t), C0.t, acc);
      after_set(C0.run, C0.t);
    }
    if (!C1.valid) return false;
    if (C1.slow) {
      go_slow = true;
      slow_run = C1.run;
      slow_t = C1.t;
      return false;
    }
    C0 = C1;
    C1 = C2;
    advance(C2);
    return true;
  };
  {
    ItemBuf<JC> X, Y, Z;
    load_cursor(C0, X);
    load_cursor(C1, Y);
    while (step(X, Z) && step(Y, X) && step(Z, Y)) {
    }
  }
  // Tail sets (last of the batch) through the slow path.
  if (go_slow) {
    run = slow_run;
    t = slow_t;
    while (set_of(run, t) < nsets) {
      d = desc_now(set_of(run, t));
      parts = set_parts(d);
      slow_set<SEAL>(L, p, d, parts * JC, set_of(run, t), t, acc);
      after_set(run, t);
      next_pos(run, t, run, t);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Lean kernel for fixed-length frames (frame_len >= 4, J = ceil((frame_len+4)/256) <= 6 blocks,
// known at compile time): the batched gate of BASELINE.json configs 2 and 4.  Each wave owns a
// balanced contiguous range of sets; loop-invariant geometry (front-fix masks, lane offsets) is
// hoisted, set addresses are scalar, results gather with one select per set.  DEPTH sets are in
// flight per wave (DEPTH-1 prefetched while one is computed); the first prefetches are issued
// before the LDS tables are staged so that HBM is busy from the first cycle.
// ---------------------------------------------------------------------------------------------

// Per-workgroup claim counters of the dynamic schedule (kCtrWordsPerBlock words per workgroup,
// one 128-byte line each): [0] = claims handed out, [1] = waves finished.  The last wave of a
// workgroup to finish resets both, so every launch finds them zero (launches of one slot are
// stream-ordered; see ufc_api.cpp).

// LOADV: the main loop's loads, lean_loadv(skip, first, mid, last): `first` / `mid` / `last` = the
// cache-policy bits (buffer-load aux) of block 0, blocks 1..J-2 and block J-1; skip = pieces of block
// 0 wholly before G load nothing (an out-of-range offset: zeros, no memory request; the front fix
// zeroes them anyway).  The lines a frame shares with its neighbours sit in its first and last block.
constexpr int lean_loadv(int skip, int first, int mid, int last) { return skip | first << 1 | mid << 6 | last << 11; }
[[maybe_unused]] constexpr int kLoadvAllNT = lean_loadv(0, kFixAuxNT, kFixAuxNT, kFixAuxNT);  // rounds 1-3 (A/B)
// Product (round 4): default policy for block 0, non-temporal for the rest: 0.2277-0.2289 against
// 0.2372-0.2383 ms per 1M x 1500 B (in-process A/B, identical results; profiles/EXPERIMENTS.md).
constexpr int kLoadvProduct = lean_loadv(0, 0, kFixAuxNT, kFixAuxNT);
template <int J, bool SEAL, int DEPTH, int SCHED, int WAVES, int LOADV = kLoadvProduct>
__global__ __launch_bounds__(WAVES * 64) void frame_crc_fixed_kernel(const KernelParams p) {
  static_assert(DEPTH >= 1 && DEPTH <= 3, "pipeline depth (4 spills at J = 6)");
  static_assert(DEPTH != 1 || SCHED != kSchedClaim, "depth 1: static schedules only");
  constexpr bool DYN = SCHED == kSchedClaim;        // claimed sets (per-workgroup counter)
  constexpr bool ILV = SCHED == kSchedInterleave;   // static: wave i takes lo + i + k * WAVES
  constexpr uint32_t kInc = ILV ? (uint32_t)WAVES : 1u;  // step of a static sequence
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const StageSet<WAVES * 64> sr = stage_load<WAVES * 64>(p);
  Lane L;
  init_lane(L, lds, p.G);

  const uint64_t stride = p.stride;
  const uint32_t len = (uint32_t)p.frame_len;  // >= 4 (host checks)
  const uint32_t n = len - 4u;
  const int pad = J * 256 - (int)len;          // E = len
  const uint32_t nsets = (uint32_t)((p.nframes + 3) >> 2);  // < 2^32 (host chunks launches)
  // The main loop covers the full sets; a partial last set (nframes % 4 frames) is done by the
  // grid's last wave after its loop.  The host guarantees a full set past the edge sets.
  const uint32_t nfull = (uint32_t)(p.nframes >> 2);
  const bool tail = (p.nframes & 3) != 0;
  const uint32_t wpb = WAVES;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t w = blockIdx.x * wpb + wid;  // global wave index
  // Sets before s_fast have a frame whose pad region precedes the buffer: they take the slow path
  // (global wave 0, before its main loop).  front_ok: bytes before the batch are readable (a
  // later chunk of a larger batch), so there are none.  With E = len the fast loads of a frame end exactly at
  // its last byte, so no set at the end of the batch is unsafe.
  const uint32_t s_edge =
      p.front_ok ? 0u : (uint32_t)min(((uint64_t)pad + 4 * stride - 1) / (4 * stride), (uint64_t)nsets);
  // A single edge set (every stride >= 65 B) is loaded on the fast path instead, with clamped
  // addresses and byte shifts (load_edge0 below), when the batch holds at least 16 bytes.
  const bool edge0 = s_edge == 1 && (p.nframes - 1) * stride + len >= 16;
  const uint32_t s_fast = edge0 ? 0u : s_edge;
  const uint32_t nfast = nfull - s_fast;
  // This wave's set sequence q0 < q1 < q2 < ... (strictly increasing, so once one is past `q_end`
  // all later ones are).  Static: a balanced contiguous range per wave.  Dynamic: the workgroup
  // owns a contiguous range; wave i starts with sets lo+i (and lo+16+i at depth 3), then claims
  // the following ones with a per-workgroup counter, so the 16 waves finish together whatever the SIMD arbitration does
  // (oldest-wave-first arbitration otherwise finishes a CU's waves in four staggered groups).
  uint32_t q_lo, q_end, q_cur, q_nx1, q_nx2;
  if (DYN || ILV) {
    q_lo = s_fast + (uint32_t)((uint64_t)nfast * blockIdx.x / gridDim.x);
    q_end = s_fast + (uint32_t)((uint64_t)nfast * (blockIdx.x + 1) / gridDim.x);
    q_cur = q_lo + wid;
    q_nx1 = q_lo + wpb + wid;
  } else {
    const uint32_t NW = gridDim.x * wpb;
    q_lo = s_fast + (uint32_t)((uint64_t)nfast * w / NW);
    q_end = s_fast + (uint32_t)((uint64_t)nfast * (w + 1) / NW);
    q_cur = q_lo;
    q_nx1 = q_lo + 1;
  }
  uint32_t* ctr = DYN ? p.ctr + blockIdx.x * kCtrWordsPerBlock : nullptr;
  // Claim the next set (lane 0 only; no atomic optimizer, see _build.py), consumed later with a
  // counted wait: the claim is issued before a step's prefetch and read after its compute.
  auto claim_issue = [&]() -> uint32_t {
    uint32_t v = 0;  // (initialised: an undefined value would let the compiler drop the lane test)
    if (L.lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  // (the first DEPTH - 1 sets of each wave are static: lo + i, lo + 16 + i)
  auto claim_set = [&](uint32_t v) -> uint32_t {
    return q_lo + (DEPTH - 1) * wpb + __builtin_amdgcn_readfirstlane(v);
  };

  // Loop invariants of this lane.
  const int64_t lane_off = (int64_t)L.grp * (int64_t)stride + 16 * L.col - pad;
  uint32_t dm[4], pre[4];
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int o = 16 * L.col + 4 * b - pad;
    const uint32_t fz = fix_word(0u, o, L.G);           // G/zero part
    const uint32_t f1 = fix_word(0xFFFFFFFFu, o, L.G);  // data mask | G part
    dm[b] = f1 & ~fz;  // data bytes
    pre[b] = fz;
  }
  uint32_t dm1, pre1;
  {
    const int o = 256 + 16 * L.col - pad;
    const uint32_t fz = fix_word(0u, o, L.G), f1 = fix_word(0xFFFFFFFFu, o, L.G);
    dm1 = f1 & ~fz;
    pre1 = fz;
  }
  const uint32_t tmask = (L.col == 15) ? 0u : 0xFFFFFFFFu;  // zero the trailer word in the CRC

  // Results: the current run of 16 finished sets in acc_* (lane (g, col = t) <- crc, and set index
  // | valid << 31, of the run's t-th set, frame g); every 16 sets the run rolls into the history
  // hist_*[0] (uniform branch, 2*RUNS moves).  They leave after the loop: a store inside the loop
  // would make every later load wait vmcnt(0) (loads and stores share vmcnt and may complete out
  // of order).  RUNS: 32 at 8 waves (256 VGPRs per wave), 8 at 16 waves (128).
  constexpr int RUNS = lean_runs(WAVES);
  uint32_t acc_crc = 0, acc_qv = 0;
  uint32_t hist_crc[RUNS], hist_qv[RUNS];
#pragma unroll
  for (int r = 0; r < RUNS; r++) hist_crc[r] = hist_qv[r] = 0;
  uint32_t t = 0, nhist = 0;  // sets in the current run, completed runs held (uniform)
  auto write_trailer = [&](uint64_t f, uint32_t crc) {  // seal: BE32 CRC into the frame's trailer
    uint8_t* a = p.wbytes + f * stride + n;
    if (((uintptr_t)a & 3u) == 0) {
      *as_global<g_u32w>((uint32_t*)a) = __builtin_bswap32(crc);
    } else {
      g_u8w* wp = as_global<g_u8w>(a);
      wp[0] = (uint8_t)(crc >> 24);
      wp[1] = (uint8_t)(crc >> 16);
      wp[2] = (uint8_t)(crc >> 8);
      wp[3] = (uint8_t)crc;
    }
  };
  // Store one run (cnt sets): per lane the CRC word and valid byte of frame 4*q + g; seal mode
  // writes the frames' trailers.
  auto store_run = [&](int cnt, uint32_t crcs, uint32_t qv) {
    const uint64_t f = (uint64_t)(qv & 0x7FFFFFFFu) * 4 + (uint64_t)L.grp;
    if (L.col < cnt && f < p.nframes) {
      if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = crcs;
      if (!SEAL && p.valid_out) *as_global<g_u8w>(p.valid_out + f) = (uint8_t)(qv >> 31);
      if (SEAL) write_trailer(f, crcs);
    }
  };
  auto store_all = [&]() {  // the partial run, then the history
    if (t > 0) store_run((int)t, acc_crc, acc_qv);
#pragma unroll
    for (int r = 0; r < RUNS; r++)
      if ((uint32_t)r < nhist) store_run(kSetsPerRun, hist_crc[r], hist_qv[r]);
  };
  // Finish set q: the trailer word (lane 15 of the frame's row) is broadcast to the row (DPP
  // row_newbcast:15), so every lane of the frame has its validity.  may_overflow: more than
  // 16 * RUNS sets may reach this wave (claimed schedule): a full history is stored first, then
  // vmcnt(0) so that no store stays pending into the loop; the static schedules never overflow
  // inside the loop (host chunking), so their loop has no store.
  auto finish = [&](uint32_t q, const Chains& c, bool may_overflow) {
    const uint32_t crc = ~group_lin(L, c);
    const uint32_t tr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c.tr, 0x15F, 0xF, 0xF, false);
    const uint32_t ok = (len >= 5u && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    acc_crc = (L.col == (int)t) ? crc : acc_crc;
    acc_qv = (L.col == (int)t) ? (q | (ok << 31)) : acc_qv;
    if (++t == kSetsPerRun) {
      if (may_overflow && nhist == RUNS) {
        t = 0;  // (acc_* is about to roll in; store_all must not store it as a partial run)
        store_all();
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
        nhist = 0;
      }
#pragma unroll
      for (int r = RUNS - 1; r > 0; r--) {
        hist_crc[r] = hist_crc[r - 1];
        hist_qv[r] = hist_qv[r - 1];
      }
      hist_crc[0] = acc_crc;
      hist_qv[0] = acc_qv;
      nhist++;
      t = 0;
    }
  };
  // Frame-set processing from a loaded item (J blocks), block by block.
  auto compute_block = [&](uint32_t q, int j, uint4 x, Chains& c) {
    {
      if (j == J - 1) {
        c.tr = x.w;
        x.w &= tmask;
      }
      if (j == 0) {
        c.v0 = (x.x & dm[0]) | pre[0];
        c.v1 = (x.y & dm[1]) | pre[1];
        c.v2 = (x.z & dm[2]) | pre[2];
        c.v3 = (x.w & dm[3]) | pre[3];
      } else {
        if (j == 1) x.x = (x.x & dm1) | pre1;
        c.v0 = chain_step(L.lds, c.v0, L.K, x.x);
        c.v1 = chain_step(L.lds, c.v1, L.K, x.y);
        c.v2 = chain_step(L.lds, c.v2, L.K, x.z);
        c.v3 = chain_step(L.lds, c.v3, L.K, x.w);
      }
    }
  };
  auto compute = [&](uint32_t q, const ItemBuf<J>& b, Chains& c) {
#pragma unroll
    for (int j = 0; j < J; j++) compute_block(q, j, b.x[j], c);
  };
  // Loads of a main-loop set: a wave-uniform set base (SGPRs) plus this lane's loop-invariant
  // 32-bit offset, so no per-set VGPR address arithmetic (whose registers the allocator may take
  // from a pending load, stalling the next prefetch on the previous one).  A set past the range
  // (the final prefetches) re-reads the last full set, which stays L2-resident.
  const uint32_t voff = (uint32_t)(lane_off + 512);  // lane_off >= -259
  auto set_base = [&](uint32_t q) -> const uint8_t* {
    return p.bytes + (uint64_t)(q < q_end ? q : nfull - 1) * 4 * stride - 512;
  };
  // Set 0 when its first frames' pad bytes precede the buffer: pieces that start before the
  // buffer load its first 16 bytes and shift them into place (the bytes before the buffer are
  // pad, masked by the front fix); pieces wholly before it are zeros.  Prologue only.
  auto load_edge0 = [&](ItemBuf<J>& b) {
    const int64_t room = (int64_t)min(p.nframes - 1, (uint64_t)3);
    const int64_t over = (int64_t)L.grp > room ? (int64_t)L.grp - room : 0;
    const int64_t off0 = lane_off - over * (int64_t)stride;
#pragma unroll
    for (int j = 0; j < J; j++) {
      const int64_t off = off0 + 256 * j;
      uint4 v = load_frame16<true>(p.bytes + (off < 0 ? 0 : off));
      if (off < 0) {
        const int64_t d = -off;
        uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32), hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
        if (d >= 16) {
          lo = hi = 0;
        } else if (d >= 8) {
          hi = lo << (8 * (d - 8));
          lo = 0;
        } else {
          hi = (hi << (8 * d)) | (lo >> (64 - 8 * d));
          lo = lo << (8 * d);
        }
        v = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
      }
      b.x[j] = v;
    }
  };
  // lean_loadv skip: this lane's block-0 offset (out of range for a piece wholly before G)
  const uint32_t voff_b0 = ((LOADV & 1) && 16 * L.col + 16 <= pad - 4) ? kFixRecords : voff;
  auto load = [&](uint32_t q, ItemBuf<J>& b) {
    constexpr int kAuxFirst = (LOADV >> 1) & 31, kAuxMid = (LOADV >> 6) & 31, kAuxLast = (LOADV >> 11) & 31;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)set_base(q), 0, (int)kFixRecords, kFixRsrcWord3);
#pragma unroll
    for (int j = 0; j < J; j++) {
      const uint32_t o = (j == 0 ? voff_b0 : voff) + 256u * j;
      u32x4 v;
      if (j == 0)
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, kAuxFirst);
      else if (j == J - 1)
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, kAuxLast);
      else
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, kAuxMid);
      b.x[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // The partial last set: lanes of frames past nframes re-read frame nframes - 1.
  auto load_tail = [&](ItemBuf<J>& b) {
    const int64_t room = (int64_t)(p.nframes - 1 - 4 * (uint64_t)nfull);
    const int64_t over = (int64_t)L.grp > room ? (int64_t)L.grp - room : 0;
    load_set<J>(p.bytes + (uint64_t)nfull * 4 * stride - 512, voff - (uint32_t)(over * (int64_t)stride), b);
  };

  // Prologue: claim (dynamic), first prefetches, then the LDS tables: HBM is busy from the start.
  // Depth 3 keeps q_cur and q_nx1 in flight and loads q_nx2 in the first step; depth 2 keeps
  // q_cur in flight and loads q_nx1 (static in both schedules) in the first step.
  // Claims are read two steps after they are issued (ring cX/cY/cZ): reading a claim waits, in
  // vmcnt order, for every load issued before it, so it must be older than the loads of the set
  // about to be computed.  The prologue issues the claims read in steps 0 and 1.
  ItemBuf<J> A, B, C;
  uint32_t cX = 0, cY = 0, cZ = 0;
  if (DYN) {
    cY = claim_issue();
    cZ = claim_issue();
  }
  if (edge0 && q_cur == 0)
    load_edge0(A);
  else
    load(q_cur, A);
  if (DEPTH == 3) load(q_nx1, B);
  stage_store<WAVES * 64>(sr, lds);
  q_nx2 = (DEPTH == 3 && !DYN) ? q_cur + 2 * kInc : 0;

  // Edge sets [0, s_fast) (the first sets of the batch only): global wave 0, before its main
  // loop (the dynamic schedule rebalances), byte loads restricted to the frame, results stored
  // per set by lane 15 of each group, then an explicit vmcnt(0) so that no store stays pending
  // into the loop.
  if (w == 0 && s_fast > 0) {
#pragma unroll 1
    for (uint32_t e = 0; e < s_fast; e++) {
      FrameDesc d = make_desc(min((uint64_t)e * 4 + (uint64_t)L.grp, p.nframes - 1) * stride, len);
      Chains ce{0u, 0u, 0u, 0u, 0u};
#pragma unroll 1
      for (int blk = 0; blk < J; blk++) {
        uint32_t wv[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int o = 256 * blk + 16 * L.col + 4 * b - d.pad;
          uint32_t a = 0;
#pragma unroll 1
          for (int k = 0; k < 4; k++) {
            const int ob = o + k;
            if (ob >= 0 && ob < (int)d.len) a |= (uint32_t)*as_global<g_u8>(p.bytes + d.start + (uint64_t)ob) << (8 * k);
          }
          wv[b] = a;
        }
        process_block<false>(L, d, blk, make_uint4(wv[0], wv[1], wv[2], wv[3]), ce);
      }
      const uint32_t crc = ~group_lin(L, ce);
      const uint32_t ok = (len >= 5u && __builtin_bswap32(ce.tr) == crc) ? 1u : 0u;
      const uint64_t f = (uint64_t)e * 4 + (uint64_t)L.grp;
      if (L.col == 15 && f < p.nframes) {
        if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = crc;
        if (!SEAL && p.valid_out) *as_global<g_u8w>(p.valid_out + f) = (uint8_t)ok;
        if (SEAL) write_trailer(f, crc);
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  }


  Chains c{0u, 0u, 0u, 0u, 0u};
  // One step: [read the claim issued two steps ago] [issue a claim] [prefetch] [compute +
  // finish the current set if it exists].  Static: the sequence is contiguous.
  auto step = [&](ItemBuf<J>& cur, ItemBuf<J>& fill, uint32_t& c_issue, uint32_t& c_read) {
    uint32_t q_load;
    if (DYN) {
      q_load = claim_set(c_read);
      c_issue = claim_issue();
    } else {
      q_load = (DEPTH == 3) ? q_nx2 : q_nx1;
    }
    load(q_load, fill);
    // Issue the prefetch before the first wait on `cur`: a wave whose data is late must not
    // also hold back its next requests.
    __builtin_amdgcn_sched_barrier(0);
    if (q_cur < q_end) {
      compute(q_cur, cur, c);
      finish(q_cur, c, DYN);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (DEPTH == 3) {
      q_cur = q_nx1;
      q_nx1 = q_load;
      q_nx2 = q_load + kInc;
    } else {
      q_cur = q_load;
      q_nx1 = q_load + kInc;
    }
  };
  // Whole rounds of DEPTH steps with one uniform trip test (no early exits inside a round: they
  // would merge into the loop latch and poison the wait counts at the loop header).  The claim
  // ring rotates with period 3: step j issues into ring[j % 3] and reads ring[(j + 1) % 3].
  if (DEPTH == 1) {  // no prefetch: each wave loads a set, waits, computes (tuning A/B)
    while (q_cur < q_end) {
      compute(q_cur, A, c);
      finish(q_cur, c, false);
      q_cur += kInc;
      load(q_cur, A);
    }
  } else if (DEPTH == 2 && !DYN) {  // static schedules: no claim ring, rounds of two steps
    while (q_cur < q_end) {
      step(A, B, cX, cY);
      step(B, A, cY, cZ);
    }
  } else if (DEPTH == 2) {
    while (q_cur < q_end) {
      step(A, B, cX, cY);
      step(B, A, cY, cZ);
      step(A, B, cZ, cX);
      step(B, A, cX, cY);
      step(A, B, cY, cZ);
      step(B, A, cZ, cX);
    }
  } else {
    while (q_cur < q_end) {
      step(A, C, cX, cY);
      step(B, A, cY, cZ);
      step(C, B, cZ, cX);
    }
  }
  // The partial last set (grid's last wave; before any LDS reuse below), results stored directly.
  if (tail && blockIdx.x == gridDim.x - 1 && wid == wpb - 1) {
    ItemBuf<J> T;
    load_tail(T);
    compute(nfull, T, c);
    const uint32_t crc = ~group_lin(L, c);
    const uint32_t tr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c.tr, 0x15F, 0xF, 0xF, false);
    const uint32_t ok = (len >= 5u && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    const uint64_t f = (uint64_t)nfull * 4 + (uint64_t)L.grp;
    if (L.col == 0 && f < p.nframes) {
      if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = crc;
      if (!SEAL && p.valid_out) *as_global<g_u8w>(p.valid_out + f) = (uint8_t)ok;
      if (SEAL) write_trailer(f, crc);
    }
  }
  if (DYN) {
    store_all();
  } else {
    // Static schedules: the workgroup's waves hold the results of its whole contiguous set range
    // [blo, bhi).  Once every wave is done with the tables, the LDS stages them in frame order and
    // the workgroup writes them with coalesced stores (each wave's own sets are 8 apart: storing
    // them directly scatters 16-byte pieces over many lines at the end of the kernel).
    uint32_t blo = q_lo, bhi = q_end;
    if (!ILV) {
      const uint64_t NW = (uint64_t)gridDim.x * wpb;
      blo = s_fast + (uint32_t)((uint64_t)nfast * (blockIdx.x * wpb) / NW);
      bhi = s_fast + (uint32_t)((uint64_t)nfast * ((blockIdx.x + 1) * wpb) / NW);
    }
    const uint32_t nfr = 4 * (bhi - blo);  // frames of the range (all < nframes)
    uint32_t* lcrc = (uint32_t*)lds;
    uint8_t* lval = (uint8_t*)lds + 4 * nfr;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    auto stage = [&](int cnt, uint32_t crcs, uint32_t qv) {
      if (L.col < cnt) {
        const uint32_t q = qv & 0x7FFFFFFFu;
        const uint32_t pos = (q - blo) * 4 + (uint32_t)L.grp;
        lcrc[pos] = crcs;
        lval[pos] = (uint8_t)(qv >> 31);
      }
    };
    if (t > 0) stage((int)t, acc_crc, acc_qv);
#pragma unroll
    for (int r = 0; r < RUNS; r++)
      if ((uint32_t)r < nhist) stage(kSetsPerRun, hist_crc[r], hist_qv[r]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    const uint64_t f0 = (uint64_t)blo * 4;
    if (p.crc_out)
      for (uint32_t i = threadIdx.x; i < nfr; i += WAVES * 64) *as_global<g_u32w>(p.crc_out + f0 + i) = lcrc[i];
    if (SEAL) {  // the workgroup's trailers in frame order, one burst after its reads, non-temporal
      for (uint32_t i = threadIdx.x; i < nfr; i += WAVES * 64) {
        const uint32_t v = __builtin_bswap32(lcrc[i]);
        uint8_t* a = p.wbytes + (f0 + i) * stride + n;
        if (((uintptr_t)a & 3u) == 0) {
          __builtin_nontemporal_store(v, as_global<g_u32w>((uint32_t*)a));
        } else {
          g_u8w* wp = as_global<g_u8w>(a);
          __builtin_nontemporal_store((uint8_t)v, wp);
          __builtin_nontemporal_store((uint8_t)(v >> 8), wp + 1);
          __builtin_nontemporal_store((uint8_t)(v >> 16), wp + 2);
          __builtin_nontemporal_store((uint8_t)(v >> 24), wp + 3);
        }
      }
    }
    if (!SEAL && p.valid_out) {
      if ((((uintptr_t)(p.valid_out + f0)) & 3u) == 0) {
        for (uint32_t i = threadIdx.x; i < nfr / 4; i += WAVES * 64)
          *as_global<g_u32w>((uint32_t*)(p.valid_out + f0) + i) = ((const uint32_t*)lval)[i];
      } else {
        for (uint32_t i = threadIdx.x; i < nfr; i += WAVES * 64) *as_global<g_u8w>(p.valid_out + f0 + i) = lval[i];
      }
    }
  }

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

// Product configuration: interleaved schedule, 8 waves, depth 2 (measured fastest, DESIGN.md
// section 5.1).  The claimed schedule at 16 waves / depth 3 (the round-1 default) is instantiated
// only in tuning builds (fixed_kernel_symbol, UFC_FIXED_CLAIM16).
#define UFC_INST_FIXED(J)                                                                                  \
  template __global__ void frame_crc_fixed_kernel<J, false, 2, kSchedInterleave, 8>(const KernelParams); \
  template __global__ void frame_crc_fixed_kernel<J, true, 2, kSchedInterleave, 8>(const KernelParams);
UFC_INST_FIXED(1) UFC_INST_FIXED(2) UFC_INST_FIXED(3) UFC_INST_FIXED(4) UFC_INST_FIXED(5) UFC_INST_FIXED(6)


const void* fixed_kernel_symbol(int J, bool seal, int depth, int sched, int waves) {
  if (depth == 2 && sched == kSchedInterleave && waves == 8) {  // the product kernel
    switch (J) {
#define UFC_PICK_FIXED(JJ)                                                                          \
  case JJ:                                                                                          \
    return seal ? (const void*)frame_crc_fixed_kernel<JJ, true, 2, kSchedInterleave, 8>          \
                : (const void*)frame_crc_fixed_kernel<JJ, false, 2, kSchedInterleave, 8>;
      UFC_PICK_FIXED(1) UFC_PICK_FIXED(2) UFC_PICK_FIXED(3) UFC_PICK_FIXED(4) UFC_PICK_FIXED(5) UFC_PICK_FIXED(6)
#undef UFC_PICK_FIXED
      default: return nullptr;
    }
  }
  return nullptr;
}

#define UFC_INST_MODES(JC)                                                                          \
  template __global__ void frame_crc_kernel<JC, 0>(const KernelParams);                             \
  template __global__ void frame_crc_kernel<JC, kModeSeal>(const KernelParams);                     \
  template __global__ void frame_crc_kernel<JC, kModeFreeze>(const KernelParams);                   \
  template __global__ void frame_crc_kernel<JC, kModeFreeze | kModeSeal>(const KernelParams);       \
  template __global__ void frame_crc_kernel<JC, kModeVarlen>(const KernelParams);                   \
  template __global__ void frame_crc_kernel<JC, kModeVarlen | kModeSeal>(const KernelParams);

#define UFC_CONFIGS(X) X(1) X(2) X(3) X(4) X(5) X(6)

UFC_CONFIGS(UFC_INST_MODES)


const void* kernel_symbol(int jc, int mode) {
#define UFC_PICK(JC)                                                                                   \
  if (jc == JC) {                                                                                      \
    switch (mode) {                                                                                    \
      case 0: return (const void*)frame_crc_kernel<JC, 0>;                                            \
      case kModeSeal: return (const void*)frame_crc_kernel<JC, kModeSeal>;                            \
      case kModeFreeze: return (const void*)frame_crc_kernel<JC, kModeFreeze>;                        \
      case kModeFreeze | kModeSeal: return (const void*)frame_crc_kernel<JC, kModeFreeze | kModeSeal>; \
      case kModeVarlen: return (const void*)frame_crc_kernel<JC, kModeVarlen>;                        \
      case kModeVarlen | kModeSeal: return (const void*)frame_crc_kernel<JC, kModeVarlen | kModeSeal>; \
      default: break;                                                                                  \
    }                                                                                                  \
  }
  UFC_CONFIGS(UFC_PICK)
#undef UFC_PICK
  return nullptr;
}

bool config_available(int jc) { return jc >= 1 && jc <= 6; }

// Seal, second pass: frame i's BE32 CRC into its trailer at i * stride + n_off.  Non-temporal
// stores, in frame order, after the whole batch has been read: measured (tools/probes/
// scatterprobe.hip, 1M x 1500 B) the stream read plus this pass take 0.277 ms, against 0.336 ms
// for the same trailer writes interleaved with the read stream (each scattered write then costs
// a DRAM read/write turnaround) and 0.334 ms for default-policy stores here (their dirty lines
// are evicted into the next read stream).
namespace {
__global__ __launch_bounds__(256) void seal_scatter_kernel(uint8_t* bytes, uint64_t stride, uint64_t n_off,
                                                           uint64_t nframes, const uint32_t* crc) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nframes; i += (uint64_t)gridDim.x * 256) {
    const uint32_t v = __builtin_bswap32(crc[i]);
    uint8_t* a = bytes + i * stride + n_off;
    if (((uintptr_t)a & 3u) == 0) {
      __builtin_nontemporal_store(v, (uint32_t*)a);
    } else {
      __builtin_nontemporal_store((uint8_t)v, a);
      __builtin_nontemporal_store((uint8_t)(v >> 8), a + 1);
      __builtin_nontemporal_store((uint8_t)(v >> 16), a + 2);
      __builtin_nontemporal_store((uint8_t)(v >> 24), a + 3);
    }
  }
}
}  // namespace

int seal_scatter(uint8_t* bytes, uint64_t stride, uint64_t frame_len, uint64_t nframes, const uint32_t* crc,
                 void* stream) {
  if (nframes == 0) return 0;
  const uint64_t blocks = std::min<uint64_t>((nframes + 255) / 256, 1u << 20);
  hipLaunchKernelGGL(seal_scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, bytes, stride,
                     frame_len - 4, nframes, crc);
  return (int)hipGetLastError();
}

}  // namespace ufc_dev
