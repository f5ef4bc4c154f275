// frame_crc_varlen8.hip -- variable-length frame-CRC kernel with 8 lanes per frame, for MI355X /
// gfx950: BASELINE.json config 3 (10M frames of U[64,1500] B) and the receive path.
//
// The batched CRC gate of Frame::read (src/frame/serial/mod.rs:675-690) and the frame seal
// (serial/mod.rs:463-470, build.rs:151-159) for frame i = bytes[offsets[i] .. offsets[i+1]) (or
// (start, end) pairs).  Same virtual stream as the other kernels (frame_crc_dev.hpp): the frame is
// right-aligned into J 256-byte blocks behind zeros and G.  What differs is the lane layout:
//   * A set is 8 frames, one per 8-lane group.  Lane col of a group loads two 16-byte pieces of
//     each block, at 16 col and 128 + 16 col, so one wave-instruction still reads 128-byte runs and
//     a set's frame loads whole 256-byte blocks.
//   * The two pieces are consecutive 128-byte sub-blocks of one Horner chain per slot: 32 slots
//     (lane col holds slots 4 col + b) with the constant A^128, i.e. V_s <- A^128 V_s ^ word twice
//     per block.  The finish is lin = XOR_s A^(4(31-s)) V_s: 32 slot words per frame instead of
//     64, so the per-frame finish (nibble lookups, the only per-frame LDS work) costs half.  On
//     gfx950 every integer VALU instruction is 4 cycles per wave and the lean varlen kernels are
//     VALU-bound (SQ_ACTIVE_INST_VALU ~ SQ_INSTS_VALU with the SIMD busy all along): per-frame work
//     -- geometry, loads, front fix, finish, results -- is shared by 8 frames instead of 4.
//   * Sets come from run-sorted records (sort_runs, frame_crc_varlen.hip): a run of 64 frames is
//     ordered by block count J, so a set's 8 frames mostly share J (one uniform block loop, no
//     frozen chains); a set mixing block counts freezes the chains of its shorter frames.
//   * Windows end at the frame's end rounded up to 4 bytes, so every load is 4-byte aligned and
//     needs no realignment: the t = 0..3 bytes past the frame are zeroed with the trailer, which
//     multiplies the linear CRC by A^t, undone at the finish with one nibble-table product
//     (A^-t, 8 lookups per frame instead of one v_perm per word and 4 DPP moves per block).
//   * Loads are default-policy raw buffer loads from one resource per wave (the lines a frame
//     shares with its neighbours, which sort into other sets, stay in L2 for them).  Lanes wholly
//     before their frame and blocks past it load nothing (out-of-range offsets).
//   * Results of a run (8 sets x 8 frames) collect in one register pair per lane and leave with
//     hidden stores once per run.  Sets with a frame the fast path cannot take (shorter than 4 B,
//     longer than 6 blocks, at the batch edges, past its end) run byte-wise, in the same loop.
#include "frame_crc_dev.hpp"

namespace ufc_dev {

namespace {

constexpr int kV8Blocks = 6;               // fast path: frames of 4..1532 B
constexpr uint32_t kV8Bias = 0x20000;      // window offsets: relative to the set's base - bias
constexpr uint32_t kV8Oob = 0x80000000u;   // out-of-range offset: zeros, no memory request
constexpr uint32_t kV8Limit = 0x7FF00000u;  // fast-path window offsets stay below this
constexpr int kV8Aux = 0;                  // default cache policy (shared boundary lines)
constexpr uint32_t kNoSet = 0xFFFFFFFFu;   // a wave's set sequence past its last claimed run
// The workgroup's run counter: nibble-image row 127, column 63 (columns 52..63 are never read).
constexpr uint32_t kV8CtrAddr = (127u * 64u + 63u) * 4u;

// Per-lane geometry of a set (one VGPR): pad [0,9), J [9,12), len >= 5 [12], t [13,15) (window
// bytes past the frame), frame index in its run [16,22), past the batch end [22].
__device__ __forceinline__ uint32_t v8_pad(uint32_t g) { return g & 511u; }
__device__ __forceinline__ uint32_t v8_J(uint32_t g) { return (g >> 9) & 7u; }
__device__ __forceinline__ uint32_t v8_t(uint32_t g) { return (g >> 13) & 3u; }
__device__ __forceinline__ uint32_t v8_orig(uint32_t g) { return (g >> 16) & 63u; }

struct Lane8 {
  const char* lds;
  uint32_t lane, col, grp;
  uint32_t K;    // chain-table key (as Lane::K)
  uint32_t K2;   // nibble key: byte i = column*4 of the slot word multiplied in nibble step i
  uint32_t rot;  // group & 3: nibble step i multiplies slot word (i + rot) & 3
  uint32_t G;
};

__device__ __forceinline__ void init_lane8(Lane8& L, char* lds, uint32_t G) {
  L.lds = lds;
  L.lane = threadIdx.x & 63u;
  L.col = L.lane & 7u;
  L.grp = L.lane >> 3;
  L.rot = L.grp & 3u;
  L.G = G;
  const uint32_t c4 = (L.lane & 31u) * 4u;
  L.K = c4 | ((c4 + 128u) << 8) | (1u << 24);
  uint32_t k2 = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) k2 |= ((4u * L.col + ((i + L.rot) & 3u)) * 4u) << (8 * i);  // column = slot
  L.K2 = k2;
}

// lin of the frame held by this 8-lane group (every lane of the group receives it).  The 32 lanes
// of an LDS half-wave read 32 distinct slot columns in every nibble step (rotation by group).
__device__ __forceinline__ uint32_t group_lin8(const Lane8& L, const Chains& c) {
  const bool r1 = (L.rot & 1u) != 0, r2 = (L.rot & 2u) != 0;
  const uint32_t a01 = r1 ? c.v1 : c.v0, a12 = r1 ? c.v2 : c.v1, a23 = r1 ? c.v3 : c.v2, a30 = r1 ? c.v0 : c.v3;
  const uint32_t X0 = r2 ? a23 : a01, X1 = r2 ? a30 : a12, X2 = r2 ? a01 : a23, X3 = r2 ? a12 : a30;
  uint32_t v = xor3(nib_mul<0>(L.lds, X0, L.K2), nib_mul<1>(L.lds, X1, L.K2), nib_mul<2>(L.lds, X2, L.K2)) ^
               nib_mul<3>(L.lds, X3, L.K2);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return v;
}

// Front-fix table in LDS: for p = 0..20 bytes of a 16-byte piece before its frame, the mask M of
// the frame's bytes and the bytes Gs of G placed before them, so that front_fix(x, p, G) =
// (x & M) | Gs (p <= 0: nothing to fix, p >= 20: all zero).  32 bytes per entry, in the unused
// columns 32..39 of the 32-slot nibble image's rows 0..20 (columns 40..51 hold the A^-t tables).
constexpr int kFixEntries = 21;
__device__ __forceinline__ uint32_t fixtab_addr(uint32_t i) { return i * 256u + 128u; }

__device__ __forceinline__ void fixtab_store(char* lds, uint32_t G) {  // threads 0..20, after the staging
  const uint32_t t = threadIdx.x;
  if (t < (uint32_t)kFixEntries) {
    const uint4 m = front_fix(make_uint4(~0u, ~0u, ~0u, ~0u), (int)t, G), g = front_fix(make_uint4(0u, 0u, 0u, 0u), (int)t, G);
    *(uint4*)(lds + fixtab_addr(t)) = make_uint4(m.x & ~g.x, m.y & ~g.y, m.z & ~g.z, m.w & ~g.w);
    *(uint4*)(lds + fixtab_addr(t) + 16) = g;
  }
}

__device__ __forceinline__ uint4 fix_piece(const char* lds, uint4 x, int p) {
  const uint32_t i = (uint32_t)min(max(p, 0), kFixEntries - 1);
  const uint4 m = *(const uint4*)(lds + fixtab_addr(i)), g = *(const uint4*)(lds + fixtab_addr(i) + 16);
  return make_uint4(__builtin_amdgcn_bitop3_b32(x.x, m.x, g.x, 0xEA), __builtin_amdgcn_bitop3_b32(x.y, m.y, g.y, 0xEA),
                    __builtin_amdgcn_bitop3_b32(x.z, m.z, g.z, 0xEA), __builtin_amdgcn_bitop3_b32(x.w, m.w, g.w, 0xEA));
}

__device__ __forceinline__ void chain4(const Lane8& L, Chains& c, uint4 x) {
#if defined(UFC_TUNING) && defined(UFC_V8_ABL) && (UFC_V8_ABL & 1)  // ablation: no chain steps
  c.v0 ^= x.x; c.v1 ^= x.y; c.v2 ^= x.z; c.v3 ^= x.w;
  return;
#endif
  c.v0 = chain_step(L.lds, c.v0, L.K, x.x);
  c.v1 = chain_step(L.lds, c.v1, L.K, x.y);
  c.v2 = chain_step(L.lds, c.v2, L.K, x.z);
  c.v3 = chain_step(L.lds, c.v3, L.K, x.w);
}

// One 256-byte block j of a frame (pieces x0 at 16 col, x1 at 128 + 16 col, window-aligned):
// front fix of block 0 (and of block 1's first word when G straddles into it), trailer capture on
// the frame's last block (in lane 7, the 4 bytes before the window's last t), two A^128 steps.
// FREEZE: chains stop after the frame's own J blocks.
template <bool FREEZE>
__device__ __forceinline__ void block8(const Lane8& L, uint32_t j, uint32_t J, uint32_t pad, uint32_t t, bool g1,
                                       bool last_any, uint4 x0, uint4 x1, Chains& c) {
  if (FREEZE ? (j + 1 == J) : last_any) {
    c.tr = t ? __builtin_amdgcn_alignbyte(x1.w, x1.z, 4u - t) : x1.w;
    if (L.col == 7u) {  // the trailer and the bytes past the frame are CRC'd as zeros
      x1.z &= 0xFFFFFFFFu >> (8u * t);
      x1.w = 0u;
    }
  }
  if (j == 0) {
    const uint4 f0 = fix_piece(L.lds, x0, (int)pad - (int)(16u * L.col));
    x1 = fix_piece(L.lds, x1, (int)pad - 128 - (int)(16u * L.col));
    c.v0 = f0.x;
    c.v1 = f0.y;
    c.v2 = f0.z;
    c.v3 = f0.w;
    chain4(L, c, x1);
    return;
  }
  if (j == 1 && g1) x0.x = fix_word(x0.x, 256 + (int)(16u * L.col) - (int)pad, L.G);
  Chains n = c;
  chain4(L, n, x0);
  chain4(L, n, x1);
  if (FREEZE) {
    const bool act = j < J;
    c.v0 = act ? n.v0 : c.v0;
    c.v1 = act ? n.v1 : c.v1;
    c.v2 = act ? n.v2 : c.v2;
    c.v3 = act ? n.v3 : c.v3;
  } else {
    c.v0 = n.v0;
    c.v1 = n.v1;
    c.v2 = n.v2;
    c.v3 = n.v3;
  }
}

struct Set8Meta {
  uint32_t Jset;  // max J of the set's frames
  bool slow;      // byte path
  bool mixed;     // block counts differ
  bool g1;        // a frame's G straddles into block 1 (pad > 256)
};

template <int J>
struct Buf8 {
  uint4 x[2 * J];
};

}  // namespace

// WAVES waves per workgroup (one workgroup per CU); DEPTH sets per wave in the ring (the set
// computed plus DEPTH - 1 in flight).  p.offsets = the run-sorted records, p.offsets_csr = the
// CSR offsets (nullptr for pairs: p.frame_len = the buffer length, relative offsets < 2^31).
// SORTW: runs are ordered by block count within aligned windows of SORTW frames (64: the whole run;
// 8: no reordering across sets, i.e. each set is 8 consecutive frames).
// GEOR (with INSORT): each run's geometry is computed once per frame, in the frame's own lane,
// before the sort (one frame per lane instead of once per set in each of a group's 8 lanes), and
// the per-set facts (max block count, mixed counts, byte path, G in block 1) once per run with
// half-row DPP reductions and ballots; a set then takes its two words per group with ds_bpermute
// and its set-level bits with one readfirstlane.  Frames the fast path cannot take sort together
// (key 7), so they spoil fewer sets.
template <bool SEAL, bool PAIRS, int WAVES, int DEPTH, bool INSORT, int SORTW = 64, int AUX = kV8Aux, bool GEOR = false>
__global__ __launch_bounds__(WAVES * 64) void frame_crc_varlen8_kernel(const KernelParams p) {
  static_assert(SORTW == 8 || SORTW == 16 || SORTW == 32 || SORTW == 64, "sort window");
  static_assert(!GEOR || INSORT, "per-run geometry needs the in-kernel sort");
  constexpr int JM = kV8Blocks;
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
#ifdef UFC_TUNING
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  Lane8 L;
  init_lane8(L, lds, p.G);
  const uint64_t nfr = p.nframes;
  const uint32_t nruns = (uint32_t)((nfr + kRunFrames - 1) / kRunFrames);
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef UFC_TUNING
  const uint32_t w = blockIdx.x * WAVES + wid;
  uint32_t nk = 0;  // sets this wave computed (timeline dumps)
#endif
  // Schedule: the workgroup owns a contiguous range of runs [WR0, WR1) (8 sets per run of 64
  // frames); wave i takes run WR0 + i first, then claims the next runs one at a time from a
  // counter in LDS (ds_add_rtn: lgkmcnt, not the vmcnt queue of the loads).  With a static run
  // range per wave, the 3 waves of a SIMD finished 400 us apart on config 3 (1200..1620 us: the
  // oldest-first issue priority runs them at different speeds, and the last waves then ran alone
  // with no latency hiding); claimed runs make a CU's waves finish within about one run.
  const uint32_t WR0 = (uint32_t)((uint64_t)nruns * blockIdx.x / gridDim.x);
  const uint32_t WR1 = (uint32_t)((uint64_t)nruns * (blockIdx.x + 1) / gridDim.x);
  uint32_t* const ctr = (uint32_t*)(lds + kV8CtrAddr);
  // The wave's set sequence: sets of run `run`, position `pos` next; kNoSet once the claims fail.
  uint32_t run = WR0 + wid < WR1 ? WR0 + wid : kNoSet, pos = 0;
  bool exhausted = run == kNoSet;

  // ---- INSORT: each run is ordered by block count inside the wave that takes it (replaces the
  // sort_runs pre-pass and its 16-byte records).  Lane i reads frame i's offsets and the lanes'
  // keys are ranked with ballots, as in sort_runs; the run's records then sit in lane = sorted
  // position (SR, pushed with ds_permute) and a set's group takes its record with ds_bpermute.
  // The next run is claimed, and its offsets loaded, one run ahead (raw_a / raw_b).
  const uint64_t* offs = p.offsets;  // INSORT: CSR offsets (n + 1) or (start, end) pairs
  struct SRec {
    uint32_t a_lo, a_hi, len, info;
  };
  SRec SR{0u, 0u, 0u, 0x80000000u};
  auto raw_load = [&](uint32_t r, uint64_t& a, uint64_t& b) {
    const uint64_t f = (uint64_t)(r == kNoSet ? 0u : r) * kRunFrames + L.lane;
    const uint64_t fi = f < nfr ? f : 0u;
    a = *as_global<g_u64>(offs + (PAIRS ? 2 * fi : fi));
    b = *as_global<g_u64>(offs + (PAIRS ? 2 * fi + 1 : fi + 1));
  };
  const uint64_t buf_end = PAIRS ? p.frame_len : *as_global<g_u64>(p.offsets_csr + nfr);
  const bool flat = PAIRS && p.frame_len < (1ull << 31) - (1ull << 20);
  // GEOR: the fast-path geometry of this lane's frame (unsorted), relative to the run's base sb
  // (the run's first frame, or the buffer itself for flat pairs, minus the bias; wave-uniform).
  struct FGeo {
    uint32_t geo, wrel;
    bool bad;
  };
  auto frame_geo = [&](uint64_t a, uint64_t len64, bool live, uint64_t sb) -> FGeo {
    const uint32_t len = (uint32_t)min(len64, (uint64_t)0x40000000u);  // (longer: J > 6, the byte path)
    const uint32_t t = (0u - ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a + len)) & 3u;  // end up to 4 B
    const uint32_t J = (len + t + 4u + 255u) >> 8;
    const uint32_t pad = (J * 256u - len - t) & 511u;
    const uint64_t rel64 = a - sb;
    FGeo g;
    g.wrel = (uint32_t)rel64 - pad;  // window start (4-byte aligned)
    g.bad = !live || len < 4u || J > (uint32_t)JM || a < (uint64_t)pad || a + len + 3 > buf_end ||
            rel64 >= (uint64_t)kV8Limit || rel64 < 512u;
    g.geo = pad | (min(J, 7u) << 9) | ((len >= 5u ? 1u : 0u) << 12) | (t << 13) | (L.lane << 16) |
            ((live ? 0u : 1u) << 22) | ((g.bad ? 1u : 0u) << 23);
    return g;
  };
  auto run_base = [&](uint64_t a) -> uint64_t {
    const uint64_t b0 = flat ? 0u : (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32)) &
                                     ~3ull);
    return b0 - kV8Bias;
  };
  // RAW: permute the raw record (a, len, lane | dead) even in GEOR mode (the byte path's re-sort:
  // the same keys, so the same permutation).
  auto sort_run = [&](uint32_t r, uint64_t a, uint64_t b, SRec& out, bool raw = false) {
    const uint64_t f = (uint64_t)r * kRunFrames + L.lane;
    const bool live = r != kNoSet && f < nfr;
    const uint64_t len = (live && b >= a) ? b - a : 0u;
    const uint64_t n4 = len >= 4 ? len - 4 : len;
    const uint64_t J = (n4 + 8 + 255) >> 8;
    uint32_t key = !live ? 8u : ((len >= 4 && len < 0x40000000ull && J <= (uint64_t)JM) ? (uint32_t)J : 7u);
    FGeo fg{0u, 0u, false};
    uint64_t sb = 0;
    if constexpr (GEOR) {
      sb = run_base(a);
      fg = frame_geo(a, len, live, sb);
      key = !live ? 8u : (fg.bad ? 7u : (uint32_t)J);
    }
    if constexpr (SORTW == 8) {  // sets of consecutive frames: no reordering
      out.a_lo = (uint32_t)a;
      out.a_hi = (uint32_t)(a >> 32);
      out.len = (uint32_t)min(len, (uint64_t)0xFFFFFFFFu);
      out.info = L.lane | (live ? 0u : 0x80000000u);
      return;
    }
    const uint64_t qmask = SORTW == 64 ? ~0ull : (((1ull << SORTW) - 1ull) << (L.lane & ~(uint32_t)(SORTW - 1)));
    uint32_t below = 0, rank_in = 0;
#pragma unroll
    for (uint32_t k = 1; k <= 8; k++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(key == k) & qmask;
      below += (k < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      rank_in = (k == key) ? rk : rank_in;
    }
    const int dst = (int)(((L.lane & ~(uint32_t)(SORTW - 1)) + below + rank_in) * 4u);
    if constexpr (GEOR) {
      if (!raw) {
        // lane = sorted position: per-set facts over each 8-lane half-row, packed into geo bits 24..29
        uint32_t geo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)fg.geo);
        out.a_hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)fg.wrel);
        out.len = (uint32_t)sb;
        out.info = (uint32_t)(sb >> 32);
        const uint32_t Jk = (geo >> 9) & 7u;
        uint32_t jx = Jk, jn = Jk;
        jx = max(jx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jx, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
        jn = min(jn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jn, 0xB1, 0xF, 0xF, false));
        jx = max(jx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jx, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
        jn = min(jn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jn, 0x4E, 0xF, 0xF, false));
        jx = max(jx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jx, 0x141, 0xF, 0xF, false));  // row_half_mirror
        jn = min(jn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)jn, 0x141, 0xF, 0xF, false));
        const uint64_t mbad = __builtin_amdgcn_ballot_w64(((geo >> 23) & 1u) != 0);
        const uint64_t mg1 = __builtin_amdgcn_ballot_w64((geo & 511u) > 256u);
        const uint32_t s8 = L.lane & ~7u;
        const uint32_t slow = ((mbad >> s8) & 0xFFu) != 0 ? 1u : 0u, g1 = ((mg1 >> s8) & 0xFFu) != 0 ? 1u : 0u;
        out.a_lo = geo | (min(jx, (uint32_t)JM) << 24) | ((jx != jn ? 1u : 0u) << 27) | (slow << 28) | (g1 << 29);
        return;
      }
    }
    out.a_lo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)a);
    out.a_hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)(a >> 32));
    out.len = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)min(len, (uint64_t)0xFFFFFFFFu));
    out.info = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(L.lane | (live ? 0u : 0x80000000u)));
  };
  auto take_rec = [&](const SRec& sr, uint32_t q, bool raw = false) -> uint4 {
    const int src = (int)(((q & 7u) * 8u + L.grp) * 4u);
    if (GEOR && !raw)
      return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_lo),
                        (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_hi), sr.len, sr.info);
    return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_lo),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_hi),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.len),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.info));
  };
  uint32_t run_nxt = kNoSet;
  uint64_t raw_a = 0, raw_b = 0;
  auto claim_next = [&]() {
    run_nxt = kNoSet;
    if (!exhausted) {
      uint32_t v = 0;
      if (L.lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      v = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
      if (WR0 + v < WR1) run_nxt = WR0 + v;
      else exhausted = true;
    }
    if constexpr (INSORT) raw_load(run_nxt, raw_a, raw_b);
  };
  auto next_q = [&]() -> uint32_t {
    if (pos == 8u) {
      pos = 0;
      if constexpr (INSORT) {
        run = run_nxt;
        sort_run(run, raw_a, raw_b, SR);
        claim_next();
      } else {
        claim_next();
        run = run_nxt;
      }
    }
    const uint32_t q = run == kNoSet ? kNoSet : run * 8u + pos;
    pos++;
    return q;
  };
  // the wave's first run: offsets first (loads in flight while the tables' loads are issued)
  uint64_t a0 = 0, b0 = 0;
  if constexpr (INSORT) raw_load(run, a0, b0);
  const StageSet<WAVES * 64> sr = stage_load<WAVES * 64>(p);
  if constexpr (INSORT) sort_run(run, a0, b0, SR);
  const uint4* rec = (const uint4*)p.offsets;

  // This group's record of set q (the same 16 bytes in the group's 8 lanes).
  auto load_rec = [&](uint32_t q) -> uint4 {
    if constexpr (INSORT) return take_rec(SR, q);
    const uint32_t qc = q == kNoSet ? 0u : q;  // (no set: reads set 0)
    const u32x4 r = *as_global<g_u32x4>((const uint32_t*)(rec + (uint64_t)qc * 8 + L.grp));
    return make_uint4(r.x, r.y, r.z, r.w);
  };
  // Geometry of the wave's set k from its record: packed per-lane geometry, block-0 piece-0
  // offset, meta, and the set's base (buffer offset of its loads' resource, minus a bias): its
  // group-0 frame's start (CSR: the fast frames of a run lie within 64 x 1.5 KB of each other),
  // or the buffer itself for pairs over less than 2 GB (pairs may come in any order).
  auto geometry = [&](uint32_t q, uint4 r, uint32_t& voff0, Set8Meta& m, uint64_t& sb) -> uint32_t {
    if constexpr (GEOR) {  // r = (geo | set bits, window start, run base lo, hi) from the run's sort
      sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r.z) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r.w) << 32);
      const uint32_t gu = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.x);
      m.Jset = (gu >> 24) & 7u;
      m.mixed = ((gu >> 27) & 1u) != 0;
      m.slow = ((gu >> 28) & 1u) != 0;
      m.g1 = ((gu >> 29) & 1u) != 0;
      const bool live = q != kNoSet && !m.slow;
      voff0 = live ? r.y + 16u * L.col : kV8Oob;
      return r.x & 0x7FFFFFu;
    }
    const uint64_t a = (uint64_t)r.x | ((uint64_t)r.y << 32);
    const uint32_t len = min(r.z, 0x40000000u);  // (longer: J > 6, the byte path)
    const bool dead = (r.w >> 31) != 0;
    const uint32_t t = (0u - ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a + len)) & 3u;  // end up to 4 B
    const uint32_t J = (len + t + 4u + 255u) >> 8;
    const uint32_t pad = (J * 256u - len - t) & 511u;
    sb = flat ? 0u : (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r.x) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r.y) << 32)) & ~3ull);
    sb -= kV8Bias;
    const uint64_t rel64 = a - sb;
    const uint32_t wrel = (uint32_t)rel64 - pad;  // window start (4-byte aligned)
    const bool bad = dead || len < 4u || J > (uint32_t)JM || a < (uint64_t)pad || a + len + 3 > buf_end ||
                     rel64 >= (uint64_t)kV8Limit || rel64 < 512u;
    m.slow = __builtin_amdgcn_ballot_w64(bad) != 0;
    uint32_t jmax = 0, jmin = 7;
#pragma unroll
    for (int g = 0; g < 8; g++) {
      const uint32_t jg = (uint32_t)__builtin_amdgcn_readlane((int)J, 8 * g);
      jmax = max(jmax, jg);
      jmin = min(jmin, jg);
    }
    m.Jset = min(jmax, (uint32_t)JM);
    m.mixed = jmin != jmax;
    m.g1 = __builtin_amdgcn_ballot_w64(pad > 256u) != 0;
    const bool live = q != kNoSet && !m.slow;
    voff0 = live ? wrel + 16u * L.col : kV8Oob;
    return pad | (min(J, 7u) << 9) | ((len >= 5u ? 1u : 0u) << 12) | (t << 13) | ((r.w & 63u) << 16) |
           ((dead ? 1u : 0u) << 22);
  };
  // The set's loads: block j's pieces at voff0 + 256 j (+ 128); pieces wholly before the frame
  // and blocks past it are out of range.
  auto load_set = [&](uint32_t voff0, uint32_t geo, uint64_t sb, Buf8<JM>& b) {
    const uint32_t J = v8_J(geo), pad = v8_pad(geo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bytes + sb), 0, (int)0x7FFFFFF0, 0x00020000);
    // one select per block (the constant part of each offset goes into the instruction's offset
    // field; an out-of-range base stays out of range with it).  Every block's load is issued, past
    // the set's block count too: skipping them under a wave-uniform branch measured 2.29 against
    // 1.52 ms (the compiler's wait counts no longer match, and it waits for everything).
#pragma unroll
    for (int j = 0; j < JM; j++) {
      const uint32_t base = ((uint32_t)j < J) ? voff0 : kV8Oob;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint32_t vo = base;
        if (j == 0) vo = (128u * h + 16u * L.col + 16u <= pad) ? kV8Oob : vo;
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vo + 256u * j + 128u * h), 0, AUX);
        b.x[2 * j + h] = make_uint4(v.x, v.y, v.z, v.w);
      }
    }
  };

  // ---- results of the current run: lane (g, col = t) <- set t's frame g; qv = orig | valid << 31
  uint32_t acc_crc = 0, acc_qv = 0;
  auto record = [&](uint32_t t, uint32_t crc, uint32_t qv) {
    acc_crc = (L.col == t) ? crc : acc_crc;
    acc_qv = (L.col == t) ? qv : acc_qv;
  };
  auto store_run = [&](uint32_t run) {  // hidden stores (see frame_crc_dev.hpp)
    const uint64_t f = (uint64_t)run * kRunFrames + (acc_qv & 63u);
    if (!(acc_qv & 0x40000000u) && f < nfr) {
      if (p.crc_out) st_u32_hidden(p.crc_out + f, acc_crc);
      if (!SEAL && p.valid_out) st_u8_hidden(p.valid_out + f, acc_qv >> 31);
    }
  };
  // A^-t of every group's lin (t from the geometry; the 32-slot image's columns 40 + 3 (g & 3) +
  // t - 1 hold the nibble tables, one copy per group of a half-wave: no bank conflicts).
  auto unshift = [&](uint32_t lin, uint32_t geo) -> uint32_t {
    const uint32_t t = v8_t(geo);
    if (__builtin_amdgcn_ballot_w64(t != 0) == 0) return lin;
    const uint32_t col = 40u + 3u * (L.grp & 3u) + (t ? t - 1u : 0u);
    const uint32_t r = nib_mul<0>(L.lds, lin, col * 4u);
    return t ? r : lin;
  };
  // The result of a set (crc in every lane of a group; trailer word in its lane 7).
  auto finish = [&](uint32_t q, uint32_t geo, const Chains& c, uint32_t voff0, uint64_t sb) {
#if defined(UFC_TUNING) && defined(UFC_V8_ABL) && (UFC_V8_ABL & 2)  // ablation: no slot combine
    const uint32_t crc = ~(c.v0 ^ c.v1 ^ c.v2 ^ c.v3 ^ geo);
#else
    const uint32_t crc = ~unshift(group_lin8(L, c), geo);
#endif
    const uint32_t tr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((L.lane | 7u) * 4u), (int)c.tr);
    const uint32_t ok = (((geo >> 12) & 1u) && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    if (SEAL && L.col == 7u && !((geo >> 22) & 1u)) {  // BE32 trailer: one dword store from lane 7
      // (4-byte aligned when t = 0; otherwise an unaligned dword store, which gfx950's unaligned access
      // mode splits in the memory pipeline: one store instruction per frame instead of four byte stores)
      // (non-temporal trailer stores measured slower: 1.912 against 1.874 ms)
      uint32_t* const ta = (uint32_t*)((uint8_t*)p.wbytes + sb + (voff0 - 16u * L.col + 256u * v8_J(geo) - v8_t(geo) - 4u));
      st_u32_hidden(ta, __builtin_bswap32(crc));
    }
    record(q & 7u, crc, v8_orig(geo) | (ok << 31) | (((geo >> 22) & 1u) << 30));
    if ((q & 7u) == 7u) store_run(q >> 3);
  };

  // Fast set: Jset blocks (uniform), the loaded pieces as they are.
  auto compute = [&](uint32_t q, uint32_t geo, const Set8Meta& m, const Buf8<JM>& b, uint32_t voff0, uint64_t sb) {
    const uint32_t J = v8_J(geo), pad = v8_pad(geo), t = v8_t(geo);
    Chains c{0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < JM; j++) {
      if ((uint32_t)j < m.Jset) {
        if (m.mixed)
          block8<true>(L, (uint32_t)j, J, pad, t, m.g1, false, b.x[2 * j], b.x[2 * j + 1], c);
        else
          block8<false>(L, (uint32_t)j, J, pad, t, m.g1, (uint32_t)j + 1 == m.Jset, b.x[2 * j], b.x[2 * j + 1], c);
      }
    }
    finish(q, geo, c, voff0, sb);
  };

  // Byte path of set q: any lengths, loads restricted to each frame; the same result handling.
  auto slow_set = [&](uint32_t q) {
    uint4 r;
    if constexpr (INSORT) {  // (the run may have left SR: sort it again)
      uint64_t a, b;
      SRec T;
      raw_load(q >> 3, a, b);
      sort_run(q >> 3, a, b, T, true);
      r = take_rec(T, q, true);
    } else {
      r = load_rec(q);
    }
    const uint64_t a = (uint64_t)r.x | ((uint64_t)r.y << 32);
    const bool dead = (r.w >> 31) != 0;
    const uint32_t len = dead ? 0u : r.z;
    const FrameDesc d = make_desc(a, len);
    uint32_t nb = 0;
#pragma unroll
    for (int g = 0; g < 8; g++) nb = max(nb, (uint32_t)__builtin_amdgcn_readlane(d.J, 8 * g));
    Chains c{0u, 0u, 0u, 0u, 0u};
    // Frame bytes [o, o + 16), zeros outside the frame: the five 4-byte-aligned words over them,
    // each loaded only if it holds a frame byte (an aligned word holding a valid byte never
    // crosses a page), realigned and masked to the frame.  All loads independent.
    const uintptr_t f0 = (uintptr_t)p.bytes + (uintptr_t)d.start, f1 = f0 + d.len;
    auto piece = [&](int o) -> uint4 {
      const uintptr_t P = f0 + (intptr_t)o, A = P & ~(uintptr_t)3;
      const uint32_t sh = (uint32_t)(P & 3u);
      uint32_t w[5];
#pragma unroll
      for (int k = 0; k < 5; k++) {
        const uintptr_t ak = A + 4 * k;
        w[k] = (ak < f1 && ak + 4 > f0) ? *as_global<g_u32>((const uint32_t*)ak) : 0u;
      }
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int ob = o + 4 * i;  // frame offset of the word's first byte
        const uint32_t lo = (uint32_t)min(max(-ob, 0), 4), hi = (uint32_t)min(max((int)d.len - ob, 0), 4);
        const uint32_t mhi = hi >= 4u ? ~0u : ((1u << ((8u * hi) & 31u)) - 1u),  // (amounts kept in range)
                       mlo = lo >= 4u ? 0u : (~0u << ((8u * lo) & 31u));
        x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh) & mhi & mlo;
      }
      return make_uint4(x[0], x[1], x[2], x[3]);
    };
#pragma unroll 1
    for (uint32_t j = 0; j < nb; j++) {
      const uint32_t jb = min(j, (uint32_t)d.J - 1u);
      const int o0 = 256 * (int)jb + 16 * (int)L.col - d.pad;
      const uint4 x0 = piece(o0);
      const uint4 x1 = piece(o0 + 128);
      block8<true>(L, j, (uint32_t)d.J, (uint32_t)d.pad, 0u, true, false, x0, x1, c);
    }
    const uint32_t geo = ((d.len >= 5u ? 1u : 0u) << 12) | ((r.w & 63u) << 16) | ((dead ? 1u : 0u) << 22);
    const uint32_t crc = ~group_lin8(L, c);
    const uint32_t tr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((L.lane | 7u) * 4u), (int)c.tr);
    const uint32_t ok = (((geo >> 12) & 1u) && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    if (SEAL && L.col == 7u && !dead && d.len >= 4u) {
      g_u8w* wp = as_global<g_u8w>(p.wbytes + d.start + d.n);
      wp[0] = (uint8_t)(crc >> 24);
      wp[1] = (uint8_t)(crc >> 16);
      wp[2] = (uint8_t)(crc >> 8);
      wp[3] = (uint8_t)crc;
    }
    record(q & 7u, crc, v8_orig(geo) | (ok << 31) | ((dead ? 1u : 0u) << 30));
    if ((q & 7u) == 7u) store_run(q >> 3);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no visible load or store stays pending
  };

  // ---- ring: set S_k in slot k % DEPTH; records DEPTH sets ahead of their geometry ----
  static_assert(DEPTH == 2 || DEPTH == 3, "ring depth");
  Buf8<JM> B[DEPTH];
  uint4 O[DEPTH];
  uint32_t GE[DEPTH], VO[DEPTH], QO[DEPTH], QG[DEPTH];  // set of O[i] / of GE[i], B[i]
  uint64_t SB[DEPTH];
  Set8Meta M[DEPTH];
  // prologue: records of the wave's first 2 DEPTH - 1 sets, geometry + loads of the first
  // DEPTH - 1 (all in the wave's first run, which needs no claim: 2 DEPTH - 1 <= 8)
  uint4 Rq[DEPTH];
  uint32_t Qq[DEPTH];
#pragma unroll
  for (int i = 0; i < DEPTH; i++) {
    Qq[i] = next_q();
    Rq[i] = load_rec(Qq[i]);
  }
#pragma unroll
  for (int i = 0; i < DEPTH - 1; i++) {
    QG[i] = Qq[i];
    GE[i] = geometry(QG[i], Rq[i], VO[i], M[i], SB[i]);
    load_set(VO[i], GE[i], SB[i], B[i]);
    QO[i] = next_q();
    O[i] = load_rec(QO[i]);
  }
  O[DEPTH - 1] = Rq[DEPTH - 1];
  QO[DEPTH - 1] = Qq[DEPTH - 1];
  stage_store<WAVES * 64>(sr, lds);
  fixtab_store(lds, p.G);  // (then an LDS-only barrier, as in stage_store: the prefetches stay in flight)
  // Runs WR0 .. WR0 + WAVES - 1 are taken statically.  (Set by the thread whose stage_store wrote
  // the word, after it: program order, then the barrier below.)
  if (threadIdx.x == 1023u % (WAVES * 64u)) *ctr = WAVES;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#ifdef UFC_TUNING
  const unsigned long long t_staged = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (INSORT) claim_next();  // the second run (the counter is set now)

  // One step: geometry + loads of set S + DEPTH - 1 (record loaded DEPTH steps ago), the record of
  // set S + 2 DEPTH - 1, then compute set S.
  auto step = [&](int cs, int fs) {
    QG[fs] = QO[fs];
    GE[fs] = geometry(QG[fs], O[fs], VO[fs], M[fs], SB[fs]);
    load_set(VO[fs], GE[fs], SB[fs], B[fs]);
    QO[fs] = next_q();
    O[fs] = load_rec(QO[fs]);
    __builtin_amdgcn_sched_barrier(0);
    if (QG[cs] != kNoSet) {
      if (!M[cs].slow)
        compute(QG[cs], GE[cs], M[cs], B[cs], VO[cs], SB[cs]);
      else
        slow_set(QG[cs]);
#ifdef UFC_TUNING
      nk++;
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // (a wave's sets are valid up to its first kNoSet, so a round stops at the first dead set)
  if constexpr (DEPTH == 3) {
    while (QG[0] != kNoSet) {
      step(0, 2);
      step(1, 0);
      step(2, 1);
    }
  } else {
    while (QG[0] != kNoSet) {
      step(0, 1);
      step(1, 0);
    }
  }
#ifdef UFC_TUNING
  if (p.dbg && L.lane == 0) {  // per-wave timeline (tools/wave_timeline.py)
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    unsigned long long* d = p.dbg + 4 * w;
    d[0] = t_start;
    d[1] = t_staged;
    d[2] = t_end;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
    d[3] = (unsigned long long)nk | ((unsigned long long)__smid() << 32) | ((unsigned long long)xcc << 56);
  }
#endif
}

#define UFC_V8_INST(SEAL, PAIRS, IS) \
  template __global__ void frame_crc_varlen8_kernel<SEAL, PAIRS, 12, 2, IS>(const KernelParams);
#define UFC_V8_INSTW(SEAL, SW) \
  template __global__ void frame_crc_varlen8_kernel<SEAL, false, 12, 2, true, SW>(const KernelParams);
#define UFC_V8_INSTA(SW) \
  template __global__ void frame_crc_varlen8_kernel<false, false, 12, 2, true, SW, 2>(const KernelParams);
#define UFC_V8_INSTG(SEAL, PAIRS) \
  template __global__ void frame_crc_varlen8_kernel<SEAL, PAIRS, 12, 2, true, 64, kV8Aux, true>(const KernelParams);
// Product: 12 waves, 2 sets per wave in the ring (three waves per SIMD; config 3 1.69 ms kernel
// against 1.93 ms at 8 waves / depth 3 and 2.4-2.6 ms at 14-16 waves, which spill), runs sorted
// in the kernel with per-run geometry (GEOR: 1.480 against 1.506 ms, config 3, in-process A/B,
// identical results).  Per-set geometry and the pre-sorted variant (records from sort_runs) are
// kept for A/B in tuning builds.
UFC_V8_INSTG(false, false) UFC_V8_INSTG(true, false) UFC_V8_INSTG(false, true) UFC_V8_INSTG(true, true)
#ifdef UFC_TUNING
UFC_V8_INST(false, false, true) UFC_V8_INST(true, false, true) UFC_V8_INST(false, true, true) UFC_V8_INST(true, true, true)
UFC_V8_INST(false, false, false) UFC_V8_INST(true, false, false) UFC_V8_INST(false, true, false) UFC_V8_INST(true, true, false)
UFC_V8_INSTW(false, 8) UFC_V8_INSTW(false, 16) UFC_V8_INSTW(false, 32) UFC_V8_INSTW(true, 8) UFC_V8_INSTW(true, 16)
UFC_V8_INSTW(true, 32) UFC_V8_INSTA(8) UFC_V8_INSTA(16) UFC_V8_INSTA(32) UFC_V8_INSTA(64)
#endif
#undef UFC_V8_INST
#undef UFC_V8_INSTW
#undef UFC_V8_INSTA
#undef UFC_V8_INSTG

const void* varlen8_kernel_symbol(bool seal, bool pairs, bool insort, int sortw, int aux, bool geor) {
  if (geor) {
    if (!insort || sortw != 64 || aux != kV8Aux) return nullptr;
    if (pairs)
      return seal ? (const void*)frame_crc_varlen8_kernel<true, true, 12, 2, true, 64, kV8Aux, true>
                  : (const void*)frame_crc_varlen8_kernel<false, true, 12, 2, true, 64, kV8Aux, true>;
    return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, true, 64, kV8Aux, true>
                : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 64, kV8Aux, true>;
  }
#ifdef UFC_TUNING
  if (insort && !pairs && !seal && aux == 2) {  // A/B: non-temporal loads (CSR validate)
    switch (sortw) {
      case 8: return (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 8, 2>;
      case 16: return (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 16, 2>;
      case 32: return (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 32, 2>;
      case 64: return (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 64, 2>;
      default: return nullptr;
    }
  }
  if (aux != kV8Aux) return nullptr;
  if (insort && !pairs && sortw != 64) {  // A/B: narrower sort windows (CSR)
    switch (sortw) {
      case 8: return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, true, 8>
                          : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 8>;
      case 16: return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, true, 16>
                           : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 16>;
      case 32: return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, true, 32>
                           : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true, 32>;
      default: return nullptr;
    }
  }
  if (insort) {  // per-set geometry (the round-3 product)
    if (pairs)
      return seal ? (const void*)frame_crc_varlen8_kernel<true, true, 12, 2, true>
                  : (const void*)frame_crc_varlen8_kernel<false, true, 12, 2, true>;
    return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, true>
                : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, true>;
  }
  if (pairs)
    return seal ? (const void*)frame_crc_varlen8_kernel<true, true, 12, 2, false>
                : (const void*)frame_crc_varlen8_kernel<false, true, 12, 2, false>;
  return seal ? (const void*)frame_crc_varlen8_kernel<true, false, 12, 2, false>
              : (const void*)frame_crc_varlen8_kernel<false, false, 12, 2, false>;
#else
  return nullptr;
#endif
}

}  // namespace ufc_dev
