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
//   * Sets come from sorted runs: the wave that takes a run of 64 frames orders it by block count J
//     (ballot ranks), so a set's 8 frames mostly share J (one uniform block loop, no frozen
//     chains); a set mixing block counts freezes the chains of its shorter frames.
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
#include <type_traits>

#include "frame_crc_dev.hpp"

namespace ufc_dev {

namespace {

constexpr int kV8Pieces = 13;              // fast path: windows of up to 13 lines (frames of 4..1532 B)
constexpr int kV8Split = 7;                // slots 0 .. 6 in a set's first load part, 7 .. 12 and 1 in its second
constexpr uint32_t kV8Bias = 0x20000;      // window offsets: relative to the run's base - bias
constexpr uint32_t kV8Oob = 0x80000000u;   // out-of-range offset: zeros, no memory request
constexpr uint32_t kV8Limit = 0x7FF00000u;  // fast-path window offsets stay below this
constexpr int kV8AuxShared = 0;            // a frame's first and last line: default policy (shared)
constexpr int kV8AuxInterior = 2;          // the lines in between: non-temporal (read once)
constexpr uint32_t kNoSet = 0xFFFFFFFFu;   // a wave's set sequence past its last claimed run
// The workgroup's run counter: nibble-image row 127, column 63 (columns 52..63 are never read).
constexpr uint32_t kV8CtrAddr = (127u * 64u + 63u) * 4u;

// Per-lane geometry of a frame on the fast path (one VGPR): r = (frame start - 4) mod 128 [0,7) (the
// window starts at the 128-byte line holding G's first byte, r bytes before it), len [7,18), index
// in its run [18,24); then the set's facts, the same in every lane of the set: Pmax = its frames' most
// lines, 0 for a byte-path set [24,28), plim = lines 0 .. plim-1 hold CRC'd data only in every frame
// [28,32).  The trailer's first byte lies at window offset zo = len + r; lines P = ceil((zo + 4) / 128).
__device__ __forceinline__ uint32_t w_r(uint32_t g) { return g & 127u; }
__device__ __forceinline__ uint32_t w_len(uint32_t g) { return (g >> 7) & 2047u; }
__device__ __forceinline__ uint32_t w_zo(uint32_t g) { return w_len(g) + w_r(g); }
__device__ __forceinline__ uint32_t w_P(uint32_t g) { return (w_zo(g) + 131u) >> 7; }
__device__ __forceinline__ uint32_t w_orig(uint32_t g) { return (g >> 18) & 63u; }

struct Lane8 {
  const char* lds;
  uint32_t lane, col, grp;
  uint32_t K;    // chain-table key (as Lane::K)
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
}

// lin of the frame held by this 8-lane group (every lane of the group receives it).  The 32 lanes
// of an LDS half-wave read 32 distinct slot columns in every nibble step (rotation by group).
__device__ __forceinline__ uint32_t group_lin8(const Lane8& L, const Chains& c) {
  const bool r1 = (L.rot & 1u) != 0, r2 = (L.rot & 2u) != 0;
  const uint32_t a01 = r1 ? c.v1 : c.v0, a12 = r1 ? c.v2 : c.v1, a23 = r1 ? c.v3 : c.v2, a30 = r1 ? c.v0 : c.v3;
  const uint32_t X0 = r2 ? a23 : a01, X1 = r2 ? a30 : a12, X2 = r2 ? a01 : a23, X3 = r2 ? a12 : a30;
  uint32_t K2 = 0;  // byte i = column*4 of the slot word multiplied in nibble step i (column = slot)
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) K2 |= ((4u * L.col + ((i + L.rot) & 3u)) * 4u) << (8 * i);
  uint32_t v = xor3(nib_mul<0>(L.lds, X0, K2), nib_mul<1>(L.lds, X1, K2), nib_mul<2>(L.lds, X2, K2)) ^
               nib_mul<3>(L.lds, X3, K2);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return v;
}

// The same with the slot constants rotated for a stream whose last word is slot e: slot s's last
// word then lies (e - s) mod 32 words before the stream's end, so it takes the constant of column
// (s + 31 - e) mod 32; nibble step i multiplies slot word (i + u) & 3 with u = (group - (31 - e)) & 3,
// so a half-wave's 32 lanes still read 32 distinct columns (bank = column).
__device__ __forceinline__ uint32_t group_lin8_rot(const Lane8& L, const Chains& c, uint32_t e) {
  const uint32_t R = 31u - e;
  const uint32_t u = (L.rot - R) & 3u;
  const bool r1 = (u & 1u) != 0, r2 = (u & 2u) != 0;
  const uint32_t a01 = r1 ? c.v1 : c.v0, a12 = r1 ? c.v2 : c.v1, a23 = r1 ? c.v3 : c.v2, a30 = r1 ? c.v0 : c.v3;
  const uint32_t X0 = r2 ? a23 : a01, X1 = r2 ? a30 : a12, X2 = r2 ? a01 : a23, X3 = r2 ? a12 : a30;
  const uint32_t K2 = rot_nibble_key(L.col, u, e);
  uint32_t v = xor3(nib_mul<0>(L.lds, X0, K2), nib_mul<1>(L.lds, X1, K2), nib_mul<2>(L.lds, X2, K2)) ^
               nib_mul<3>(L.lds, X3, K2);
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
  c.v0 = chain_step(L.lds, c.v0, L.K, x.x);
  c.v1 = chain_step(L.lds, c.v1, L.K, x.y);
  c.v2 = chain_step(L.lds, c.v2, L.K, x.z);
  c.v3 = chain_step(L.lds, c.v3, L.K, x.w);
}

// One line of a frame whose stream may end inside it: lim = bytes of the lane's 16 before the end of
// the CRC'd data.  Words before the frame's end (the data's and the trailer's) step their slots,
// the trailer's bytes and those past the data as zeros; words past the frame's end do not step.
__device__ __forceinline__ void chain4_masked(const Lane8& L, Chains& c, uint4 x, int lim) {
  const uint32_t n0 = chain_step(L.lds, c.v0, L.K, x.x & data_mask(lim));
  const uint32_t n1 = chain_step(L.lds, c.v1, L.K, x.y & data_mask(lim - 4));
  const uint32_t n2 = chain_step(L.lds, c.v2, L.K, x.z & data_mask(lim - 8));
  const uint32_t n3 = chain_step(L.lds, c.v3, L.K, x.w & data_mask(lim - 12));
  c.v0 = lim > -4 ? n0 : c.v0;
  c.v1 = lim > 0 ? n1 : c.v1;
  c.v2 = lim > 4 ? n2 : c.v2;
  c.v3 = lim > 8 ? n3 : c.v3;
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
  uint32_t Pmax;  // most lines of the set's frames
  uint32_t plim;  // lines 0 .. plim-1 hold CRC'd data only, in every frame of the set
  bool slow;      // byte path
};

// A set's loads: slot 0 = line 0, slot 1 = the frame's last line, slot k >= 2 = line k - 1; tr =
// the trailer (4 bytes at zo).
struct Buf13 {
  uint4 x[kV8Pieces];
  uint32_t tr = 0;
};

}  // namespace

// One workgroup of kV8Waves waves per CU, 2 sets per wave in the ring (the set computed plus one in
// flight).  p.offsets = the CSR offsets (n + 1) or, with PAIRS, the (start, end) pairs (p.frame_len =
// the buffer length).  Each run of 64 frames is ordered by block count in the wave that takes it,
// after each frame's fast-path geometry has been computed in the frame's own lane; the per-set
// facts (max block count, mixed counts, byte path, G in block 1) come once per run from half-row
// DPP reductions and ballots, and a set takes its two words per group with ds_bpermute and its
// set-level bits with one readfirstlane.  Frames the fast path cannot take sort together (key 7),
// so they spoil fewer sets.
constexpr int kV8Waves = 12;
template <bool SEAL, bool PAIRS>
__global__ __launch_bounds__(kV8Waves * 64) void frame_crc_varlen8_kernel(const KernelParams p) {
  constexpr int WAVES = kV8Waves;
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  Lane8 L;
  init_lane8(L, lds, p.G);
  const uint64_t nfr = p.nframes;
  const uint32_t nruns = (uint32_t)((nfr + kRunFrames - 1) / kRunFrames);
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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

  // ---- Each run is ordered by block count inside the wave that takes it: lane i reads frame i's
  // offsets, the lanes' keys are ranked with ballots, the run's per-frame words then sit in lane =
  // sorted position (SR, pushed with ds_permute) and a set's group takes them with ds_bpermute.  The
  // next run is claimed, and its offsets loaded, one run ahead (raw_a / raw_b).
  const uint64_t* offs = p.offsets;
  // A sorted run: lane = sorted position.  Fast path: a_lo = geometry | set facts, a_hi = window start,
  // sb = the run base (wave-uniform).  Raw (the byte path): a_lo, a_hi = frame start, len, info = index
  // | dead.
  struct SRec {
    uint32_t a_lo, a_hi, len, info;
    uint64_t sb;
  };
  SRec SR{0u, 0u, 0u, 0x80000000u, 0u};
  auto raw_load = [&](uint32_t r, uint64_t& a, uint64_t& b) {
    const uint64_t f = (uint64_t)(r == kNoSet ? 0u : r) * kRunFrames + L.lane;
    const uint64_t fi = f < nfr ? f : 0u;
    a = *as_global<g_u64>(offs + (PAIRS ? 2 * fi : fi));
    b = *as_global<g_u64>(offs + (PAIRS ? 2 * fi + 1 : fi + 1));
  };
  const bool flat = PAIRS && p.frame_len < (1ull << 31) - (1ull << 20);
  // The fast-path geometry of this lane's frame (unsorted), relative to the run's base sb (the run's
  // first frame, or the buffer itself for flat pairs, minus the bias; wave-uniform).  The window runs
  // from the 128-byte line holding G's first byte (4 bytes before the frame) to the line holding the
  // frame's last byte: every load is one whole line, and the lines a frame shares with its
  // neighbours are its first and its last.  (A window may end past the buffer, inside the buffer's
  // last line: that line's page holds the buffer's last byte.)
  struct FGeo {
    uint32_t geo, wrel;
    bool bad;
  };
  auto frame_geo = [&](uint64_t a, uint64_t len64, bool live, uint64_t sb) -> FGeo {
    const uint32_t len = (uint32_t)min(len64, (uint64_t)0x40000000u);  // (longer: past 13 lines, the byte path)
    const uint32_t r = ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a - 4u) & 127u;
    const uint32_t zo = len + r;  // the trailer's first byte: (a + len - 4) - (a - 4 - r)
    const uint32_t P = (zo + 131u) >> 7;
    const uint64_t rel64 = a - sb;
    FGeo g;
    g.wrel = (uint32_t)rel64 - 4u - r;  // window start (128-byte aligned in memory)
    g.bad = !live || len < 4u || P > (uint32_t)kV8Pieces || a < 4u + r || rel64 >= (uint64_t)kV8Limit || rel64 < 512u;
    g.geo = r | (min(len, 2047u) << 7) | (L.lane << 18);
    return g;
  };
  auto run_base = [&](uint64_t a) -> uint64_t {
    const uint64_t b0 = flat ? 0u : (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32)) &
                                     ~3ull);
    return b0 - kV8Bias;
  };
  // Each run's frames ranked by key = pieces P (1..13), 14 = byte path, 15 = past the batch end.
  // RAW: permute the raw record (a, len, lane | dead) instead of the geometry (the byte path's
  // re-sort: the same keys, so the same permutation).
  auto sort_run = [&](uint32_t r, uint64_t a, uint64_t b, SRec& out, bool raw = false) {
    const uint64_t f = (uint64_t)r * kRunFrames + L.lane;
    const bool live = r != kNoSet && f < nfr;
    const uint64_t len = (live && b >= a) ? b - a : 0u;
    const uint64_t sb = run_base(a);
    const FGeo fg = frame_geo(a, len, live, sb);
    const uint32_t key = !live ? 15u : (fg.bad ? 14u : w_P(fg.geo));  // (a set with a dead frame: byte path)
    uint32_t below = 0, rank_in = 0;
#pragma unroll
    for (uint32_t k = 1; k <= 15; k++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(key == k);
      below += (k < key) ? (uint32_t)__builtin_popcountll(m) : 0u;
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      rank_in = (k == key) ? rk : rank_in;
    }
    const int dst = (int)((below + rank_in) * 4u);
    if (!raw) {
      // lane = sorted position: per-set facts over each 8-lane half-row, into geo bits 24..31
      const uint32_t geo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)fg.geo);
      const uint32_t bad = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(key >= 14u ? 1u : 0u));
      out.a_hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)fg.wrel);
      out.sb = sb;
      uint32_t px = w_P(geo), zn = w_zo(geo) >> 7;
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
      zn = min(zn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)zn, 0xB1, 0xF, 0xF, false));
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
      zn = min(zn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)zn, 0x4E, 0xF, 0xF, false));
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0x141, 0xF, 0xF, false));  // row_half_mirror
      zn = min(zn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)zn, 0x141, 0xF, 0xF, false));
      const uint64_t mbad = __builtin_amdgcn_ballot_w64(bad != 0u);
      const bool slow = ((mbad >> (L.lane & ~7u)) & 0xFFu) != 0;
      out.a_lo = (geo & 0xFFFFFFu) | ((slow ? 0u : min(px, 15u)) << 24) | (min(zn, 15u) << 28);
      return;
    }
    out.a_lo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)a);
    out.a_hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)(a >> 32));
    out.len = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)min(len, (uint64_t)0xFFFFFFFFu));
    out.info = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(L.lane | (live ? 0u : 0x80000000u)));
  };
  // The raw words of this group's frame of set q (the same in the group's 8 lanes): start lo, hi,
  // length, index | dead.
  auto take_raw = [&](const SRec& sr, uint32_t q) -> uint4 {
    const int src = (int)(((q & 7u) * 8u + L.grp) * 4u);
    return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_lo),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_hi),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.len),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.info));
  };
  // Set q's words: geometry | set facts and window start (the same in the group's 8 lanes), the run
  // base (wave-uniform: scalar registers).
  struct Rec {
    uint32_t geo, wrel;
    uint64_t sb;
  };
  auto take_rec = [&](const SRec& sr, uint32_t q) -> Rec {
    const int src = (int)(((q & 7u) * 8u + L.grp) * 4u);
    return Rec{(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_lo),
               (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)sr.a_hi), sr.sb};
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
    raw_load(run_nxt, raw_a, raw_b);
  };
  auto next_q = [&]() -> uint32_t {
    if (pos == 8u) {
      pos = 0;
      run = run_nxt;
      sort_run(run, raw_a, raw_b, SR);
      claim_next();
    }
    const uint32_t q = run == kNoSet ? kNoSet : run * 8u + pos;
    pos++;
    return q;
  };
  // the wave's first run: offsets first (loads in flight while the tables' loads are issued)
  uint64_t a0 = 0, b0 = 0;
  raw_load(run, a0, b0);
  const StageSet<WAVES * 64> sr = stage_load<WAVES * 64>(p);
  sort_run(run, a0, b0, SR);

  auto load_rec = [&](uint32_t q) -> Rec { return take_rec(SR, q); };
  // Geometry of set q from its words: per-lane geometry, the lane's line-0 offset, the set facts, the
  // run base (the buffer offset of the loads' resource, minus a bias: the run's first frame's start,
  // or the buffer itself for flat pairs).
  auto geometry = [&](uint32_t q, const Rec& r, uint32_t& voff0, Set8Meta& m, uint64_t& sb) -> uint32_t {
    sb = r.sb;
    const uint32_t gu = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.geo);
    m.Pmax = (gu >> 24) & 15u;
    m.plim = gu >> 28;
    m.slow = m.Pmax == 0u;
    const bool live = q != kNoSet && !m.slow;
    voff0 = live ? r.wrel + 16u * L.col : kV8Oob;
    return r.geo;
  };
  // The set's loads (struct Buf13): slots 0 and 1, the lines the frame shares with its neighbours
  // (which the sort puts in other sets), with default policy so that they stay in L2 for them; the
  // lines in between, each read by this set alone, non-temporal; lanes wholly before G, lines past the
  // frame's own and a frame's second slot when it has one line are out of range (zeros, no request).
  // Then the trailer, one dword at zo.
  // Issued in two parts (PART 0: slots 0 and 2 .. kV8Split - 1 and the trailer; PART 1: the rest), the
  // second in the middle of the previous set's compute, once its first lines' registers are free.
  auto load_set = [&](uint32_t voff0, uint32_t geo, uint64_t sb, Buf13& b, auto part) {
    constexpr int PART = decltype(part)::value;
    const uint32_t P = w_P(geo), front = w_r(geo) + 4u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bytes + sb), 0, (int)0x7FFFFFF0, 0x00020000);
    if constexpr (PART == 0) {
      const uint32_t vo = (16u * L.col + 16u <= front) ? kV8Oob : voff0;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, kV8AuxShared);
      b.x[0] = make_uint4(v.x, v.y, v.z, v.w);
    }
#pragma unroll
    for (int k = PART == 0 ? 2 : kV8Split; k < (PART == 0 ? kV8Split : kV8Pieces); k++) {  // line k - 1
      const uint32_t vo = (uint32_t)k + 1u <= P ? voff0 : kV8Oob;  // (an out-of-range base stays out of range)
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vo + 128u * (uint32_t)(k - 1)), 0, kV8AuxInterior);
      b.x[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
    if constexpr (PART == 0) {
      if constexpr (!SEAL) {
        const uint32_t vt = voff0 == kV8Oob ? kV8Oob : voff0 - 16u * L.col + w_zo(geo);
        b.tr = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)vt, 0, kV8AuxShared);
      }
    } else {
      const uint32_t vo = P >= 2u ? voff0 + 128u * (P - 1u) : kV8Oob;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, 0, kV8AuxShared);
      b.x[1] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  using Part0 = std::integral_constant<int, 0>;
  using Part1 = std::integral_constant<int, 1>;

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
  // A^-t of every group's lin (the 32-slot image's columns 40 + 3 (g & 3) + t - 1 hold the nibble
  // tables, one copy per group of a half-wave: no bank conflicts).
  auto unshift = [&](uint32_t lin, uint32_t t) -> uint32_t {
    if (__builtin_amdgcn_ballot_w64(t != 0) == 0) return lin;
    const uint32_t col = 40u + 3u * (L.grp & 3u) + (t ? t - 1u : 0u);
    const uint32_t r = nib_mul<0>(L.lds, lin, col * 4u);
    return t ? r : lin;
  };

  // Fast set.  The stream of a frame is its window with the bytes before G zeroed, G, the data, the
  // trailer as zeros, up to the end of the word holding the frame's last byte (e: that word's slot,
  // t = 0..3 bytes past the frame in it): lin = A^t (register after the data), undone at the finish.
  // Line order: slot 0 (line 0), slots 2.. (lines 1 .. P-2), slot 1 (line P-1); lines past a frame's
  // own step nothing (masked), so every frame's slots see its lines in order.
  auto compute = [&](uint32_t q, uint32_t geo, const Set8Meta& m, const Buf13& b, uint32_t voff0, uint64_t sb, auto mid) {
    const uint32_t zo = w_zo(geo), P = w_P(geo), front = w_r(geo) + 4u;
    const int lim0 = (int)zo - (int)(16u * L.col);
    Chains c{0u, 0u, 0u, 0u, 0u};
    {  // line 0: zeros before G, G, the frame's first bytes
      const uint4 x = fix_piece(L.lds, b.x[0], (int)front - (int)(16u * L.col));
      if (m.plim >= 1u) {
        c.v0 = x.x;
        c.v1 = x.y;
        c.v2 = x.z;
        c.v3 = x.w;
      } else {
        c.v0 = x.x & data_mask(lim0);
        c.v1 = x.y & data_mask(lim0 - 4);
        c.v2 = x.z & data_mask(lim0 - 8);
        c.v3 = x.w & data_mask(lim0 - 12);
      }
    }
#pragma unroll
    for (int j = 1; j < kV8Pieces - 1; j++) {  // line j from slot j + 1
      if (j + 1 == kV8Split) {  // slots 2 .. kV8Split - 1 consumed: the next set's second part
        __builtin_amdgcn_sched_barrier(0);
        mid();
        __builtin_amdgcn_sched_barrier(0);
      }
      uint4 x = b.x[j + 1];
      if (j == 1) x.x = fix_word(x.x, 128 + (int)(16u * L.col) - (int)front, L.G);  // G's last bytes (r >= 125)
      if ((uint32_t)j < m.plim)
        chain4(L, c, x);
      else if ((uint32_t)j + 1u < m.Pmax)
        chain4_masked(L, c, x, (uint32_t)j + 1u < P ? lim0 - 128 * j : -4);
    }
    if (m.Pmax >= 2u) {  // the last line (a one-line frame: no step)
      uint4 x = b.x[1];
      if (P == 2u) x.x = fix_word(x.x, 128 + (int)(16u * L.col) - (int)front, L.G);
      chain4_masked(L, c, x, P >= 2u ? lim0 - 128 * (int)(P - 1u) : -4);
    }
    const uint32_t e = ((zo + 3u) >> 2) & 31u, t = (0u - zo) & 3u;
    const uint32_t crc = ~unshift(group_lin8_rot(L, c, e), t);
    const uint32_t ok = (!SEAL && w_len(geo) >= 5u && __builtin_bswap32(b.tr) == crc) ? 1u : 0u;
    if (SEAL && L.col == 0u) {  // BE32 trailer: one (unaligned) dword store per frame
      // (non-temporal trailer stores measured slower: 1.912 against 1.874 ms)
      uint32_t* const ta = (uint32_t*)((uint8_t*)p.wbytes + sb + (voff0 + zo));
      st_u32_hidden(ta, __builtin_bswap32(crc));
    }
    record(q & 7u, crc, w_orig(geo) | (ok << 31));
    if ((q & 7u) == 7u) store_run(q >> 3);
  };

  // Byte path of set q: any lengths, loads restricted to each frame; the same result handling.
  auto slow_set = [&](uint32_t q) {
    uint4 r;
    {  // (the run may have left SR: sort it again)
      uint64_t a, b;
      SRec T;
      raw_load(q >> 3, a, b);
      sort_run(q >> 3, a, b, T, true);
      r = take_raw(T, q);
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
      for (int i = 0; i < 4; i++)  // (o + 4 i: the frame offset of the word's first byte)
        x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh) & frame_word_mask(o + 4 * i, d.len);
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
    const uint32_t crc = ~group_lin8(L, c);
    const uint32_t tr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((L.lane | 7u) * 4u), (int)c.tr);
    const uint32_t ok = (d.len >= 5u && __builtin_bswap32(tr) == crc) ? 1u : 0u;
    if (SEAL && L.col == 7u && !dead && d.len >= 4u) {
      g_u8w* wp = as_global<g_u8w>(p.wbytes + d.start + d.n);
      wp[0] = (uint8_t)(crc >> 24);
      wp[1] = (uint8_t)(crc >> 16);
      wp[2] = (uint8_t)(crc >> 8);
      wp[3] = (uint8_t)crc;
    }
    record(q & 7u, crc, (r.w & 63u) | (ok << 31) | ((dead ? 1u : 0u) << 30));
    if ((q & 7u) == 7u) store_run(q >> 3);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no visible load or store stays pending
  };

  // ---- ring: set S_k in slot k % DEPTH; records DEPTH sets ahead of their geometry ----
  constexpr int DEPTH = 2;
  Buf13 B[DEPTH];
  Rec O[DEPTH];
  uint32_t GE[DEPTH], VO[DEPTH], QO[DEPTH], QG[DEPTH];  // set of O[i] / of GE[i], B[i]
  uint64_t SB[DEPTH];
  Set8Meta M[DEPTH];
  // prologue: records of the wave's first 2 DEPTH - 1 sets, geometry + loads of the first
  // DEPTH - 1 (all in the wave's first run, which needs no claim: 2 DEPTH - 1 <= 8)
  Rec Rq[DEPTH];
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
    load_set(VO[i], GE[i], SB[i], B[i], Part0{});
    load_set(VO[i], GE[i], SB[i], B[i], Part1{});
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
  claim_next();  // the second run (the counter is set now)

  // One step: geometry + loads of set S + DEPTH - 1 (record loaded DEPTH steps ago), the record of
  // set S + 2 DEPTH - 1, then compute set S.
  auto step = [&](int cs, int fs) {
    QG[fs] = QO[fs];
    GE[fs] = geometry(QG[fs], O[fs], VO[fs], M[fs], SB[fs]);
    load_set(VO[fs], GE[fs], SB[fs], B[fs], Part0{});
    QO[fs] = next_q();
    O[fs] = load_rec(QO[fs]);
    __builtin_amdgcn_sched_barrier(0);
    auto second = [&]() { load_set(VO[fs], GE[fs], SB[fs], B[fs], Part1{}); };
    if (QG[cs] != kNoSet && !M[cs].slow) {
      compute(QG[cs], GE[cs], M[cs], B[cs], VO[cs], SB[cs], second);
    } else {
      second();
      if (QG[cs] != kNoSet) slow_set(QG[cs]);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // (a wave's sets are valid up to its first kNoSet, so a round stops at the first dead set)
  while (QG[0] != kNoSet) {
    step(0, 1);
    step(1, 0);
  }
}

// Product: 12 waves, 2 sets per wave in the ring (three waves per SIMD; config 3 1.69 ms kernel
// against 1.93 ms at 8 waves / depth 3 and 2.4-2.6 ms at 14-16 waves, which spill), runs sorted in
// the kernel with per-run geometry (1.480 against 1.506 ms with per-set geometry, config 3,
// in-process A/B, identical results; profiles/EXPERIMENTS.md).
template __global__ void frame_crc_varlen8_kernel<false, false>(const KernelParams);
template __global__ void frame_crc_varlen8_kernel<true, false>(const KernelParams);
template __global__ void frame_crc_varlen8_kernel<false, true>(const KernelParams);
template __global__ void frame_crc_varlen8_kernel<true, true>(const KernelParams);

const void* varlen8_kernel_symbol(bool seal, bool pairs) {
  if (pairs)
    return seal ? (const void*)frame_crc_varlen8_kernel<true, true> : (const void*)frame_crc_varlen8_kernel<false, true>;
  return seal ? (const void*)frame_crc_varlen8_kernel<true, false> : (const void*)frame_crc_varlen8_kernel<false, false>;
}
int varlen8_waves() { return kV8Waves; }

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

}  // namespace ufc_dev
