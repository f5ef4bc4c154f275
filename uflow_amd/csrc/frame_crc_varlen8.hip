// frame_crc_varlen8.hip -- variable-length frame-CRC kernel with 8 lanes per frame, for MI355X /
// gfx950: BASELINE.json config 3 (10M frames of U[64,1500] B) and the receive path.
//
// The batched CRC gate of Frame::read (src/frame/serial/mod.rs:675-690) and the frame seal
// (serial/mod.rs:463-470, build.rs:151-159) for frame i = bytes[offsets[i] .. offsets[i+1]) (or
// (start, end) pairs).  What this kernel does differently from the fixed-length one:
//   * A set is 8 frames, one per 8-lane group; lane col of a group loads the 16 bytes at 16 col of
//     each 128-byte line of its frame's window, so one wave-instruction reads 8 whole lines.
//   * Windows are aligned to 128-byte lines: from the line holding G's first byte (4 bytes before the
//     frame) to the line holding the frame's last byte, P lines.  Every load is one whole line, and
//     the lines a frame shares with its neighbours are only its first and its last (default cache
//     policy, so they stay in L2 for the neighbour, which the sort puts in another set); the lines in
//     between are read once (non-temporal).  Measured as a loads-only pattern: 1.18 ms and 1.025 x the
//     plain stream's requests on config 3, against 1.30 ms and 1.11 x for windows right-aligned to the
//     frame's end (profiles/EXPERIMENTS.md, round 5).
//   * Each lane's 4 words are 4 slot chains with the constant A^128 (32 slots per frame); the stream
//     ends at the word holding the frame's last byte (slot e, t = 0..3 bytes past the frame), so the
//     finish takes the slot constants rotated by e (group_lin8_rot) and undoes A^t with one nibble
//     lookup per lane (its own nibble of lin) summed over the group.  Words past a frame's end step nothing; the bytes past its data are masked out.
//   * Slots run right-aligned: position s = 0 .. 12 holds line s - 13 + P, so every frame's last line
//     is at position 12 and the lines before a frame's first are zeros (chains stay zero).  A set runs
//     positions 13 - Pmax .. 12 straight through (one copy of the sequence per entry point, chosen by a
//     switch on its longest frame); line 0 (slot 0, loaded apart for its cache policy) goes in at
//     position 13 - P.  Only positions 11 and 12 can need masked steps.
//   * One set buffer per wave, software-pipelined: each slot of the next set is issued as soon as the
//     current set has consumed that slot's registers (128 VGPRs: 16 waves per CU).  The straight copy
//     per entry point keeps the order of those loads the same on every path, so the compiler's load
//     waits stay counted (with one shared sequence it waited for every load at each entry point).
//   * Sets come from runs of 64 frames sorted by line count in the wave that takes them (four one-bit
//     radix split passes); the per-set facts come once per run from half-row reductions and ballots.
//   * Results of a run (8 sets x 8 frames) collect in one register pair per lane and leave with
//     hidden stores once per run.  Sets with a frame the fast path cannot take (shorter than 5 B, at
//     the batch edges, past its end) run byte-wise, in the same loop (the byte path keeps the 256-byte
//     block layout of frame_crc_dev.hpp: block8 below); frames longer than 13 lines go from there to a
//     second launch (frame_crc_long8_kernel, below).
//   * Built with uniform branches left unstructured (_build.py): the set-level branches otherwise get
//     register-copy blocks at every merge.
#include <type_traits>

#include "frame_crc_dev.hpp"

namespace ufc_dev {

// Structured buffer load (index, offset): llvm.amdgcn.struct.ptr.buffer.load, which clang exposes no
// builtin for.  Address = base + index * stride + voffset; an index at or past num_records (a
// "negative" one included) loads zeros and makes no memory request.
extern "C" __device__ u32x4 ufc_struct_buffer_load_b128(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset,
                                                        int soffset, int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");

namespace {

constexpr int kV8Pieces = 13;              // fast path: windows of up to 13 lines (frames of 4..1532 B)
constexpr uint32_t kV8Bias = 0x20000;      // window offsets: relative to the run's base - bias
constexpr uint32_t kV8Oob = 0x80000000u;   // out-of-range offset: zeros, no memory request
constexpr uint32_t kV8Limit = 0x7FF00000u;  // fast-path window offsets stay below this
constexpr int kV8AuxShared = 0;            // a frame's first and last line: default policy (shared)
constexpr int kV8AuxInterior = 2;          // the lines in between: non-temporal (read once)
constexpr uint32_t kNoSet = 0xFFFFFFFFu;   // a wave's set sequence past its last claimed run
// Slot loads k >= 1 (load_slot): record counts 3 + k against the index 16 - P; 29 lines off the base.
constexpr int kV8SlotRecords = 3;
constexpr uint64_t kV8SlotBase = 29u * 128u;
// The workgroup's run counter: nibble-image row 127, column 63 (rows 80..127 of columns 32..63 are
// never read).
constexpr uint32_t kV8CtrAddr = (127u * 64u + 63u) * 4u;
// Deferred frames: the workgroup's list counter and p.defer_list / p.defer_counts (read where they are
// used, from LDS: no scalar registers held across the loop).  Staged by thread 1023, which sets them.
constexpr uint32_t kV8DefAddr = (127u * 64u + 62u) * 4u;
constexpr uint32_t kV8ListPtrAddr = (127u * 64u + 58u) * 4u, kV8CountsPtrAddr = (127u * 64u + 56u) * 4u;
constexpr uint32_t kV8CrcPtrAddr = (127u * 64u + 54u) * 4u, kV8ValidPtrAddr = (127u * 64u + 52u) * 4u;
// A pointer kept in LDS at byte `addr` (the kernel's static LDS starts at address 0), read at the point of
// use: a volatile ds_read_b64 (lgkmcnt only), never hoisted into registers held across the loop.
template <typename T>
__device__ __forceinline__ T* lds_ptr(uint32_t addr) {
  typedef T* volatile __attribute__((address_space(3))) * LdsPtrSlot;
  return *(LdsPtrSlot)(uintptr_t)addr;
}

// Per-lane geometry of a frame on the fast path (one VGPR): r = (frame start - 4) mod 128 [0,7) (the
// window starts at the 128-byte line holding G's first byte, r bytes before it), len [7,18), index
// in its run [18,24); then the set's facts, the same in every lane of the set: Pmax = its frames' most
// lines, 0 for a byte-path set [24,28), Pmin = their fewest [28,32).  The trailer's first byte lies at
// window offset zo = len + r; lines P = ceil((zo + 4) / 128).  The window start's word (wrel) keeps
// bits 7.. of the start in [0,24) (its low 7 bits are the same for the whole run) and two more set
// facts: kV8PenultData (no frame's trailer starts in its line P - 2: that line holds CRC'd data only
// wherever it is a frame's) and kV8G1 (a frame's G reaches into line 1: r >= 125).
__device__ __forceinline__ uint32_t w_r(uint32_t g) { return g & 127u; }
__device__ __forceinline__ uint32_t w_zo(uint32_t g) { return (g >> 7) & 2047u; }
__device__ __forceinline__ uint32_t w_P(uint32_t g) { return (w_zo(g) + 131u) >> 7; }
__device__ __forceinline__ uint32_t w_orig(uint32_t g) { return (g >> 18) & 63u; }
constexpr uint32_t kV8PenultData = 1u << 25, kV8G1 = 1u << 26;

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
  uint32_t v = nib_mul4(L.lds, X0, X1, X2, X3, K2);
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
  uint32_t v = nib_mul4(L.lds, X0, X1, X2, X3, K2);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return v;
}

// A^-t of every group's lin, one nibble per lane: lane col of a group looks up A^-t of lin's nibble
// col in its own column 32 + (lane & 31) of the 32-slot image (rows 16 (t + 1) + nibble value; a
// half-wave's 32 lanes read 32 banks) and the group sums its 8 terms over DPP.
__device__ __forceinline__ uint32_t unshift8(const Lane8& L, uint32_t lin, uint32_t t) {
  if (__builtin_amdgcn_ballot_w64(t != 0) == 0) return lin;
  const uint32_t nib = __builtin_amdgcn_ubfe(lin, 4u * L.col, 4u);
  uint32_t r = *(const uint32_t*)(L.lds + ((nib << 8) | ((t << 12) | (L.K & 0xFFu))) + (4096u + 128u));
  r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return t ? r : lin;
}

// Front-fix table in LDS: for p = 0..20 bytes of a 16-byte piece before its frame, the mask M of
// the frame's bytes and the bytes Gs of G placed before them, so that front_fix(x, p, G) =
// (x & M) | Gs (p <= 0: nothing to fix, p >= 20: all zero).  32 bytes per entry, in the unused
// columns 32..39 of the 32-slot nibble image's rows 0..20 (rows 32..79 of columns 32..63 hold the
// A^-t tables).
constexpr int kFixEntries = 21;
__device__ __forceinline__ uint32_t fixtab_addr(uint32_t i) { return i * 256u + 128u; }

// End table, beside it (columns 40..47 of rows 0..20): entry j for lim = j - 4 bytes of the lane's 16 before
// the end of the CRC'd data (j = 0..20, lim clamped to -4..16): the data mask (bytes 0 .. lim - 1) and the
// keep mask (word w all ones when it lies wholly past the frame's end, lim <= 4 w - 4: it does not step).
__device__ __forceinline__ uint32_t endtab_addr(uint32_t j) { return j * 256u + 160u; }

__device__ __forceinline__ void fixtab_store(char* lds, uint32_t G) {  // threads 0..41, after the staging
  const uint32_t t = threadIdx.x;
  if (t < (uint32_t)kFixEntries) {
    const uint4 m = front_fix(make_uint4(~0u, ~0u, ~0u, ~0u), (int)t, G), g = front_fix(make_uint4(0u, 0u, 0u, 0u), (int)t, G);
    *(uint4*)(lds + fixtab_addr(t)) = make_uint4(m.x & ~g.x, m.y & ~g.y, m.z & ~g.z, m.w & ~g.w);
    *(uint4*)(lds + fixtab_addr(t) + 16) = g;
  } else if (t < 2u * (uint32_t)kFixEntries) {
    const uint32_t j = t - (uint32_t)kFixEntries;
    const int lim = (int)j - 4;
    *(uint4*)(lds + endtab_addr(j)) = make_uint4(data_mask(lim), data_mask(lim - 4), data_mask(lim - 8), data_mask(lim - 12));
    *(uint4*)(lds + endtab_addr(j) + 16) = make_uint4(lim <= -4 ? ~0u : 0u, lim <= 0 ? ~0u : 0u, lim <= 4 ? ~0u : 0u,
                                                      lim <= 8 ? ~0u : 0u);
  }
}

__device__ __forceinline__ uint4 fix_piece(const char* lds, uint4 x, int p) {
  asm("" : "+v"(p));  // (p opaque: its clamp stays one v_med3, not folded into the terms of p)
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
// The first lim bytes of a lane's 16 (lim clamped to 0..16), from the front-fix table: its entry n holds
// the mask of bytes n .. 15 (fixtab_store: the frame's bytes, G's excluded), so the data mask is its
// complement -- one ds_read_b128 and one bitop3 per word instead of a shift mask per word.
__device__ __forceinline__ uint4 end_masked(const char* lds, uint4 x, int lim) {
  const uint32_t i = (uint32_t)min(max(lim, 0), 16);
  const uint4 m = *(const uint4*)(lds + fixtab_addr(i));
  return make_uint4(x.x & ~m.x, x.y & ~m.y, x.z & ~m.z, x.w & ~m.w);
}

__device__ __forceinline__ void chain4_masked(const Lane8& L, Chains& c, uint4 x, int lim) {
  const uint4 d = end_masked(L.lds, x, lim);
  const uint32_t n0 = chain_step(L.lds, c.v0, L.K, d.x);
  const uint32_t n1 = chain_step(L.lds, c.v1, L.K, d.y);
  const uint32_t n2 = chain_step(L.lds, c.v2, L.K, d.z);
  const uint32_t n3 = chain_step(L.lds, c.v3, L.K, d.w);
  c.v0 = lim > -4 ? n0 : c.v0;
  c.v1 = lim > 0 ? n1 : c.v1;
  c.v2 = lim > 4 ? n2 : c.v2;
  c.v3 = lim > 8 ? n3 : c.v3;
}

// The same from the end table (lim4 = lim + 4): the data mask and the words that keep their chains in one
// table entry, one bitop3 per word instead of a compare and a select.
__device__ __forceinline__ void chain4_end(const Lane8& L, Chains& c, uint4 x, int lim4) {
  asm("" : "+v"(lim4));  // (one v_med3 for the clamp)
  const uint32_t j = (uint32_t)min(max(lim4, 0), 20);
  const uint4 dm = *(const uint4*)(L.lds + endtab_addr(j)), kp = *(const uint4*)(L.lds + endtab_addr(j) + 16);
  const uint32_t n0 = chain_step(L.lds, c.v0, L.K, x.x & dm.x);
  const uint32_t n1 = chain_step(L.lds, c.v1, L.K, x.y & dm.y);
  const uint32_t n2 = chain_step(L.lds, c.v2, L.K, x.z & dm.z);
  const uint32_t n3 = chain_step(L.lds, c.v3, L.K, x.w & dm.w);
  c.v0 = __builtin_amdgcn_bitop3_b32(n0, c.v0, kp.x, 0xD8);  // kp ? old : new
  c.v1 = __builtin_amdgcn_bitop3_b32(n1, c.v1, kp.y, 0xD8);
  c.v2 = __builtin_amdgcn_bitop3_b32(n2, c.v2, kp.z, 0xD8);
  c.v3 = __builtin_amdgcn_bitop3_b32(n3, c.v3, kp.w, 0xD8);
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
  uint32_t Pmax;    // most lines of the set's frames
  uint32_t Pmin;    // fewest
  bool penult_data;  // no frame's trailer starts in its line P - 2
  bool g1;          // a frame's G reaches into its line 1
  bool slow;        // byte path
};

// A set's loads, right-aligned: slot 0 = line 0, slot s >= 1 = line s - 13 + P (its last line P - 1 in
// slot 12; slots that would hold line 0 or a line before it are out of range, zeros).
struct Buf13 {
  uint4 x[kV8Pieces];
};

}  // namespace

// One workgroup of kV8Waves waves per CU (128 VGPRs: 4 waves per SIMD), one set buffer per wave,
// software-pipelined: the next set's slots are issued into the registers the current set has just
// consumed.  p.offsets = the CSR offsets (n + 1) or, with PAIRS, the (start, end) pairs (p.frame_len =
// the buffer length).  Each run of 64 frames is ordered by line count in the wave that takes it,
// after each frame's fast-path geometry has been computed in the frame's own lane; the per-set facts
// come once per run from half-row DPP reductions and ballots, and a set takes its two words per group
// with ds_bpermute and its set-level bits with one readfirstlane.  Frames the fast path cannot take
// sort together (key 14), so they spoil fewer sets.
constexpr int kV8Waves = 16;
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
    g.bad = !live || len < 5u || P > (uint32_t)kV8Pieces || a < 4u + r || rel64 >= (uint64_t)kV8Limit || rel64 < 512u;
    g.geo = r | (min(zo, 2047u) << 7) | (L.lane << 18);
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
    // Stable counting order by key: four one-bit split passes (LSD radix) over (key, lane) words,
    // each moved to its new position with one ds_permute; then sorted position i holds frame src.
    uint32_t v = (key << 6) | L.lane;
#pragma unroll
    for (uint32_t b = 6; b < 10; b++) {
      const bool one = ((v >> b) & 1u) != 0;
      const uint64_t m = __builtin_amdgcn_ballot_w64(one);
      const uint32_t ob = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t pos = one ? 64u - (uint32_t)__builtin_popcountll(m) + ob : L.lane - ob;
      v = (uint32_t)__builtin_amdgcn_ds_permute((int)(pos * 4u), (int)v);
    }
    const int src = (int)((v & 63u) * 4u);
    if (!raw) {
      // lane = sorted position: per-set facts over each 8-lane half-row, into geo bits 24..31
      const uint32_t geo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)fg.geo);
      const uint32_t bad = (v >> 6) >= 14u ? 1u : 0u;
      out.a_hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)fg.wrel);
      out.sb = sb;
      const uint32_t P = w_P(geo), zo = w_zo(geo);
      uint32_t px = P, pn = P;
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
      pn = min(pn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pn, 0xB1, 0xF, 0xF, false));
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
      pn = min(pn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pn, 0x4E, 0xF, 0xF, false));
      px = max(px, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)px, 0x141, 0xF, 0xF, false));  // row_half_mirror
      pn = min(pn, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pn, 0x141, 0xF, 0xF, false));
      const uint32_t hr = L.lane & ~7u;  // the set's half-row
      const bool slow = ((__builtin_amdgcn_ballot_w64(bad != 0u) >> hr) & 0xFFu) != 0;
      const bool pe = ((__builtin_amdgcn_ballot_w64(P >= 2u && zo < 128u * (P - 1u)) >> hr) & 0xFFu) == 0;
      const bool g1 = ((__builtin_amdgcn_ballot_w64(w_r(geo) >= 125u) >> hr) & 0xFFu) != 0;
      out.a_lo = (geo & 0xFFFFFFu) | ((slow ? 0u : min(px, 15u)) << 24) | (min(pn, 15u) << 28);
      out.a_hi = (out.a_hi >> 7) | (pe ? kV8PenultData : 0u) | (g1 ? kV8G1 : 0u);
      return;
    }
    out.a_lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)a);
    out.a_hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(a >> 32));
    out.len = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)min(len, (uint64_t)0xFFFFFFFFu));
    out.info = (v & 63u) | ((v >> 6) == 15u ? 0x80000000u : 0u);
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
  // The next run is claimed and its offsets requested one set before the switch (at position 7, before
  // that iteration issues its slots): the sort at the switch then waits for loads issued one set earlier,
  // older than that set's 13 slot loads, a count the compiler can keep.  (Requested a whole run ahead,
  // they sat behind ~100 younger loads, which the compiler could not count across the loop: it drained
  // every load in flight, vmcnt(0), once per run.)
  auto next_q = [&]() -> uint32_t {
    if (pos == 8u) {
      pos = 0;
      run = run_nxt;
      sort_run(run, raw_a, raw_b, SR);
    }
    if (pos == 7u) claim_next();
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
  auto geometry = [&](uint32_t q, const Rec& r, uint32_t& voff0, Set8Meta& m, uint64_t& sb, uint32_t& vidx,
                      uint32_t& voffn) -> uint32_t {
    sb = r.sb;
    const uint32_t gu = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.geo);
    const uint32_t hu = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.wrel);
    m.Pmax = (gu >> 24) & 15u;
    m.Pmin = gu >> 28;
    m.penult_data = (hu & kV8PenultData) != 0;
    m.g1 = (hu & kV8G1) != 0;
    m.slow = m.Pmax == 0u;
    const bool live = q != kNoSet && !m.slow;
    // (the window start's low 7 bits: bytes + sb + start is 128-byte aligned)
    const uint32_t low7 = (0u - (uint32_t)(uintptr_t)p.bytes - (uint32_t)sb) & 127u;
    voff0 = live ? (((r.wrel & 0xFFFFFFu) << 7) | low7) + 16u * L.col : kV8Oob;
    // the record index of every slot k >= 1: 16 - P (3 .. 15), or 16 for a set with no loads (past every
    // slot's record count, kV8SlotRecords); opaque, so that the select stays here once per set and is not
    // pushed into the slots.  The index contributes (16 - P) 128 to the address, so the slots' common offset
    // carries 2 P 128 (voffn; the constant part is in the descriptor's base, kV8SlotBase).
    const uint32_t P = live ? w_P(r.geo) : 0u;
    vidx = 16u - P;
    asm("" : "+v"(vidx));
    voffn = voff0 + (P << 8);
    return r.geo;
  };
  // The set's loads (struct Buf13): line 0 (slot 0) and the last line (slot 12), the lines the frame
  // shares with its neighbours (which the sort puts in other sets), with default policy so that they
  // stay in L2 for them; the lines in between, each read by this set alone, non-temporal; lanes wholly
  // before G and slots before a frame's line 1 are out of range (zeros, no request).  Slot k of a set
  // (k = 0: line 0; k >= 1: line k - 13 + P, out of range before line 1) is issued one at a time, as
  // the current set frees the slot's registers.
  // dep (DEP): the chain words of the position that has just consumed slot k: the load is issued
  // after them, so that it can take the slot's own registers (otherwise the scheduler issues it
  // while the position's last XORs still read the slot, the load goes into other registers, and each
  // straight copy of the positions ends with a different register assignment, moved back at the
  // loop's merge behind a vmcnt(1) wait)
  auto load_slot = [&](int k, uint32_t voff0, uint32_t geo, uint64_t sb, uint32_t& vidx, uint32_t voffn, Buf13& b,
                       const Chains* dep) {
    const uint32_t front = w_r(geo) + 4u;
    if (k == 0) {
      // (the slots' base, kV8SlotBase below the run's, with kV8SlotBase in the instruction's offset: one base
      // for every slot's descriptor)
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(p.bytes + sb - kV8SlotBase), 0, (int)0x7FFFFFF0, 0x00020000);
      const uint32_t vo = (16u * L.col + 16u <= front) ? kV8Oob : voff0;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vo + (uint32_t)kV8SlotBase), 0, kV8AuxShared);
      b.x[0] = make_uint4(v.x, v.y, v.z, v.w);
      return;
    }
    // slot k = line k - 13 + P: a structured load of record vidx = 16 - P (stride 128) from a descriptor
    // whose record count is 3 + k, so that the slot is in range exactly when P > 13 - k (line >= 1): lines
    // before line 1 load zeros and make no request, and the slots share one index register (no add per
    // slot).  Address = base + (16 - P) 128 + voff0 + 2 P 128 - 29 128 + 128 k = base + voff0 + 128 (k - 13 + P)
    // with the -29 128 in the base (kV8SlotBase) and 128 k in the instruction's offset.
    // (the record count set here, in the slot's own position: otherwise the 12 descriptors are hoisted out of
    // the loop as invariants, 48 scalar registers, and spill)
    int nrec;
    asm volatile("s_mov_b32 %0, %1" : "=s"(nrec) : "n"(kV8SlotRecords + k));
    const __amdgpu_buffer_rsrc_t rss =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.bytes + sb - kV8SlotBase), 128, nrec, 0x00020000);
    if (dep) asm("" : "+v"(vidx) : "v"(dep->v0), "v"(dep->v1), "v"(dep->v2), "v"(dep->v3));
    const u32x4 v = ufc_struct_buffer_load_b128(rss, (int)vidx, (int)(voffn + 128u * (uint32_t)k), 0,
                                                k == kV8Pieces - 1 ? kV8AuxShared : kV8AuxInterior);
    b.x[k] = make_uint4(v.x, v.y, v.z, v.w);
  };

  // ---- results of the current run: lane (g, col = t) <- set t's frame g; qv = orig | valid << 31
  uint32_t acc_crc = 0, acc_qv = 0;
  auto record = [&](uint32_t t, uint32_t crc, uint32_t qv) {  // (lanes col == t: a scalar mask, no compare)
    const bool mine = __builtin_amdgcn_inverse_ballot_w64(0x0101010101010101ull << t);
    acc_crc = mine ? crc : acc_crc;
    acc_qv = mine ? qv : acc_qv;
  };
  auto store_run = [&](uint32_t run) {  // hidden stores (see frame_crc_dev.hpp)
    const uint64_t f = (uint64_t)run * kRunFrames + (acc_qv & 63u);
    if (!(acc_qv & 0x40000000u) && f < nfr) {
      // (the output pointers from LDS, read here: no scalar registers held across the loop for them)
      uint32_t* const co = lds_ptr<uint32_t>(kV8CrcPtrAddr);
      if (co) st_u32_hidden(co + f, acc_crc);
      if (!SEAL) {
        uint8_t* const vo = lds_ptr<uint8_t>(kV8ValidPtrAddr);
        if (vo) st_u8_hidden(vo + f, acc_qv >> 31);
      }
    }
  };
  auto unshift = [&](uint32_t lin, uint32_t t) -> uint32_t { return unshift8(L, lin, t); };

  // Fast set.  The stream of a frame is its window with the bytes before G zeroed, G, the data, the
  // trailer as zeros, up to the end of the word holding the frame's last byte (e: that word's slot,
  // t = 0..3 bytes past the frame in it): lin = A^t (register after the data), undone at the finish.
  // The slots run right-aligned: position s = 0 .. 12 holds line s - 13 + P of each frame, so every
  // frame's last line is at position 12 and its line 0 at 13 - P (line 0 comes from slot 0: it is put
  // in at that position, front-fixed).  Positions before a frame's line 0 hold zeros, which leave its
  // chains at zero: the set runs positions 13 - Pmax .. 12 straight through, every lane stepping at
  // every position, entered once by a switch on Pmax (one merge of the chain registers per set).  Only
  // positions 11 and 12 (lines P - 2 and P - 1) can hold bytes past the CRC'd data (masked steps).
  auto compute = [&](uint32_t q, uint32_t geo, const Set8Meta& m, const Buf13& b, uint32_t voff0, uint64_t sb,
                     auto issue) {
    static_assert(kV8Pieces == 13, "the position sequence below");
    const uint32_t zo = w_zo(geo), P = w_P(geo), front = w_r(geo) + 4u;
    const int lim0 = (int)zo - (int)(16u * L.col);
    const int lim12 = lim0 - 128 * (int)(P - 1u), lim11 = lim12 + 128;
    const int g1 = 128 + (int)(16u * L.col) - (int)front;  // G's last bytes in line 1 (r >= 125)
    const uint4 fx = fix_piece(L.lds, b.x[0], (int)front - (int)(16u * L.col));  // line 0
    issue(0);
    const uint32_t Iend = 13u - m.Pmin;  // positions holding some frame's line 0: 13 - Pmax .. Iend
    auto xin = [&](int s) -> uint4 {  // position s's piece
      uint4 x = s == 0 ? make_uint4(0u, 0u, 0u, 0u) : b.x[s];
      if ((uint32_t)s <= Iend) {
        const bool l0 = (uint32_t)s + P == 13u;
        x = make_uint4(l0 ? fx.x : x.x, l0 ? fx.y : x.y, l0 ? fx.z : x.z, l0 ? fx.w : x.w);
      }
      if (m.g1 && (uint32_t)s + m.Pmax >= 14u && (uint32_t)s <= Iend + 1u)
        x.x = fix_word(x.x, (uint32_t)s + P == 14u ? g1 : 0, L.G);
      return x;
    };
    Chains c{0u, 0u, 0u, 0u, 0u};
    // The gate's trailer, from the registers of the last two lines (no load of its own): it starts
    // at u = zo - 128 (P - 1) in line P - 1 (-3 .. 124; u < 0 only when it starts in the last word of
    // line P - 2), in line words a0 = floor(u / 4) and a1 = a0 + 1, which lanes a >> 2 of the group
    // hold as component a & 3: each lane picks the group's component and ds_bpermute gathers them.
    const int u = (int)zo - 128 * (int)(P - 1u);
    const uint32_t a1 = min((uint32_t)(u + 4) >> 2, 31u), a0 = max((uint32_t)(u + 4) >> 2, 1u) - 1u;
    uint32_t tw_p = 0u, tw0 = 0u, tw1 = 0u;  // word 31 of line P - 2 (in the group's lane 0), the trailer's words
    auto pick = [](const uint4& x, uint32_t k) {
      const uint32_t lo = (k & 1u) ? x.y : x.x, hi = (k & 1u) ? x.w : x.z;
      return (k & 2u) ? hi : lo;
    };
    auto trailer_words = [&](int s, const uint4& x) {
      if constexpr (!SEAL) {
        if (s == 11) {  // line P - 2's last word, into the group's lane 0 (row_half_mirror: no lane index)
          tw_p = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.w, 0x141, 0xF, 0xF, false);
        } else if (s == 12) {  // the trailer's first word: from line P - 2 (lane 0) when it starts there
          const uint32_t gb = L.lane & ~7u;
          tw0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((gb + (a0 >> 2)) * 4u), (int)(u < 0 ? tw_p : pick(x, a0 & 3u)));
          tw1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((gb + (a1 >> 2)) * 4u), (int)pick(x, a1 & 3u));
        }
      }
    };
    auto masked_init = [&](uint4 x, int lim) {  // from zero chains: words past the end stay zero
      const uint4 d = end_masked(L.lds, x, lim);
      c = Chains{d.x, d.y, d.z, d.w, 0u};
    };
    auto entry = [&](int s) {
      for (int k = 1; k < s; k++) issue(k);  // (slots this set does not use)
      const uint4 x = xin(s);
      trailer_words(s, x);
      if (s == 12)
        masked_init(x, lim12);
      else if (s == 11 && !m.penult_data)
        masked_init(x, lim11);
      else
        c = Chains{x.x, x.y, x.z, x.w, 0u};
      if (s > 0) issue(s, &c);
    };
    auto stepk = [&](int s) {
      const uint4 x = xin(s);
      trailer_words(s, x);
      if (s == 12)
        chain4_end(L, c, x, lim12 + 4);
      else if (s == 11 && !m.penult_data)  // (every word of line P - 2 lies before the frame's end: data mask only)
        chain4(L, c, end_masked(L.lds, x, lim11));
      else
        chain4(L, c, x);
      issue(s, &c);
    };
    // one straight copy of the positions per entry point (no merges inside: the loads the positions
    // issue keep one order on every path, so their waits stay counted)
    auto from = [&](auto e) {
      constexpr int E = decltype(e)::value;
      entry(E);
#pragma unroll
      for (int k = E + 1; k <= 12; k++) stepk(k);
    };
    // Wave priority 2 over the line positions, 0 for the finish and the loop top: a SIMD's waves that
    // consume slots (and issue the next set's loads as they go) issue ahead of those in their finish
    // (1.3908 against 1.4002 ms; 3 or 1 instead of 2, or 2 from the loop top, within 0.1 % of it).
    __builtin_amdgcn_s_setprio(2);
    switch (m.Pmax) {  // enter at position 13 - Pmax
      case 13: from(std::integral_constant<int, 0>{}); break;
      case 12: from(std::integral_constant<int, 1>{}); break;
      case 11: from(std::integral_constant<int, 2>{}); break;
      case 10: from(std::integral_constant<int, 3>{}); break;
      case 9: from(std::integral_constant<int, 4>{}); break;
      case 8: from(std::integral_constant<int, 5>{}); break;
      case 7: from(std::integral_constant<int, 6>{}); break;
      case 6: from(std::integral_constant<int, 7>{}); break;
      case 5: from(std::integral_constant<int, 8>{}); break;
      case 4: from(std::integral_constant<int, 9>{}); break;
      case 3: from(std::integral_constant<int, 10>{}); break;
      case 2: from(std::integral_constant<int, 11>{}); break;
      default: from(std::integral_constant<int, 12>{}); break;
    }
    __builtin_amdgcn_s_setprio(0);
    const uint32_t e = ((zo + 3u) >> 2) & 31u, t = (0u - zo) & 3u;
    const uint32_t crc = ~unshift(group_lin8_rot(L, c, e), t);
    const uint32_t tr = __builtin_amdgcn_alignbyte(tw1, tw0, (uint32_t)u & 3u);
    const uint32_t ok = (!SEAL && __builtin_bswap32(tr) == crc) ? 1u : 0u;  // (fast-path frames have >= 5 B)
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
    // Longer than the fast path, window inside the buffer: to the workgroup's list for the second launch
    // (frame_crc_long8_kernel), which stores its results; here it counts as dead.
    const uint32_t rr = ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a - 4u) & 127u;
    const bool defer = (r.w >> 31) == 0 && r.z >= 4u && r.z < 0x40000000u && r.z + rr > 128u * 13u - 4u &&
                       a >= 4u + rr;
    // (a deferred frame's 8 lanes all store its index into its slot: no per-column lane mask)
    const uint64_t dm = __builtin_amdgcn_ballot_w64(defer);
    if (dm != 0) {
      uint32_t base = 0;
      if (L.lane == 0)
        base = __hip_atomic_fetch_add((uint32_t*)(lds + kV8DefAddr), (uint32_t)__builtin_popcountll(dm) >> 3,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u)) >> 3;
      uint32_t* const dl = lds_ptr<uint32_t>(kV8ListPtrAddr);  // (this workgroup's part of the list)
      if (defer) *as_global<g_u32w>(dl + base + rk) = (q >> 3) * kRunFrames + (r.w & 63u);
      if (L.lane == 0) {
        uint32_t* const dc = lds_ptr<uint32_t>(kV8CountsPtrAddr);  // (this workgroup's count)
        __hip_atomic_fetch_add(as_global<g_u32w>(dc), (uint32_t)__builtin_popcountll(dm) >> 3, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const bool dead = (r.w >> 31) != 0 || defer;
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

  // ---- software pipeline over one buffer: set S computes while set S + 1's slots are issued into
  // the registers S has just consumed; records one set ahead of their geometry ----
  Buf13 B;
  Rec O;  // record of set QO
  uint32_t QO, QG, GE, VO;  // QG: the set being computed (its geometry GE, VO, SB, M)
  uint64_t SB;
  Set8Meta M;
  {  // prologue: the first set's geometry and loads, the second set's record
    QG = next_q();
    const Rec r0 = load_rec(QG);
    uint32_t X0, VX0;
    GE = geometry(QG, r0, VO, M, SB, X0, VX0);
#pragma unroll
    for (int k = 0; k < kV8Pieces; k++) load_slot(k, VO, GE, SB, X0, VX0, B, nullptr);
    QO = next_q();
    O = load_rec(QO);
  }
  stage_store<WAVES * 64>(sr, lds);
  fixtab_store(lds, p.G);  // (then an LDS-only barrier, as in stage_store: the prefetches stay in flight)
  // Runs WR0 .. WR0 + WAVES - 1 are taken statically.  (Set by the thread whose stage_store wrote
  // the word, after it: program order, then the barrier below.)
  if (threadIdx.x == 1023u % (WAVES * 64u)) {
    *ctr = WAVES;
    *(uint32_t*)(lds + kV8DefAddr) = 0u;
    *(uint32_t**)(lds + kV8ListPtrAddr) = p.defer_list + (uint64_t)WR0 * kRunFrames;
    *(uint32_t**)(lds + kV8CountsPtrAddr) = p.defer_counts + blockIdx.x;
    *(uint32_t**)(lds + kV8CrcPtrAddr) = p.crc_out;
    *(uint8_t**)(lds + kV8ValidPtrAddr) = p.valid_out;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  // (the second run is claimed at the first run's position 7, in next_q: the counter is set now)

  // (a wave's sets are valid up to its first kNoSet)
  while (QG != kNoSet) {
    // the next set: geometry from its record; the record after it
    uint32_t VN, XN, VXN;
    uint64_t SBN;
    Set8Meta MN;
    const uint32_t QN = QO;
    const uint32_t GN = geometry(QN, O, VN, MN, SBN, XN, VXN);
    QO = next_q();
    O = load_rec(QO);
    __builtin_amdgcn_sched_barrier(0);
    auto issue = [&](int k, const Chains* dep = nullptr) { load_slot(k, VN, GN, SBN, XN, VXN, B, dep); };
    if (!M.slow) {
      compute(QG, GE, M, B, VO, SB, issue);
    } else {
#pragma unroll
      for (int k = 0; k < kV8Pieces; k++) issue(k);
      slow_set(QG);
    }
    __builtin_amdgcn_sched_barrier(0);
    QG = QN;
    GE = GN;
    VO = VN;
    SB = SBN;
    M = MN;
  }

}

// ---- Frames longer than the fast path (over 13 lines, 1532 B): the second launch ----
// frame_crc_varlen8_kernel's byte path leaves them to this kernel (p.defer_list, p.defer_counts) instead
// of running them byte-wise, since its loop's 128 VGPRs have no room for a line loop (a line-loop path
// inside it cost config 3 0.3-0.45 %, profiles/EXPERIMENTS.md).  Workgroup b takes the frames workgroup b
// of the first launch deferred (a workgroup with none reads its count and leaves before staging any
// table) and zeroes its count for the next first launch.
// Its waves claim chunks of 64 frames, order each chunk by line count (radix split passes, as the first
// launch orders its runs), and run the chunk as sets of 8 frames, 8 lanes per frame: the same slot-chain
// CRC over whole 128-byte lines of the same window (the line holding G's first byte to the line holding
// the frame's last byte), right-aligned so that every frame's last line comes at the set's last step:
// steps before a frame's line 0 load its line 0 again and are zeroed (its chains stay zero), line 0 is
// front-fixed, the last two steps are masked at the end of the CRC'd data, and the trailer comes from the
// last two lines' registers.  Four lines per frame are in flight (loads issued four steps ahead).
constexpr int kL8Waves = 16;
template <bool SEAL, bool PAIRS>
__global__ __launch_bounds__(kL8Waves * 64) void frame_crc_long8_kernel(const KernelParams p, uint32_t main_blocks) {
  constexpr int WAVES = kL8Waves;
  const uint32_t cnt = __builtin_amdgcn_readfirstlane((int)p.defer_counts[blockIdx.x]);
  if (cnt == 0) return;
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const StageSet<WAVES * 64> sr = stage_load<WAVES * 64>(p);
  Lane8 L;
  init_lane8(L, lds, p.G);
  const uint64_t nfr = p.nframes;
  const uint32_t nruns = (uint32_t)((nfr + kRunFrames - 1) / kRunFrames);
  const uint64_t region = (uint64_t)((uint64_t)nruns * blockIdx.x / main_blocks) * kRunFrames;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* const ctr = (uint32_t*)(lds + kV8CtrAddr);
  stage_store<WAVES * 64>(sr, lds);
  fixtab_store(lds, p.G);
  if (threadIdx.x == 1023u % (WAVES * 64u)) *ctr = WAVES;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  // Every wave has read the count (before the barrier): zero it for the next first launch on this
  // stream, whose byte path adds to it (a vector store).
  if (threadIdx.x == 0) st_u32_hidden(p.defer_counts + blockIdx.x, 0u);
  const uint32_t nchunks = (cnt + 63u) / 64u;
  const uint64_t* offs = p.offsets;
  for (uint32_t c = wid; c < nchunks;) {
    // ---- the chunk's frames, one per lane, ordered by line count ----
    const uint32_t here = min(cnt - 64u * c, 64u);
    const bool live = L.lane < here;
    const uint32_t f = live ? p.defer_list[region + 64u * c + L.lane] : 0u;
    const uint64_t a = *as_global<g_u64>(offs + (PAIRS ? 2 * (uint64_t)f : f));
    const uint64_t b = *as_global<g_u64>(offs + (PAIRS ? 2 * (uint64_t)f + 1 : f + 1));
    const uint32_t len = (uint32_t)(b - a);  // (>= 1533 and < 2^30: the first launch's rule)
    const uint32_t r0 = ((uint32_t)(uintptr_t)p.bytes + (uint32_t)a - 4u) & 127u;
    const uint32_t P0 = (len + r0 + 131u) >> 7;
    uint32_t v = ((live ? min(P0, 127u) : 255u) << 6) | L.lane;
#pragma unroll
    for (uint32_t bit = 6; bit < 14; bit++) {  // stable LSD radix split by key (8 bits)
      const bool one = ((v >> bit) & 1u) != 0;
      const uint64_t m = __builtin_amdgcn_ballot_w64(one);
      const uint32_t ob = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t pos = one ? 64u - (uint32_t)__builtin_popcountll(m) + ob : L.lane - ob;
      v = (uint32_t)__builtin_amdgcn_ds_permute((int)(pos * 4u), (int)v);
    }
    const int src = (int)((v & 63u) * 4u);  // sorted position L.lane holds frame (lane) src / 4
    const uint32_t s_f = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)f);
    const uint32_t s_alo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)a);
    const uint32_t s_ahi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(a >> 32));
    const uint32_t s_len = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)len);
    // next chunk (claimed now, used after this one)
    uint32_t nxt = 0;
    if (L.lane == 0) nxt = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)nxt);

    const uint32_t nsets = (here + 7u) / 8u;
    for (uint32_t q = 0; q < nsets; q++) {
      // group g: sorted position 8 q + g (positions past the chunk repeat its last frame, unstored)
      const uint32_t sp = min(8u * q + L.grp, here - 1u);
      const bool dead = 8u * q + L.grp >= here;
      const int sl = (int)(sp * 4u);
      const uint32_t fr = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)s_f);
      const uint64_t fa = (uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)s_alo) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)s_ahi) << 32);
      const uint32_t fl = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)s_len);
      const uint32_t r = ((uint32_t)(uintptr_t)p.bytes + (uint32_t)fa - 4u) & 127u;
      const uint32_t front = r + 4u, zo = fl + r, P = (zo + 131u) >> 7;
      uint32_t Pmax = 0, Pmin = 0xFFFFFFFFu;
#pragma unroll
      for (int g = 0; g < 8; g++) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)P, 8 * g);
        Pmax = max(Pmax, x);
        Pmin = min(Pmin, x);
      }
      const uint32_t P4 = (Pmax + 3u) & ~3u;  // steps: a multiple of 4, every frame's last line at step P4 - 1
      const uint32_t sh = P4 - P;             // frame line j = step - sh
      const uint8_t* const wbase = p.bytes + (fa - 4u - r) + 16u * L.col;
      auto load_line = [&](uint32_t k) -> uint4 {  // step k's line, clamped into the frame's window
        const int j = (int)k - (int)sh;
        const uint32_t jc = (uint32_t)min(max(j, 0), (int)P - 1);
        const u32x4 x = __builtin_nontemporal_load(as_global<g_u32x4>(wbase + 128u * jc));
        return make_uint4(x.x, x.y, x.z, x.w);
      };
      const int lim0 = (int)zo - (int)(16u * L.col);
      const int uu = (int)zo - 128 * (int)(P - 1u);  // the trailer's first byte in line P - 1 (-3 .. 124)
      const uint32_t a1 = min((uint32_t)(uu + 4) >> 2, 31u), a0 = max((uint32_t)(uu + 4) >> 2, 1u) - 1u;
      auto pick = [](const uint4& x, uint32_t k) {
        const uint32_t lo = (k & 1u) ? x.y : x.x, hi = (k & 1u) ? x.w : x.z;
        return (k & 2u) ? hi : lo;
      };
      uint32_t tw_p = 0u, tw0 = 0u, tw1 = 0u;
      Chains ch{0u, 0u, 0u, 0u, 0u};
      uint4 X[4];
#pragma unroll
      for (int u = 0; u < 4; u++) X[u] = load_line((uint32_t)u);
      const uint32_t pre_end = P4 - Pmin + 2u;  // steps up to a frame's line 1 (zeros, front fix, G's tail)
      for (uint32_t k0 = 0; k0 < P4; k0 += 4u) {
        const bool last = k0 + 4u == P4;  // (uniform)
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t k = k0 + (uint32_t)u;
          uint4 x = X[u];
          if (!last) X[u] = load_line(k + 4u);
          if (k < pre_end) {
            const int j = (int)k - (int)sh;
            const bool z = j < 0;  // (component selects: a select of whole vectors goes through the stack)
            x = make_uint4(z ? 0u : x.x, z ? 0u : x.y, z ? 0u : x.z, z ? 0u : x.w);
            if (__builtin_amdgcn_ballot_w64(j == 0) != 0) {
              const uint4 fx = fix_piece(L.lds, x, (int)front - (int)(16u * L.col));
              const bool l0 = j == 0;
              x = make_uint4(l0 ? fx.x : x.x, l0 ? fx.y : x.y, l0 ? fx.z : x.z, l0 ? fx.w : x.w);
            }
            if (__builtin_amdgcn_ballot_w64(j == 1) != 0)
              x.x = j == 1 ? fix_word(x.x, 128 + (int)(16u * L.col) - (int)front, L.G) : x.x;
          }
          if (last && u == 2) {  // line P - 2
            if constexpr (!SEAL) tw_p = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((L.lane & ~7u) + 7u) * 4u), (int)x.w);
            chain4_masked(L, ch, x, lim0 - 128 * (int)(P - 2u));
          } else if (last && u == 3) {  // line P - 1
            if constexpr (!SEAL) {
              const uint32_t gb = L.lane & ~7u;
              tw0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((gb + (a0 >> 2)) * 4u), (int)pick(x, a0 & 3u));
              tw1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((gb + (a1 >> 2)) * 4u), (int)pick(x, a1 & 3u));
            }
            chain4_masked(L, ch, x, lim0 - 128 * (int)(P - 1u));
          } else {
            chain4(L, ch, x);
          }
        }
      }
      const uint32_t e = ((zo + 3u) >> 2) & 31u, t = (0u - zo) & 3u;
      const uint32_t crc = ~unshift8(L, group_lin8_rot(L, ch, e), t);
      if (L.col == 0u && !dead) {
        if (p.crc_out) st_u32_hidden(p.crc_out + fr, crc);
        if constexpr (SEAL) {
          st_u32_hidden((uint32_t*)(p.wbytes + fa + fl - 4u), __builtin_bswap32(crc));
        } else {
          const uint32_t tr = __builtin_amdgcn_alignbyte(tw1, uu < 0 ? tw_p : tw0, (uint32_t)uu & 3u);
          if (p.valid_out) st_u8_hidden(p.valid_out + fr, __builtin_bswap32(tr) == crc ? 1u : 0u);
        }
      }
    }
    c = nxt;
  }
}

// Product (round 5): 16 waves, one pipelined buffer each, one straight copy of the positions per entry
// point (1.4337 against 1.4723 ms for 12 waves with two buffers each, config 3, in-process A/B,
// identical results; profiles/EXPERIMENTS.md).
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

template __global__ void frame_crc_long8_kernel<false, false>(const KernelParams, uint32_t);
template __global__ void frame_crc_long8_kernel<true, false>(const KernelParams, uint32_t);
template __global__ void frame_crc_long8_kernel<false, true>(const KernelParams, uint32_t);
template __global__ void frame_crc_long8_kernel<true, true>(const KernelParams, uint32_t);

const void* long8_kernel_symbol(bool seal, bool pairs) {
  if (pairs)
    return seal ? (const void*)frame_crc_long8_kernel<true, true> : (const void*)frame_crc_long8_kernel<false, true>;
  return seal ? (const void*)frame_crc_long8_kernel<true, false> : (const void*)frame_crc_long8_kernel<false, false>;
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

}  // namespace ufc_dev
