// frame_crc_dev.hpp -- device helpers shared by the frame-CRC kernels (frame_crc.hip,
// frame_crc_varlen.hip).
//
//
// Replaces, in batch, the per-frame loop of src/frame/serial/crc.rs:94-104 used by the CRC gate
// of Frame::read (src/frame/serial/mod.rs:675-690) and by the frame seal
// (src/frame/serial/mod.rs:463-470, src/frame/serial/build.rs:151-159).
//
// Algorithm (all linear over GF(2), register domain; see crc_math.hpp):
//   * A frame of len bytes has n = len-4 CRC'd bytes followed by the 4-byte trailer (n = len and
//     4 virtual zero bytes when len < 4).  With E = n + 4 the frame is right-aligned into a virtual
//     stream of J*256 bytes:
//         [ zeros | G (4 bytes) | frame[0..n) | T (4 bytes) ],  J = ceil((E+4)/256),  pad = 256J - E,
//     so frame offset o sits at virtual byte o + pad (pad in 4..259).  G = A^-4(~0) folds the
//     reference's init (~0) into a plain linear CRC.  T is the trailer: it is the LAST virtual word,
//     arrives with the coalesced block loads, is kept for the validity check and is replaced by zero
//     in the CRC; the zero word's A^4 is undone by the slot constants below.
//   * Virtual word w (4 bytes) belongs to slot s = w mod 64.  Slot s runs a Horner chain over the
//     J blocks with the constant A^256:  V_s <- A^256(V_s) ^ word.  A^256 is applied with four
//     byte tables held in LDS, replicated 32x so that lane l always reads bank l mod 32
//     (conflict-free ds_read_b32 whatever the data).
//   * lin = XOR_s A^(4(63-s))(V_s)  (= A^-4 of the stream's linear CRC, i.e. the register after
//     frame[0..n) with init ~0); crc = ~lin.  Each slot's value is multiplied by its constant via
//     per-slot nibble tables in LDS (8 lookups), then XOR-reduced in the frame's 16 lanes by DPP.
// Wave layout: 4 frames per set, 16 lanes per frame; lane col of a frame loads the 16 bytes at
// 16*col of each 256-byte block with one non-temporal global_load_dwordx4, so a wave-instruction
// reads four contiguous 256-byte runs.  Lane col holds slots 4*col+b (b=0..3) in four independent
// chains.  A wave walks contiguous runs of kSetsPerRun sets (64 frames): results accumulate in
// registers (lane i <-> frame i of the run) and leave as one coalesced store per run.  Frames
// whose block count differs inside a set (varlen) run the set's maximum and freeze their chains
// after their own last block.
//
// LDS (one 1024-thread workgroup per CU, 160 KiB), laid out so that every table address is ONE
// v_perm_b32 (byte select) of the value being looked up:
//   [0, 32K)     nibble tables: slot s, nibble k, value e at byte k*4096 + e*256 + c(s)*4, with
//                c(s) = (s >> 1) + 32*(s & 1); k*4096 goes in the ds_read offset.  In nibble step i,
//                frames in odd 16-lane groups use chain (i+2)&3, so the 32 lanes of an LDS
//                lane-group hit 32 distinct banks.
//   [32K, 160K)  chain tables (two per 256-byte row): table k = 2p + t, entry e, copy c at byte
//                32768 + p*65536 + e*256 + t*128 + c*4, c = lane & 31 (bank = c: conflict-free).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "frame_crc_kernels.hpp"

namespace ufc_dev {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Global-address-space views: loads through them compile to global_load_* (vmcnt only).  Plain
// or non-temporal loads through generic pointers can become flat_load_*, which also count in
// lgkmcnt and make every LDS wait drain the HBM prefetch.
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_u32;
typedef const __attribute__((address_space(1))) uint64_t g_u64;
typedef __attribute__((address_space(1))) uint8_t g_u8w;
typedef __attribute__((address_space(1))) uint32_t g_u32w;

template <typename G, typename T>
__device__ __forceinline__ G* as_global(T* p) {
  return (G*)(p);
}

constexpr int kSetsPerRun = 16;  // 16 sets x 4 frames = 64 frames = one result per lane

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// v_perm_b32 byte select: result byte i = byte sel.i of the 8 bytes {hi: a, lo: b};
// selector 0..3 picks b's bytes, 4..7 a's bytes, 0x0C gives 0x00.
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
  return __builtin_amdgcn_perm(a, b, sel);
}

constexpr uint32_t kChainBase = 32768u;
// Address of table k's entry for byte k of v: bytes [c4 + 128*(k&1), v.byte_k, k>>1, 0] with
// K = per-lane bytes [c4, c4 + 128, 0, 1]; the 32 KiB base goes in the ds_read offset.
constexpr uint32_t kSelChain0 = 0x0C020400u, kSelChain1 = 0x0C020501u, kSelChain2 = 0x0C030600u,
                   kSelChain3 = 0x0C030701u;

// A^256(v) ^ x with the replicated byte tables: 4 v_perm + 4 ds_read_b32 + 2 v_bitop3.
__device__ __forceinline__ uint32_t chain_step(const char* lds, uint32_t v, uint32_t K, uint32_t x) {
  const char* t = lds + kChainBase;
  const uint32_t r0 = *(const uint32_t*)(t + perm(v, K, kSelChain0));
  const uint32_t r1 = *(const uint32_t*)(t + perm(v, K, kSelChain1));
  const uint32_t r2 = *(const uint32_t*)(t + perm(v, K, kSelChain2));
  const uint32_t r3 = *(const uint32_t*)(t + perm(v, K, kSelChain3));
  return xor3(xor3(r0, r1, r2), r3, x);
}

// Multiply v by the constant of the slot whose column byte-offset is byte I of K2:
// nibble k of v indexes row (k*16 + e); address bytes [K2.byte_I, nibble, 0, 0] + k*4096.
template <int I>
__device__ __forceinline__ uint32_t nib_mul(const char* lds, uint32_t v, uint32_t K2) {
  const uint32_t lo = v & 0x0F0F0F0Fu;          // nibbles 0,2,4,6 as bytes
  const uint32_t hi = (v >> 4) & 0x0F0F0F0Fu;   // nibbles 1,3,5,7 as bytes
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t sel = 0x0C0C0000u | ((uint32_t)(4 + (k >> 1)) << 8) | (uint32_t)I;
    r[k] = *(const uint32_t*)(lds + perm((k & 1) ? hi : lo, K2, sel) + k * 4096);
  }
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), xor3(r[6], r[7], 0u));
}

// The 8 lookups of nib_mul<I> without their sum.
template <int I>
__device__ __forceinline__ void nib_terms(const char* lds, uint32_t v, uint32_t K2, uint32_t* r) {
  const uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t sel = 0x0C0C0000u | ((uint32_t)(4 + (k >> 1)) << 8) | (uint32_t)I;
    r[k] = *(const uint32_t*)(lds + perm((k & 1) ? hi : lo, K2, sel) + k * 4096);
  }
}

// nib_mul<0>(X0) ^ nib_mul<1>(X1) ^ nib_mul<2>(X2) ^ nib_mul<3>(X3) as one tree over the 32 lookups:
// 16 three-input XORs instead of 18.
__device__ __forceinline__ uint32_t nib_mul4(const char* lds, uint32_t X0, uint32_t X1, uint32_t X2, uint32_t X3,
                                             uint32_t K2) {
  uint32_t r[32];
  nib_terms<0>(lds, X0, K2, r);
  nib_terms<1>(lds, X1, K2, r + 8);
  nib_terms<2>(lds, X2, K2, r + 16);
  nib_terms<3>(lds, X3, K2, r + 24);
  uint32_t t[12];
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = xor3(r[3 * k], r[3 * k + 1], r[3 * k + 2]);
  t[10] = r[30];
  t[11] = r[31];
  const uint32_t u0 = xor3(t[0], t[1], t[2]), u1 = xor3(t[3], t[4], t[5]), u2 = xor3(t[6], t[7], t[8]),
                 u3 = xor3(t[9], t[10], t[11]);
  return xor3(u0, u1, u2) ^ u3;
}

// XOR over the 16 lanes of a DPP row; every lane of the row receives the total.
__device__ __forceinline__ uint32_t row_xor16(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// ---- Mask and shift helpers (host and device: tests/c/ubsan_helpers.hip drives every one of them over
// its whole argument range as host code under UBSan).  Every variable shift amount is kept in range
// in every arm, selected or not.

// Word of the virtual stream whose first byte sits at frame offset o (o < 0: before the frame).
// Bytes at frame offsets [-4, 0) are G's bytes, below -4 zeros, from 0 on the loaded data v.
__host__ __device__ __forceinline__ uint32_t fix_word(uint32_t v, int o, uint32_t G) {
  const uint64_t pv = (uint64_t)G << 32;
  const uint32_t sh = (uint32_t)(8 * (o + 8)) & 63u;  // in [8, 56] when o in (-8, 0)
  const uint32_t pre = (uint32_t)(pv >> sh);
  const uint32_t dm = (o > -4 && o < 0) ? (0xFFFFFFFFu << ((uint32_t)(-8 * o) & 31u)) : 0u;
  const uint32_t mixed = (v & dm) | (pre & ~dm);
  return (o >= 0) ? v : ((o <= -8) ? 0u : mixed);
}

// Block 0 of a frame, lane with p = pad - 16 col bytes before the frame: bytes before the frame
// become zeros, except the 4 right before it, which become G (the reference's initial ~0 folded
// into a linear CRC).  p <= 0: the data unchanged; p >= 20: all zero.
__host__ __device__ __forceinline__ uint4 front_fix(uint4 x, int p, uint32_t G) {
  const uint32_t pc = (uint32_t)(p < 0 ? 0 : (p > 20 ? 20 : p));
  const uint32_t s = 8u * pc;  // data bytes start at bit s of the 128-bit lane
  const uint64_t lo = (uint64_t)x.x | ((uint64_t)x.y << 32), hi = (uint64_t)x.z | ((uint64_t)x.w << 32);
  const uint64_t mlo = s >= 64u ? 0ull : ~0ull << (s & 63u);
  const uint64_t mhi = s >= 128u ? 0ull : (s <= 64u ? ~0ull : ~0ull << ((s - 64u) & 63u));
  const int q = (int)pc - 4;  // G's first byte in the lane: -4..16
  const uint64_t g = G;
  const uint64_t glo = q < 0 ? (g >> ((uint32_t)(-8 * q) & 63u)) & (q == -4 ? 0ull : ~0ull)
                             : (q < 8 ? g << ((uint32_t)(8 * q) & 63u) : 0ull);
  const uint64_t ghi = q <= 4 ? 0ull
                              : (q < 8 ? g >> ((uint32_t)(64 - 8 * q) & 63u)
                                       : (q < 16 ? g << ((uint32_t)(8 * (q - 8)) & 63u) : 0ull));
  const uint64_t rlo = (lo & mlo) | glo, rhi = (hi & mhi) | ghi;
  return make_uint4((uint32_t)rlo, (uint32_t)(rlo >> 32), (uint32_t)rhi, (uint32_t)(rhi >> 32));
}

// Byte mask of a word with lb of its bytes before the end of the CRC'd data (lb >= 4: all, <= 0: none).
__host__ __device__ __forceinline__ uint32_t data_mask(int lb) {
  return lb >= 4 ? 0xFFFFFFFFu : (lb > 0 ? 0xFFFFFFFFu >> ((uint32_t)(32 - 8 * lb) & 31u) : 0u);
}

// The same from b = 8 lb (bits instead of bytes, any int): three VALU (clamp, 64-bit shift, not).
__host__ __device__ __forceinline__ uint32_t data_mask_bits(int b) {
  const uint32_t s = (uint32_t)(b < 0 ? 0 : (b > 32 ? 32 : b));
  return ~(uint32_t)(0xFFFFFFFFFFFFFFFFull << s);
}

// Byte mask of the word whose first byte sits at frame offset ob, for a frame of len bytes: the
// word's bytes at offsets [0, len).
__host__ __device__ __forceinline__ uint32_t frame_word_mask(int ob, uint32_t len) {
  const int lo = -ob < 0 ? 0 : (-ob > 4 ? 4 : -ob);  // bytes before the frame
  const int64_t h = (int64_t)len - ob;
  const int hi = h < 0 ? 0 : (h > 4 ? 4 : (int)h);    // bytes before the frame's end
  const uint32_t mhi = hi >= 4 ? ~0u : ((1u << ((uint32_t)(8 * hi) & 31u)) - 1u),
                 mlo = lo >= 4 ? 0u : (~0u << ((uint32_t)(8 * lo) & 31u));
  return mhi & mlo;
}

// The nibble-table key of the 8-lane finish with the slot constants rotated for a stream whose last
// word is slot e (frame_crc_varlen8.hip, group_lin8_rot): byte i = 4 * column multiplied in nibble
// step i, column = (4 col + ((i + u) & 3) + 31 - e) & 31 with u = (rot - (31 - e)) & 3.
__host__ __device__ __forceinline__ uint32_t rot_nibble_key(uint32_t col, uint32_t u, uint32_t e) {
  const uint32_t R = 31u - (e & 31u), sh = (8u * u) & 31u;
  const uint32_t steps = (0x03020100u >> sh) | (0x03020100u << ((32u - sh) & 31u));  // byte i = (i + u) & 3
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t rb = __builtin_amdgcn_perm(0u, R, 0u);  // R in every byte: one v_perm, not a 32-bit multiply
#else
  const uint32_t rb = R * 0x01010101u;
#endif
  return ((steps + (4u * (col & 7u)) * 0x01010101u + rb) & 0x1F1F1F1Fu) << 2;  // (the column part is per lane)
}

// Per-frame description for one 16-lane group.
struct FrameDesc {
  uint64_t start;  // byte offset of the frame in the batch buffer
  uint32_t len;    // frame length (bytes)
  uint32_t n;      // CRC'd bytes: len - 4, or len when len < 4
  int J;           // 256-byte blocks of the virtual stream
  int pad;         // 256*J - (n + 4)
};

__device__ __forceinline__ FrameDesc make_desc(uint64_t start, uint64_t len64) {
  FrameDesc d;
  d.start = start;
  d.len = (uint32_t)len64;
  d.n = d.len >= 4u ? d.len - 4u : d.len;
  const uint32_t E = d.n + 4u;
  d.J = (int)((E + 4u + 255u) >> 8);
  d.pad = d.J * 256 - (int)E;
  return d;
}

struct Lane {
  const char* lds;
  int lane;       // 0..63
  int col;        // lane within the frame's 16-lane group
  int grp;        // frame group 0..3 inside the wave
  bool odd;       // grp & 1
  uint32_t K;     // chain-table perm key: bytes [c4, c4 + 128, 0, 1], c4 = (lane & 31) * 4
  uint32_t K2;    // nibble-table perm key: byte i = column*4 of the slot multiplied in nibble step i
  uint32_t G;
};

struct Chains {
  uint32_t v0, v1, v2, v3;
  uint32_t tr;    // the frame's trailer word (lane col 15 only)
};

// One 256-byte block of the virtual stream: front fix (block 0, and the single word of block 1
// that straddles the G/data boundary when pad > 256), trailer capture on the last block, then the
// A^256 Horner step.
template <bool FREEZE>
__device__ __forceinline__ void process_block(const Lane& L, const FrameDesc& d, int blk, uint4 x, Chains& c) {
  {  // the last block's lane-15 last word is the trailer T: keep it, CRC it as zero
    const bool t = (L.col == 15) && (blk == d.J - 1);
    c.tr = t ? x.w : c.tr;
    x.w = t ? 0u : x.w;
  }
  if (blk == 0) {
    const int o = 16 * L.col - d.pad;
    c.v0 = fix_word(x.x, o, L.G);
    c.v1 = fix_word(x.y, o + 4, L.G);
    c.v2 = fix_word(x.z, o + 8, L.G);
    c.v3 = fix_word(x.w, o + 12, L.G);
    return;
  }
  if (blk == 1) x.x = fix_word(x.x, 256 + 16 * L.col - d.pad, L.G);
  const uint32_t n0 = chain_step(L.lds, c.v0, L.K, x.x);
  const uint32_t n1 = chain_step(L.lds, c.v1, L.K, x.y);
  const uint32_t n2 = chain_step(L.lds, c.v2, L.K, x.z);
  const uint32_t n3 = chain_step(L.lds, c.v3, L.K, x.w);
  if (FREEZE) {
    const bool act = blk < d.J;
    c.v0 = act ? n0 : c.v0;
    c.v1 = act ? n1 : c.v1;
    c.v2 = act ? n2 : c.v2;
    c.v3 = act ? n3 : c.v3;
  } else {
    c.v0 = n0; c.v1 = n1; c.v2 = n2; c.v3 = n3;
  }
}

// Stage the tables into LDS: one global round trip per thread (blockDim.x == 1024).
__device__ __forceinline__ void stage_tables(const KernelParams& p, char* lds) {
  const int t = threadIdx.x;
  const uint32_t cv = *as_global<g_u32>(p.chain_tab + t);
  const u32x4 n0 = *as_global<g_u32x4>(p.nib_img + 8 * t);
  const u32x4 n1 = *as_global<g_u32x4>(p.nib_img + 8 * t + 4);
  const uint32_t k = (uint32_t)t >> 8, e = (uint32_t)t & 255u;
  const uint32_t cbase = kChainBase + (k >> 1) * 65536u + e * 256u + (k & 1u) * 128u;
  const u32x4 cr = {cv, cv, cv, cv};
#pragma unroll
  for (int i = 0; i < 8; i++) *(u32x4*)(lds + cbase + 16 * i) = cr;
  *(u32x4*)(lds + 32 * t) = n0;
  *(u32x4*)(lds + 32 * t + 16) = n1;
  __syncthreads();
}

__device__ __forceinline__ void init_lane(Lane& L, char* lds, uint32_t G) {
  L.lds = lds;
  L.lane = threadIdx.x & 63;
  L.col = L.lane & 15;
  L.grp = L.lane >> 4;
  L.odd = (L.grp & 1) != 0;
  L.G = G;
  const uint32_t c4 = (uint32_t)(L.lane & 31) * 4u;
  L.K = c4 | ((c4 + 128u) << 8) | (1u << 24);
  uint32_t k2 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int sl = 4 * L.col + ((i + (L.odd ? 2 : 0)) & 3);
    k2 |= (uint32_t)(((sl >> 1) + 32 * (sl & 1)) * 4) << (8 * i);
  }
  L.K2 = k2;
}

// lin of the frame held by this 16-lane group (every lane of the group receives it).
__device__ __forceinline__ uint32_t group_lin(const Lane& L, const Chains& c) {
  const uint32_t X0 = L.odd ? c.v2 : c.v0, X1 = L.odd ? c.v3 : c.v1;
  const uint32_t X2 = L.odd ? c.v0 : c.v2, X3 = L.odd ? c.v1 : c.v3;
  const uint32_t lin = xor3(nib_mul<0>(L.lds, X0, L.K2), nib_mul<1>(L.lds, X1, L.K2), nib_mul<2>(L.lds, X2, L.K2)) ^
                       nib_mul<3>(L.lds, X3, L.K2);
  return row_xor16(lin);
}

// Fast-path item buffer: JC blocks of the set's four frames (one 16-byte piece per lane each).
template <int JC>
struct ItemBuf {
  uint4 x[JC];
};

template <bool NT>
__device__ __forceinline__ uint4 load_frame16(const uint8_t* q) {
  u32x4 v;
  if constexpr (NT)
    v = __builtin_nontemporal_load(as_global<g_u32x4>(q));
  else
    v = *as_global<g_u32x4>(q);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// One set's J blocks for this lane: block j at sbase + voff + 256*j, as raw buffer loads on a
// wave-uniform resource (base = sbase, in SGPRs) with this lane's loop-invariant 32-bit offset in
// a VGPR: no per-set VGPR address arithmetic, whose registers the allocator may otherwise take
// from a pending load (the next prefetch then waits for the previous one).
constexpr uint32_t kFixRecords = 0x7FFFFFF0u;  // far above any lane offset (host-checked stride)
constexpr int kFixRsrcWord3 = 0x00020000;      // gfx9-family raw buffer descriptor word 3
constexpr int kFixAuxNT = 2;                   // cache policy of the frame loads: nt (streaming)
template <int J>
__device__ __forceinline__ void load_set(const uint8_t* sbase, uint32_t voff, ItemBuf<J>& b) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)sbase, 0, (int)kFixRecords, kFixRsrcWord3);
#pragma unroll
  for (int j = 0; j < J; j++) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(voff + 256u * j), 0, kFixAuxNT);
    b.x[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// Stores written as inline asm: hipcc's wait-count model never sees them, so it keeps counting
// loads only (a store it could see would make every later load wait vmcnt(0), since loads and
// stores share vmcnt and may complete out of order).  A hidden store can only make a counted
// wait stricter (loads return in order), never looser.
__device__ __forceinline__ void st_u32_hidden(uint32_t* a, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off" : : "v"(a), "v"(v));
}
__device__ __forceinline__ void st_u8_hidden(uint8_t* a, uint32_t v) {
  asm volatile("global_store_byte %0, %1, off" : : "v"(a), "v"(v));
}

// The tables are staged as 1024 chunks (one chain-table word replicated 32x + 32 B of the nibble
// image each); a workgroup of THREADS threads stages ceil(1024 / THREADS) chunks per thread (the
// last round partially when THREADS does not divide 1024, e.g. 768).
struct StageRegs {
  uint32_t cv;
  u32x4 n0, n1;
};
template <int THREADS = 1024>
struct StageSet {
  static constexpr int kRounds = (1024 + THREADS - 1) / THREADS;
  StageRegs r[kRounds];
};

template <int THREADS = 1024>
__device__ __forceinline__ StageSet<THREADS> stage_load(const KernelParams& p) {
  StageSet<THREADS> s;
#pragma unroll
  for (int i = 0; i < StageSet<THREADS>::kRounds; i++) {
    const int t = min((int)threadIdx.x + i * THREADS, 1023);  // (a partial round re-reads chunk 1023)
    s.r[i].cv = *as_global<g_u32>(p.chain_tab + t);
    s.r[i].n0 = *as_global<g_u32x4>(p.nib_img + 8 * t);
    s.r[i].n1 = *as_global<g_u32x4>(p.nib_img + 8 * t + 4);
  }
  return s;
}

// LDS writes of the staged tables, then a workgroup barrier that orders LDS only: data
// prefetches issued before it stay in flight (no vmcnt(0) at the barrier).
template <int THREADS = 1024>
__device__ __forceinline__ void stage_store(const StageSet<THREADS>& s, char* lds) {
#pragma unroll
  for (int i = 0; i < StageSet<THREADS>::kRounds; i++) {
    const int t = (int)threadIdx.x + i * THREADS;
    if (1024 % THREADS != 0 && t >= 1024) break;
    const StageRegs& r = s.r[i];
    const uint32_t k = (uint32_t)t >> 8, e = (uint32_t)t & 255u;
    const uint32_t cbase = kChainBase + (k >> 1) * 65536u + e * 256u + (k & 1u) * 128u;
    const u32x4 cr = {r.cv, r.cv, r.cv, r.cv};
#pragma unroll
    for (int j = 0; j < 8; j++) *(u32x4*)(lds + cbase + 16 * j) = cr;
    *(u32x4*)(lds + 32 * t) = r.n0;
    *(u32x4*)(lds + 32 * t + 16) = r.n1;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
}  // namespace ufc_dev
