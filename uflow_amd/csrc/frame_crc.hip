// frame_crc.hip -- batched frame CRC-32 (uflow, polynomial 0x132c00699) for MI355X / gfx950.
//
// Replaces, in batch, the per-frame loop of src/frame/serial/crc.rs:94-104 used by the CRC gate
// of Frame::read (src/frame/serial/mod.rs:675-690) and by the frame seal
// (src/frame/serial/mod.rs:463-470, src/frame/serial/build.rs:151-159).
//
// Algorithm (all linear over GF(2), register domain; see crc_math.hpp):
//   * A frame's n CRC bytes are right-aligned into a virtual stream of J*256 bytes:
//       [ zeros | G (4 bytes) | frame[0..n) ],  J = ceil((n+4)/256),  pad = 256*J - n  (4..259).
//     G = A^-4(~0) makes the linear CRC of the stream equal the reference's register after
//     init ~0, so crc = ~lin(stream).
//   * Virtual word w (4 bytes) belongs to slot s = w mod 64.  Slot s runs a Horner chain over the
//     J blocks with the constant A^256:  V_s <- A^256(V_s) ^ word.  A^256 is applied with four
//     byte tables held in LDS, replicated 32x so that lane l always reads bank l mod 32
//     (conflict-free ds_read_b32 whatever the data).
//   * lin = XOR_s A^(4(64-s))(V_s): each slot's final value is multiplied by its own constant via
//     per-slot nibble tables in LDS (8 lookups), then XOR-reduced inside the frame's 16 lanes
//     with DPP.
// Wave layout: 4 frames per wave, 16 lanes per frame; lane col of a frame loads the 16 bytes
// at 16*col of each 256-byte block with one global_load_dwordx4 (non-temporal), so a
// wave-instruction reads four contiguous 256-byte runs.  Lane col holds slots 4*col+b (b=0..3)
// in four independent chains.  Frames whose block count differs inside a wave (varlen) run the
// wave's maximum and freeze their chains after their own last block.
//
// LDS (one 1024-thread workgroup per CU, 160 KiB), laid out so that every table address is ONE
// v_perm_b32 (byte select) of the value being looked up:
//   [0, 32K)     nibble tables: slot s, nibble k, value e at byte k*4096 + e*256 + c(s)*4, with
//                c(s) = (s >> 1) + 32*(s & 1); k*4096 goes in the ds_read offset.  In nibble step i,
//                frames in odd 16-lane groups use chain (i+2)&3, so the 32 lanes of an LDS
//                lane-group hit 32 distinct banks.
//   [32K, 160K)  chain tables (two per 256-byte row): table k = 2p + t, entry e, copy c at byte
//                32768 + p*65536 + e*256 + t*128 + c*4, c = lane & 31 (bank = c: conflict-free).
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

__device__ __forceinline__ uint32_t lds_ld(const char* lds, uint32_t byteoff) {
  return *(const uint32_t*)(lds + byteoff);
}

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

// Multiply v by the constant of the slot whose column byte-offset is byte `i` of K2:
// nibble k of v indexes row (k*16 + e); address bytes [K2.byte_i, nibble, 0, 0] + k*4096.
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
  return xor3(xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6]), r[7], 0u);
}

// XOR over the 16 lanes of a DPP row; every lane of the row receives the total.
__device__ __forceinline__ uint32_t row_xor16(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// Word of the virtual stream whose first byte sits at frame offset o (o < 0: before the frame).
// Bytes at frame offsets [-4, 0) are G's bytes, below -4 zeros, from 0 on the loaded data v.
__device__ __forceinline__ uint32_t fix_word(uint32_t v, int o, uint32_t G) {
  const uint64_t pv = (uint64_t)G << 32;
  const int sh = 8 * (o + 8);                       // in [8, 56] when o in (-8, 0)
  const uint32_t pre = (uint32_t)(pv >> (sh & 63));
  const uint32_t dm = (o > -4) ? (0xFFFFFFFFu << ((8 * (-o)) & 31)) : 0u;
  const uint32_t mixed = (v & dm) | (pre & ~dm);
  return (o >= 0) ? v : ((o <= -8) ? 0u : mixed);
}

// Per-frame description for one 16-lane group.
struct FrameDesc {
  uint64_t start;  // byte offset of the frame in the batch buffer
  uint32_t len;    // frame length (bytes)
  uint32_t n;      // CRC'd bytes: len - 4, or len when len < 4
  int J;           // 256-byte blocks of the virtual stream
  int pad;         // 256*J - n  (4..259)
};

__device__ __forceinline__ FrameDesc make_desc(uint64_t start, uint64_t len64) {
  FrameDesc d;
  d.start = start;
  d.len = (uint32_t)len64;
  d.n = d.len >= 4u ? d.len - 4u : d.len;
  d.J = (int)((d.n + 4u + 255u) >> 8);
  d.pad = d.J * 256 - (int)d.n;
  return d;
}

struct Lane {
  const char* lds;
  int col;        // lane within the frame's 16-lane group
  int grp;        // frame group 0..3 inside the wave
  bool odd;       // grp & 1
  uint32_t K;     // chain-table perm key: bytes [c4, c4 + 128, 0, 1], c4 = (lane & 31) * 4
  uint32_t K2;    // nibble-table perm key: byte i = column*4 of the slot multiplied in nibble step i
  uint32_t G;
};

struct Chains {
  uint32_t v0, v1, v2, v3;
};

// One 256-byte block of the virtual stream: front fix (block 0, and the single word of block 1
// that straddles the G/data boundary when pad > 256), then the A^256 Horner step.
template <bool FREEZE>
__device__ __forceinline__ void process_block(const Lane& L, const FrameDesc& d, int blk, uint4 x, Chains& c) {
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

// Slot constants, 16-lane XOR, outputs of one frame set.
template <bool SEAL>
__device__ __forceinline__ void finish_set(const Lane& L, const KernelParams& p, uint64_t set, const FrameDesc& d,
                                           const Chains& c, uint32_t trailer_le) {
  const uint32_t X0 = L.odd ? c.v2 : c.v0, X1 = L.odd ? c.v3 : c.v1;
  const uint32_t X2 = L.odd ? c.v0 : c.v2, X3 = L.odd ? c.v1 : c.v3;
  uint32_t acc = xor3(nib_mul<0>(L.lds, X0, L.K2), nib_mul<1>(L.lds, X1, L.K2), nib_mul<2>(L.lds, X2, L.K2)) ^
                 nib_mul<3>(L.lds, X3, L.K2);
  acc = row_xor16(acc);
  const uint32_t crc = ~acc;
  const uint64_t f = set * 4 + (uint64_t)L.grp;
  if (L.col == 0 && f < p.nframes) {
    if (SEAL) {
      if (d.len >= 4u) {
        g_u8w* t = as_global<g_u8w>(p.wbytes + d.start + d.n);
        t[0] = (uint8_t)(crc >> 24);
        t[1] = (uint8_t)(crc >> 16);
        t[2] = (uint8_t)(crc >> 8);
        t[3] = (uint8_t)crc;
      }
      if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = crc;
    } else {
      if (p.crc_out) *as_global<g_u32w>(p.crc_out + f) = crc;
      if (p.valid_out) {
        uint8_t ok = 0;
        if (d.len >= 5u) ok = (__builtin_bswap32(trailer_le) == crc) ? 1 : 0;
        *as_global<g_u8w>(p.valid_out + f) = ok;
      }
    }
  }
}

// Slow path for a whole frame set (edge/tail sets: frames whose fast loads could leave the
// buffer).  Byte loads restricted to [0, n) of the frame, one block at a time, not unrolled, so
// that it adds no register pressure to the fast path.
template <bool FREEZE, bool SEAL>
__device__ __forceinline__ void slow_set(const Lane& L, const KernelParams& p, uint64_t set, const FrameDesc& d,
                                         int nblocks) {
  Chains c{0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int blk = 0; blk < nblocks; blk++) {
    const int bl = min(blk, d.J - 1);
    uint32_t w[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int o = 256 * bl + 16 * L.col + 4 * b - d.pad;
      uint32_t acc = 0;
#pragma unroll 1
      for (int k = 0; k < 4; k++) {
        const int ob = o + k;
        if (ob >= 0 && ob < (int)d.n) acc |= (uint32_t)*as_global<g_u8>(p.bytes + d.start + (uint64_t)ob) << (8 * k);
      }
      w[b] = acc;
    }
    process_block<true>(L, d, blk, make_uint4(w[0], w[1], w[2], w[3]), c);
  }
  uint32_t tr = 0;
  if (!SEAL && d.len >= 5u) {
    g_u8* t = as_global<g_u8>(p.bytes + d.start + d.n);
    tr = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
  }
  finish_set<SEAL>(L, p, set, d, c, tr);
}

// Fast-path item buffer: JC blocks of each of the NS frame sets of a wave-iteration, plus the
// frames' trailer words.  The trailer word is loaded together with the data so that no load
// is issued after the next item's prefetch (in-order vmcnt would force a wait on it).
template <int NS, int JC>
struct ItemBuf {
  uint4 x[NS][JC];
  uint32_t tr[NS];  // 4 trailer bytes (little-endian load); validate mode only
};

template <int NS, int JC, bool SEAL, bool NO_TRAILER = false>
__device__ __forceinline__ void load_item(const uint8_t* const (&lane_base)[NS], const uint8_t* const (&trailer)[NS],
                                          int chunk, ItemBuf<NS, JC>& b) {
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const uint8_t* q = lane_base[k] + (int64_t)chunk * (JC * 256);
#pragma unroll
    for (int j = 0; j < JC; j++) {
      const u32x4 v = __builtin_nontemporal_load(as_global<g_u32x4>(q + 256 * j));
      b.x[k][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
    if (!SEAL && !NO_TRAILER) b.tr[k] = *as_global<g_u32>(trailer[k]);
    if (NO_TRAILER) b.tr[k] = 0;
  }
}

// Blocks j of all NS sets are processed back to back (j outer, k inner): 4*NS independent
// chains per lane hide the LDS latency of each Horner step.
template <int NS, int JC, bool FREEZE, bool CHUNK0>
__device__ __forceinline__ void compute_item(const Lane& L, const FrameDesc (&d)[NS], int chunk,
                                             const ItemBuf<NS, JC>& b, Chains (&c)[NS]) {
#pragma unroll
  for (int j = 0; j < JC; j++)
#pragma unroll
    for (int k = 0; k < NS; k++) process_block<FREEZE>(L, d[k], CHUNK0 ? j : chunk * JC + j, b.x[k][j], c[k]);
}

template <int NS, int JC, int MODE>
__global__ __launch_bounds__(1024) void frame_crc_kernel(const KernelParams p) {
  constexpr bool VARLEN = (MODE & kModeVarlen) != 0;
  constexpr bool SEAL = (MODE & kModeSeal) != 0;
  constexpr bool FREEZE = VARLEN || (MODE & kModeFreeze) != 0;  // blocks past J may occur in a chunk
  constexpr bool NO_COMPUTE = (MODE & kModeAblateCompute) != 0;  // tuning builds only
  constexpr bool NO_LOADS = (MODE & kModeAblateLoads) != 0;      // tuning builds only
  constexpr bool NO_TRAILER = (MODE & 32) != 0;                  // tuning builds only
  constexpr bool NO_STORES = (MODE & 64) != 0;                   // tuning builds only
  constexpr bool NO_STAGING = (MODE & 128) != 0;                 // tuning builds only
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // ---- stage the tables into LDS: one global round trip per thread ----
  if (!NO_STAGING) {
    const int t = threadIdx.x;  // blockDim.x == 1024 (set by the launcher)
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
  }
  __syncthreads();

  Lane L;
  L.lds = lds;
  const int lane = threadIdx.x & 63;
  L.col = lane & 15;
  L.grp = lane >> 4;
  L.odd = (L.grp & 1) != 0;
  {
    const uint32_t c4 = (uint32_t)(lane & 31) * 4u;
    L.K = c4 | ((c4 + 128u) << 8) | (1u << 24);
    uint32_t k2 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int s = 4 * L.col + ((i + (L.odd ? 2 : 0)) & 3);
      k2 |= (uint32_t)(((s >> 1) + 32 * (s & 1)) * 4) << (8 * i);
    }
    L.K2 = k2;
  }
  L.G = p.G;
  const uint64_t nsets = (p.nframes + 3) >> 2;        // 4 frames per set (one per 16-lane group)
  const uint64_t nsup = (nsets + NS - 1) / NS;        // NS sets per wave-iteration
  const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
  // Wave-uniform item counter, made provably uniform (SGPR) so that loop control compiles to
  // scalar branches and no load sits behind an exec mask.
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t sup = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wid;
  if (sup >= nsup) return;
  // End of the readable batch bytes (fast loads must stay below it).
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
  auto item_nch = [&](const FrameDesc (&dd)[NS]) -> int {
    int m = 0;
#pragma unroll
    for (int k = 0; k < NS; k++) m = max(m, dd[k].J);
    return (wave_max(m) + JC - 1) / JC;
  };
  // Fast loads read [start - pad, start - pad + 256*JC*nch) of every frame: stay in the buffer.
  auto item_slow = [&](const FrameDesc (&dd)[NS], int nch) -> bool {
    int bad = 0;
#pragma unroll
    for (int k = 0; k < NS; k++)
      bad |= (dd[k].start < (uint64_t)dd[k].pad ||
              dd[k].start - dd[k].pad + (uint64_t)(256 * JC) * nch > buf_end) ? 1 : 0;
    return wave_max(bad) != 0;
  };
  auto trailer_ptr = [&](const FrameDesc& dd) -> const uint8_t* {
    return p.bytes + dd.start + (dd.len >= 4u ? dd.n : 0u);  // frames without trailer: harmless address
  };
  auto slow_item = [&](uint64_t s, const FrameDesc (&dd)[NS], int nch) {
#pragma unroll 1
    for (int k = 0; k < NS; k++)
      if (s * NS + k < nsets) slow_set<FREEZE, SEAL>(L, p, s * NS + k, dd[k], nch * JC);
  };

  FrameDesc d[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) d[k] = desc_now(sup * NS + k);
  int nch = item_nch(d);
  // Edge items (first sets of the batch) through the slow path.
  while (item_slow(d, nch)) {
    slow_item(sup, d, nch);
    sup += W;
    if (sup >= nsup) return;
#pragma unroll
    for (int k = 0; k < NS; k++) d[k] = desc_now(sup * NS + k);
    nch = item_nch(d);
  }

  // Varlen: the offsets of the NEXT item are loaded one item ahead.
  uint64_t pre_a[NS], pre_b[NS];
  auto prefetch_offsets = [&](uint64_t s2) {
    if (VARLEN) {
#pragma unroll
      for (int k = 0; k < NS; k++) {
        const uint64_t f = frame_index((s2 < nsup ? s2 : sup) * NS + k);
        pre_a[k] = *as_global<g_u64>(p.offsets + f);
        pre_b[k] = *as_global<g_u64>(p.offsets + f + 1);
      }
    }
  };
  auto desc_next = [&](uint64_t s2, FrameDesc (&dd)[NS]) {
#pragma unroll
    for (int k = 0; k < NS; k++)
      dd[k] = VARLEN ? make_desc(pre_a[k], pre_b[k] - pre_a[k]) : make_desc(frame_index(s2 * NS + k) * p.stride, p.frame_len);
  };
  prefetch_offsets(sup + W);

  // Main loop, double-buffered over items (super-set, chunk): the next item's loads are in
  // flight while the current one is computed.  Buffers alternate explicitly (a register copy
  // would make hipcc wait for every outstanding load at the loop head).
  Chains c[NS];
  int chunk = 0;
  const uint8_t* base_cur[NS];
  const uint8_t* tr_cur[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    base_cur[k] = p.bytes + d[k].start - d[k].pad + 16 * L.col;
    tr_cur[k] = trailer_ptr(d[k]);
  }
  bool go_slow = false;  // the next item needs the slow path (tail of the batch)
  auto step = [&](ItemBuf<NS, JC>& cur, ItemBuf<NS, JC>& nxt) -> bool {
    uint64_t sup2 = sup;
    int chunk2 = chunk + 1, nch2 = nch;
    FrameDesc d2[NS];
    const uint8_t* base2[NS];
    const uint8_t* tr2[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) { d2[k] = d[k]; base2[k] = base_cur[k]; tr2[k] = tr_cur[k]; }
    const bool newitem = (chunk2 == nch);
    bool more = true;
    if (newitem) {
      sup2 = sup + W;
      chunk2 = 0;
      more = sup2 < nsup;
      if (more) {
        desc_next(sup2, d2);
        nch2 = item_nch(d2);
        prefetch_offsets(sup2 + W);
        if (item_slow(d2, nch2)) {
          go_slow = true;
          more = false;
        }
#pragma unroll
        for (int k = 0; k < NS; k++) {
          base2[k] = p.bytes + d2[k].start - d2[k].pad + 16 * L.col;
          tr2[k] = trailer_ptr(d2[k]);
        }
      }
    }
    // Unconditional prefetch (the last one re-reads the current item): a load behind a branch
    // makes the waitcnt pass assume it was skipped and wait for the whole prefetch.
    {
      const uint8_t* lb[NS];
      const uint8_t* lt[NS];
#pragma unroll
      for (int k = 0; k < NS; k++) { lb[k] = more ? base2[k] : base_cur[k]; lt[k] = more ? tr2[k] : tr_cur[k]; }
      if (NO_LOADS) {
#pragma unroll
        for (int k = 0; k < NS; k++)
#pragma unroll
          for (int j = 0; j < JC; j++) nxt.x[k][j] = make_uint4(cur.x[k][j].y, cur.x[k][j].z, cur.x[k][j].w, cur.x[k][j].x ^ chunk2);
      } else {
        load_item<NS, JC, SEAL, NO_TRAILER>(lb, lt, more ? chunk2 : chunk, nxt);
      }
    }
    if (NO_COMPUTE) {
#pragma unroll
      for (int k = 0; k < NS; k++)
#pragma unroll
        for (int j = 0; j < JC; j++) c[k].v0 ^= cur.x[k][j].x ^ cur.x[k][j].y ^ cur.x[k][j].z ^ cur.x[k][j].w;
    } else if (chunk == 0)
      compute_item<NS, JC, FREEZE, true>(L, d, 0, cur, c);
    else {
      __builtin_assume(chunk >= 1);
      compute_item<NS, JC, FREEZE, false>(L, d, chunk, cur, c);
    }
    if (newitem) {
#pragma unroll
      for (int k = 0; k < NS; k++) {
        if (NO_STORES) {
          if (c[k].v0 == 0x12345678u && c[k].v1 == cur.tr[k]) *as_global<g_u32w>(p.crc_out) = 1u;  // keep live
        } else {
          finish_set<SEAL>(L, p, sup * NS + k, d[k], c[k], cur.tr[k]);
        }
      }
    }
    if (go_slow) {  // hand the tail item over to the slow loop below
      sup = sup2;
#pragma unroll
      for (int k = 0; k < NS; k++) d[k] = d2[k];
      nch = nch2;
      return false;
    }
    sup = sup2; chunk = chunk2; nch = nch2;
#pragma unroll
    for (int k = 0; k < NS; k++) { d[k] = d2[k]; base_cur[k] = base2[k]; tr_cur[k] = tr2[k]; }
    return more;
  };
  {
    ItemBuf<NS, JC> A, B;
    load_item<NS, JC, SEAL, NO_TRAILER>(base_cur, tr_cur, 0, A);
    while (step(A, B) && step(B, A)) {
    }
  }
  // Tail items (last of the batch) through the slow path.
  if (go_slow) {
    for (; sup < nsup; sup += W) {
#pragma unroll
      for (int k = 0; k < NS; k++) d[k] = desc_now(sup * NS + k);
      nch = item_nch(d);
      slow_item(sup, d, nch);
    }
  }
}

#define UFC_INST_MODES(NS, JC)                                                                          \
  template __global__ void frame_crc_kernel<NS, JC, 0>(const KernelParams);                             \
  template __global__ void frame_crc_kernel<NS, JC, kModeSeal>(const KernelParams);                     \
  template __global__ void frame_crc_kernel<NS, JC, kModeFreeze>(const KernelParams);                   \
  template __global__ void frame_crc_kernel<NS, JC, kModeFreeze | kModeSeal>(const KernelParams);       \
  template __global__ void frame_crc_kernel<NS, JC, kModeVarlen>(const KernelParams);                   \
  template __global__ void frame_crc_kernel<NS, JC, kModeVarlen | kModeSeal>(const KernelParams);

#define UFC_CONFIGS(X) X(1, 1) X(1, 2) X(1, 3) X(1, 6) X(2, 1) X(2, 2) X(2, 3) X(4, 1)

UFC_CONFIGS(UFC_INST_MODES)

#ifdef UFC_TUNING
template __global__ void frame_crc_kernel<1, 6, kModeAblateCompute>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, kModeAblateLoads>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, kModeAblateCompute | 32>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, kModeAblateCompute | 32 | 64>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, kModeAblateCompute | 32 | 64 | 128>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, 32>(const KernelParams);
template __global__ void frame_crc_kernel<1, 6, 64>(const KernelParams);
#endif

const void* kernel_symbol(int ns, int jc, int mode) {
#define UFC_PICK(NS, JC)                                                                                   \
  if (ns == NS && jc == JC) {                                                                              \
    switch (mode) {                                                                                        \
      case 0: return (const void*)frame_crc_kernel<NS, JC, 0>;                                            \
      case kModeSeal: return (const void*)frame_crc_kernel<NS, JC, kModeSeal>;                            \
      case kModeFreeze: return (const void*)frame_crc_kernel<NS, JC, kModeFreeze>;                        \
      case kModeFreeze | kModeSeal: return (const void*)frame_crc_kernel<NS, JC, kModeFreeze | kModeSeal>;\
      case kModeVarlen: return (const void*)frame_crc_kernel<NS, JC, kModeVarlen>;                        \
      case kModeVarlen | kModeSeal: return (const void*)frame_crc_kernel<NS, JC, kModeVarlen | kModeSeal>;\
      default: break;                                                                                      \
    }                                                                                                      \
  }
  UFC_CONFIGS(UFC_PICK)
#undef UFC_PICK
#ifdef UFC_TUNING
  if (ns == 1 && jc == 6 && mode == kModeAblateCompute) return (const void*)frame_crc_kernel<1, 6, kModeAblateCompute>;
  if (ns == 1 && jc == 6 && mode == kModeAblateLoads) return (const void*)frame_crc_kernel<1, 6, kModeAblateLoads>;
  if (ns == 1 && jc == 6 && mode == (kModeAblateCompute | 32)) return (const void*)frame_crc_kernel<1, 6, kModeAblateCompute | 32>;
  if (ns == 1 && jc == 6 && mode == (kModeAblateCompute | 32 | 64)) return (const void*)frame_crc_kernel<1, 6, kModeAblateCompute | 32 | 64>;
  if (ns == 1 && jc == 6 && mode == (kModeAblateCompute | 32 | 64 | 128)) return (const void*)frame_crc_kernel<1, 6, kModeAblateCompute | 32 | 64 | 128>;
  if (ns == 1 && jc == 6 && mode == 32) return (const void*)frame_crc_kernel<1, 6, 32>;
  if (ns == 1 && jc == 6 && mode == 64) return (const void*)frame_crc_kernel<1, 6, 64>;
#endif
  return nullptr;
}

bool config_available(int ns, int jc) {
#define UFC_HAVE(NS, JC) if (ns == NS && jc == JC) return true;
  UFC_CONFIGS(UFC_HAVE)
#undef UFC_HAVE
  return false;
}

}  // namespace ufc_dev
