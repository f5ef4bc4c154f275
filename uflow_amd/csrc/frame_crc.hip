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
// LDS (one 1024-thread workgroup per CU, 160 KiB):
//   [0, 128K)    chain tables: entry e of table k, copy c at byte k*32768 + e*128 + c*4
//   [128K,160K)  nibble tables: slot s, nibble k, value e at byte 131072 + (k*16+e)*256 + c(s)*4,
//                c(s) = (s >> 1) + 32*(s & 1).  In nibble step i, frames in odd 16-lane groups use
//                chain (i+2)&3, so the 32 lanes of an LDS lane-group hit 32 distinct banks.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "frame_crc_kernels.hpp"

namespace ufc_dev {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_ld(const char* lds, uint32_t byteoff) {
  return *(const uint32_t*)(lds + byteoff);
}

// A^256(v) with the replicated byte tables; c4 = (lane & 31) * 4.
__device__ __forceinline__ uint32_t chain_step(const char* lds, uint32_t v, uint32_t c4) {
  const uint32_t a0 = ((v << 7) & 0x7F80u) | c4;
  const uint32_t a1 = ((v >> 1) & 0x7F80u) | c4;
  const uint32_t a2 = ((v >> 9) & 0x7F80u) | c4;
  const uint32_t a3 = ((v >> 17) & 0x7F80u) | c4;
  return lds_ld(lds, a0) ^ lds_ld(lds, a1 + 32768u) ^ lds_ld(lds, a2 + 65536u) ^ lds_ld(lds, a3 + 98304u);
}

// Multiply by the slot constant whose nibble-table column starts at byte `base`.
__device__ __forceinline__ uint32_t nib_mul(const char* lds, uint32_t v, uint32_t base) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int sh = 4 * k - 8;  // nibble k -> bits [8, 12) of the row offset (row stride 256 B)
    const uint32_t e = (sh >= 0) ? (v >> sh) : (v << (-sh));
    r ^= lds_ld(lds, (e & 0xF00u) + base + (uint32_t)(k * 4096));
  }
  return r;
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
  uint32_t c4;    // (lane & 31) * 4
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
  const uint32_t n0 = chain_step(L.lds, c.v0, L.c4) ^ x.x;
  const uint32_t n1 = chain_step(L.lds, c.v1, L.c4) ^ x.y;
  const uint32_t n2 = chain_step(L.lds, c.v2, L.c4) ^ x.z;
  const uint32_t n3 = chain_step(L.lds, c.v3, L.c4) ^ x.w;
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
                                           const Chains& c) {
  const uint32_t X0 = L.odd ? c.v2 : c.v0, X1 = L.odd ? c.v3 : c.v1;
  const uint32_t X2 = L.odd ? c.v0 : c.v2, X3 = L.odd ? c.v1 : c.v3;
  uint32_t acc = 0;
  const uint32_t X[4] = {X0, X1, X2, X3};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int s = 4 * L.col + ((i + (L.odd ? 2 : 0)) & 3);
    const uint32_t nbase = 131072u + (uint32_t)((s >> 1) + 32 * (s & 1)) * 4u;
    acc ^= nib_mul(L.lds, X[i], nbase);
  }
  acc = row_xor16(acc);
  const uint32_t crc = ~acc;
  const uint64_t f = set * 4 + (uint64_t)L.grp;
  if (L.col == 0 && f < p.nframes) {
    if (SEAL) {
      if (d.len >= 4u) {
        uint8_t* t = p.wbytes + d.start + d.n;
        t[0] = (uint8_t)(crc >> 24);
        t[1] = (uint8_t)(crc >> 16);
        t[2] = (uint8_t)(crc >> 8);
        t[3] = (uint8_t)crc;
      }
      if (p.crc_out) p.crc_out[f] = crc;
    } else {
      if (p.crc_out) p.crc_out[f] = crc;
      if (p.valid_out) {
        uint8_t ok = 0;
        if (d.len >= 5u) {
          const uint8_t* t = p.bytes + d.start + d.n;
          const uint32_t rx = ((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | (uint32_t)t[3];
          ok = (rx == crc) ? 1 : 0;
        }
        p.valid_out[f] = ok;
      }
    }
  }
}

// Slow path for a whole frame set (edge/tail sets: frames whose fast loads could leave the
// buffer).  Byte loads clamped into [0, n) of the frame; one block at a time, not unrolled.
template <bool FREEZE, bool SEAL>
__device__ __noinline__ void slow_set(const Lane& L, const KernelParams& p, uint64_t set, const FrameDesc& d,
                                      int nblocks) {
  Chains c{0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int blk = 0; blk < nblocks; blk++) {
    const int bl = min(blk, d.J - 1);
    uint32_t w[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int o = 256 * bl + 16 * L.col + 4 * b + k - d.pad;
        const int oc = min(max(o, 0), max((int)d.n - 1, 0));
        const uint32_t byte = (d.n > 0u) ? (uint32_t)p.bytes[d.start + (uint64_t)oc] : 0u;
        acc |= ((o >= 0) ? byte : 0u) << (8 * k);
      }
      w[b] = acc;
    }
    process_block<true>(L, d, blk, make_uint4(w[0], w[1], w[2], w[3]), c);
  }
  finish_set<SEAL>(L, p, set, d, c);
}

template <int JC, bool FREEZE, bool CHUNK0>
__device__ __forceinline__ void compute_chunk(const Lane& L, const FrameDesc& d, int chunk, const uint4 (&x)[JC],
                                              Chains& c) {
#pragma unroll
  for (int j = 0; j < JC; j++) process_block<FREEZE>(L, d, CHUNK0 ? j : chunk * JC + j, x[j], c);
}

// Fast load of one chunk: one non-temporal dwordx4 per block at base + 256*blk (base already
// includes 16*col - pad; block 0 may read bytes before the frame, which fix_word masks).
template <int JC>
__device__ __forceinline__ void load_chunk(const uint8_t* lane_base, int chunk, uint4 (&x)[JC]) {
  const uint8_t* q = lane_base + (int64_t)chunk * (JC * 256);
#pragma unroll
  for (int j = 0; j < JC; j++) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)(q + 256 * j));
    x[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <int JC, int MODE>
__global__ __launch_bounds__(1024) void frame_crc_kernel(const KernelParams p) {
  constexpr bool VARLEN = (MODE & kModeVarlen) != 0;
  constexpr bool SEAL = (MODE & kModeSeal) != 0;
  constexpr bool FREEZE = VARLEN || (MODE & kModeFreeze) != 0;  // blocks past J may occur in a chunk
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // ---- stage the tables into LDS: one global round trip per thread ----
  {
    const int t = threadIdx.x;  // blockDim.x == 1024 (set by the launcher)
    const uint32_t cv = p.chain_tab[t];
    const u32x4 n0 = *(const u32x4*)(p.nib_img + 8 * t);
    const u32x4 n1 = *(const u32x4*)(p.nib_img + 8 * t + 4);
    const uint32_t cbase = (uint32_t)(t >> 8) * 32768u + (uint32_t)(t & 255) * 128u;
    const u32x4 cr = {cv, cv, cv, cv};
#pragma unroll
    for (int i = 0; i < 8; i++) *(u32x4*)(lds + cbase + 16 * i) = cr;
    *(u32x4*)(lds + 131072 + 32 * t) = n0;
    *(u32x4*)(lds + 131072 + 32 * t + 16) = n1;
  }
  __syncthreads();

  Lane L;
  L.lds = lds;
  const int lane = threadIdx.x & 63;
  L.col = lane & 15;
  L.grp = lane >> 4;
  L.odd = (L.grp & 1) != 0;
  L.c4 = (uint32_t)(lane & 31) * 4u;
  L.G = p.G;
  const uint64_t nsets = (p.nframes + 3) >> 2;  // 4 frames per wave-iteration
  const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
  uint64_t set = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (set >= nsets) return;
  // End of the readable batch bytes (fast loads must stay below it).
  const uint64_t buf_end = VARLEN ? p.offsets[p.nframes] : (p.nframes - 1) * p.stride + p.frame_len;

  auto frame_index = [&](uint64_t s) -> uint64_t {
    const uint64_t f = s * 4 + (uint64_t)L.grp;
    return f < p.nframes ? f : p.nframes - 1;
  };
  auto desc_now = [&](uint64_t s) -> FrameDesc {
    const uint64_t f = frame_index(s);
    if (VARLEN) {
      const uint64_t a = p.offsets[f], b = p.offsets[f + 1];
      return make_desc(a, b - a);
    }
    return make_desc(f * p.stride, p.frame_len);
  };
  auto wave_any = [&](int v) -> bool {
    return (__builtin_amdgcn_readlane(v, 0) | __builtin_amdgcn_readlane(v, 16) | __builtin_amdgcn_readlane(v, 32) |
            __builtin_amdgcn_readlane(v, 48)) != 0;
  };
  auto wave_nch = [&](int J) -> int {
    int m = __builtin_amdgcn_readlane(J, 0);
    m = max(m, __builtin_amdgcn_readlane(J, 16));
    m = max(m, __builtin_amdgcn_readlane(J, 32));
    m = max(m, __builtin_amdgcn_readlane(J, 48));
    return (m + JC - 1) / JC;
  };
  // Fast loads of the set read [start - pad, start - pad + 256*JC*nch); they must stay in the buffer.
  auto wave_slow = [&](const FrameDesc& d, int nch) -> bool {
    const bool bad = d.start < (uint64_t)d.pad || d.start - d.pad + (uint64_t)(256 * JC) * nch > buf_end;
    return wave_any(bad ? 1 : 0);
  };

  FrameDesc d = desc_now(set);
  int nch = wave_nch(d.J);
  // Edge sets (first sets of the batch) through the slow path.
  while (wave_slow(d, nch)) {
    slow_set<FREEZE, SEAL>(L, p, set, d, nch * JC);
    set += W;
    if (set >= nsets) return;
    d = desc_now(set);
    nch = wave_nch(d.J);
  }

  // Varlen: the offsets of the NEXT set are loaded one set ahead.
  uint64_t pre_a = 0, pre_b = 0;
  auto prefetch_offsets = [&](uint64_t s2) {
    if (VARLEN) {
      const uint64_t f = frame_index(s2 < nsets ? s2 : set);
      pre_a = p.offsets[f];
      pre_b = p.offsets[f + 1];
    }
  };
  auto desc_next = [&](uint64_t s2) -> FrameDesc {
    if (VARLEN) return make_desc(pre_a, pre_b - pre_a);
    return make_desc(frame_index(s2) * p.stride, p.frame_len);
  };
  prefetch_offsets(set + W);

  // Main loop, double-buffered over items (set, chunk): the next item's loads are in flight
  // while the current one is computed.  The buffers alternate explicitly (a register copy
  // would make hipcc wait for every outstanding load at the loop head).
  Chains c{0u, 0u, 0u, 0u};
  int chunk = 0;
  const uint8_t* base_cur = p.bytes + d.start - d.pad + 16 * L.col;
  bool go_slow = false;  // the next set needs the slow path (tail of the batch)
  auto step = [&](uint4 (&cur)[JC], uint4 (&nxt)[JC]) -> bool {
    uint64_t set2 = set;
    int chunk2 = chunk + 1, nch2 = nch;
    FrameDesc d2 = d;
    const uint8_t* base2 = base_cur;
    const bool newset = (chunk2 == nch);
    bool more = true;
    if (newset) {
      set2 = set + W;
      chunk2 = 0;
      more = set2 < nsets;
      if (more) {
        d2 = desc_next(set2);
        nch2 = wave_nch(d2.J);
        prefetch_offsets(set2 + W);
        if (wave_slow(d2, nch2)) {
          go_slow = true;
          more = false;
        }
        base2 = p.bytes + d2.start - d2.pad + 16 * L.col;
      }
    }
    if (more) load_chunk<JC>(base2, chunk2, nxt);
    if (chunk == 0)
      compute_chunk<JC, FREEZE, true>(L, d, 0, cur, c);
    else {
      __builtin_assume(chunk >= 1);
      compute_chunk<JC, FREEZE, false>(L, d, chunk, cur, c);
    }
    if (newset) finish_set<SEAL>(L, p, set, d, c);
    if (go_slow) {  // hand the tail set over to the slow loop below
      set = set2;
      d = d2;
      nch = nch2;
      return false;
    }
    set = set2; chunk = chunk2; nch = nch2; d = d2; base_cur = base2;
    return more;
  };
  {
    uint4 A[JC], B[JC];
    load_chunk<JC>(base_cur, 0, A);
    while (step(A, B) && step(B, A)) {
    }
  }
  // Tail sets (last sets of the batch) through the slow path.
  if (go_slow) {
    for (; set < nsets; set += W) {
      d = desc_now(set);
      nch = wave_nch(d.J);
      slow_set<FREEZE, SEAL>(L, p, set, d, nch * JC);
    }
  }
}

#define UFC_INSTANTIATE(JC)                                                          \
  template __global__ void frame_crc_kernel<JC, 0>(const KernelParams);                 \
  template __global__ void frame_crc_kernel<JC, kModeSeal>(const KernelParams);         \
  template __global__ void frame_crc_kernel<JC, kModeVarlen>(const KernelParams);       \
  template __global__ void frame_crc_kernel<JC, kModeVarlen | kModeSeal>(const KernelParams); \
  template __global__ void frame_crc_kernel<JC, kModeFreeze>(const KernelParams);       \
  template __global__ void frame_crc_kernel<JC, kModeFreeze | kModeSeal>(const KernelParams);

UFC_INSTANTIATE(1)
UFC_INSTANTIATE(2)
UFC_INSTANTIATE(3)
UFC_INSTANTIATE(4)
UFC_INSTANTIATE(5)
UFC_INSTANTIATE(6)

const void* kernel_symbol(int jc, int mode) {
#define UFC_PICK(JC)                                                                                      \
  case JC:                                                                                                \
    switch (mode) {                                                                                       \
      case 0: return (const void*)frame_crc_kernel<JC, 0>;                                               \
      case kModeSeal: return (const void*)frame_crc_kernel<JC, kModeSeal>;                               \
      case kModeVarlen: return (const void*)frame_crc_kernel<JC, kModeVarlen>;                           \
      case kModeVarlen | kModeSeal: return (const void*)frame_crc_kernel<JC, kModeVarlen | kModeSeal>;   \
      case kModeFreeze: return (const void*)frame_crc_kernel<JC, kModeFreeze>;                           \
      case kModeFreeze | kModeSeal: return (const void*)frame_crc_kernel<JC, kModeFreeze | kModeSeal>;   \
      default: return nullptr;                                                                            \
    }
  switch (jc) {
    UFC_PICK(1)
    UFC_PICK(2)
    UFC_PICK(3)
    UFC_PICK(4)
    UFC_PICK(5)
    UFC_PICK(6)
    default:
      return nullptr;
  }
#undef UFC_PICK
}

}  // namespace ufc_dev
