// frame_parse.hip -- batched Frame::read after the batched CRC gate, on device-resident frames
// (on-GPU datagram header parse/validation).
//
// Three steps on the caller's stream, workgroups of 256 frames (one thread per frame):
//   1. walk:  gate + parse of frame_codec_core.hpp (restating src/frame/serial/mod.rs:54-434,
//             694-705) -> the frame's ufc_frame_info (item_first aside), its item count, a mode
//             byte and, for data frames, the frame offsets of its datagram headers: u16 slots in
//             LDS while the thread walks (no global store inside the dependent load chain), then
//             written compactly per workgroup.  Only the bytes the walk needs are read (each
//             datagram's first byte and its length bytes).
//   2. scan:  exclusive sum of the item counts (hipcub) -> each frame's first item.
//   3. emit:  item-parallel over the workgroup's item range: lane j finds its frame (binary search
//             over the firsts in LDS), loads the header bytes (independent 4-byte loads across
//             items), decodes the ufc_item (datagram with datagram_is_valid of
//             packet_receiver/mod.rs:12-30, or ack group) and stores it: consecutive lanes write
//             consecutive 24-byte records.  Frames whose headers did not fit the slots (more than
//             kPosSlots datagrams, or longer than 64 KiB) are walked again by their own thread,
//             storing directly.
// Round-1 shape (one thread walking and storing every item, 1.18 ms for 1M frames): every item
// store sat in the same vmcnt queue as the walk's next header load, and the stores of a wave
// scattered over 64 frames' item ranges.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstddef>

#include "frame_codec_core.hpp"
#include "frame_parse.hpp"

namespace ufc_dev {

namespace {

constexpr int kParseThreads = 256;
#ifndef UFC_POS_SLOTS
#define UFC_POS_SLOTS 64
#endif
constexpr uint32_t kPosSlots = UFC_POS_SLOTS;  // datagram headers recorded per frame (a data frame holds <= 127)
constexpr uint64_t kSegWords = (uint64_t)kPosSlots * kParseThreads;  // u16 per workgroup segment
enum : uint8_t { kItemsNone = 0, kItemsPos = 1, kItemsAck = 2, kItemsWalk = 3 };

typedef hipcub::BlockScan<uint32_t, kParseThreads> BlockScan;

struct DevBytes {
  const uint8_t* p;
  __device__ uint32_t operator()(uint32_t i) const {
    return *(const __attribute__((address_space(1))) uint8_t*)(p + i);
  }
};

// Walk sink: only the header offsets, into this thread's LDS slots (slot k at k * kParseThreads).
struct PosSink {
  static constexpr bool kDecode = false;
  uint16_t* slot;
  __device__ bool on() const { return true; }
  __device__ void operator()(uint32_t, const ufc_item&) const {}
  __device__ void header(uint32_t k, uint32_t off) const { slot[k * kParseThreads] = (uint16_t)off; }
};

// Items as three 8-byte stores each (ufc_item is 24 bytes, laid out as below).
static_assert(sizeof(ufc_item) == 24 && offsetof(ufc_item, channel_id) == 4 && offsetof(ufc_item, form) == 5 &&
                  offsetof(ufc_item, window_parent_lead) == 6 && offsetof(ufc_item, channel_parent_lead) == 8 &&
                  offsetof(ufc_item, fragment_id) == 10 && offsetof(ufc_item, fragment_id_last) == 12 &&
                  offsetof(ufc_item, flags) == 14 && offsetof(ufc_item, data_offset) == 16 &&
                  offsetof(ufc_item, data_len) == 20,
              "ufc_item layout");
__device__ __forceinline__ void store_item(ufc_item* p, const ufc_item& it) {
  typedef __attribute__((address_space(1))) uint64_t g_u64w;
  g_u64w* q = (g_u64w*)p;
  q[0] = (uint64_t)it.id | ((uint64_t)it.channel_id << 32) | ((uint64_t)it.form << 40) |
         ((uint64_t)it.window_parent_lead << 48);
  q[1] = (uint64_t)it.channel_parent_lead | ((uint64_t)it.fragment_id << 16) | ((uint64_t)it.fragment_id_last << 32) |
         ((uint64_t)it.flags << 48);
  q[2] = (uint64_t)it.data_offset | ((uint64_t)it.data_len << 32);
}
struct PackedSink {
  static constexpr bool kDecode = true;
  ufc_item* p;
  __device__ bool on() const { return p != nullptr; }
  __device__ void operator()(uint32_t k, const ufc_item& it) const { store_item(p + k, it); }
  __device__ void header(uint32_t, uint32_t) const {}
};

__device__ __forceinline__ uint32_t frame_len32(const uint64_t* offsets, uint64_t i, uint64_t& a) {
  a = offsets[i];
  const uint64_t b = offsets[i + 1];
  const uint64_t len64 = b >= a ? b - a : 0;
  return len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
}

__global__ __launch_bounds__(kParseThreads) void parse_walk_kernel(const uint8_t* bytes, const uint64_t* offsets,
                                                                   uint64_t n, const uint8_t* valid,
                                                                   ufc_frame_info* infos, uint32_t* counts,
                                                                   uint8_t* modes, uint16_t* pos_seg,
                                                                   uint32_t* seg_cursor, uint32_t* seg_base,
                                                                   uint64_t seg_cap) {
  __shared__ uint16_t slots[kSegWords];
  __shared__ typename BlockScan::TempStorage scan_tmp;
  __shared__ uint32_t base_lds;
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * kParseThreads + t;
  uint32_t npos = 0;
  uint8_t mode = kItemsNone;
  if (i < n) {
    uint64_t a;
    const uint32_t len = frame_len32(offsets, i, a);
    ufc_frame_info info;
    const bool ok = ufc_codec::read_frame_to(DevBytes{bytes + a}, len, valid[i] != 0, info, PosSink{slots + t},
                                             kPosSlots);
    const uint32_t cnt = ok ? info.item_count : 0u;
    if (cnt) {
      if (info.kind == UFC_FRAME_ACK) {
        mode = kItemsAck;
      } else if (cnt <= kPosSlots && len <= 0xFFFFu) {
        mode = kItemsPos;
        npos = cnt;
      } else {
        mode = kItemsWalk;
      }
    }
    info.item_first = 0;  // written by the emit step
    infos[i] = info;
    counts[i] = cnt;
  }
  uint32_t lo, total;
  BlockScan(scan_tmp).ExclusiveSum(npos, lo, total);
  // the workgroup's segment of header slots, from the launch's bump counter (no room: the emit
  // step re-walks this workgroup's frames instead)
  if (t == 0) {
    uint32_t b = total ? atomicAdd(seg_cursor, total) : 0u;
    if (total && (uint64_t)b + total > seg_cap) b = 0xFFFFFFFFu;
    base_lds = b;
    seg_base[blockIdx.x] = b;
  }
  __syncthreads();
  const uint32_t base = base_lds;
  if (i < n) modes[i] = (mode == kItemsPos && base == 0xFFFFFFFFu) ? (uint8_t)kItemsWalk : mode;
  if (base != 0xFFFFFFFFu) {  // (each thread reads back only the slots it wrote)
    uint16_t* seg = pos_seg + base;
    for (uint32_t k = 0; k < npos; k++) seg[lo + k] = slots[k * kParseThreads + t];
  }
}

__global__ __launch_bounds__(kParseThreads) void parse_emit_kernel(
    const uint8_t* bytes, const uint64_t* offsets, uint64_t n, const uint8_t* valid, ufc_frame_info* infos,
    const uint32_t* counts, const uint32_t* firsts, const uint8_t* modes, const uint16_t* pos_seg,
    const uint32_t* seg_base, ufc_item* items, uint64_t cap, uint64_t* items_used) {
  __shared__ uint32_t lfirst[kParseThreads], lseg[kParseThreads];
  __shared__ uint64_t lstart[kParseThreads];
  __shared__ uint8_t lmode[kParseThreads];
  __shared__ uint32_t lend;
  __shared__ typename BlockScan::TempStorage scan_tmp;
  const uint32_t t = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * kParseThreads, i = i0 + t;
  const uint32_t nb = (uint32_t)min((uint64_t)kParseThreads, n - i0);  // frames of this workgroup
  uint32_t first = 0, cnt = 0;
  uint8_t mode = kItemsNone;
  uint64_t a = 0;
  if (i < n) {
    first = firsts[i];
    cnt = counts[i];
    mode = modes[i];
    a = offsets[i];
    infos[i].item_first = first;
    if (i == n - 1 && items_used) *items_used = (uint64_t)first + cnt;
  }
  uint32_t lo;
  BlockScan(scan_tmp).ExclusiveSum(mode == kItemsPos ? cnt : 0u, lo);
  lfirst[t] = first;
  lseg[t] = lo;
  lstart[t] = a;
  lmode[t] = mode;
  if (t == nb - 1) lend = first + cnt;
  __syncthreads();

  // Header bytes through a buffer resource over the workgroup's bytes (4-byte aligned base, range
  // rounded up to whole dwords: a dword holding a frame byte never leaves that byte's page); five
  // dword loads cover 16 bytes from any offset.  Spans of 4 GiB and more take byte loads.
  const uint64_t span_lo = lstart[0];
  const uint64_t span_hi = offsets[i0 + nb];
  const uintptr_t base_addr = (uintptr_t)(bytes + span_lo);
  const uint32_t delta = (uint32_t)(base_addr & 3u);
  const uint64_t range = (span_hi - span_lo + delta + 3) & ~(uint64_t)3;
  const bool buf_ok = span_hi >= span_lo && range < 0xFFFFFFF0ull;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(base_addr - delta), 0, buf_ok ? (int)(uint32_t)range : 0, 0x00020000);

  const uint32_t g0 = lfirst[0], g1 = lend;
  const uint32_t sb = seg_base[blockIdx.x];  // (0xFFFFFFFF: no segment, and no kItemsPos frame either)
  const uint16_t* seg = pos_seg + (sb == 0xFFFFFFFFu ? 0u : sb);
  if (items) {
    for (uint32_t g = g0 + t; g < g1 && (uint64_t)g < cap; g += kParseThreads) {
      uint32_t lo_f = 0, hi_f = nb - 1;  // owner: the last frame whose first item is <= g
      while (lo_f < hi_f) {
        const uint32_t mid = (lo_f + hi_f + 1) >> 1;
        if (lfirst[mid] <= g)
          lo_f = mid;
        else
          hi_f = mid - 1;
      }
      const uint32_t f = lo_f, k = g - lfirst[f];
      const uint8_t m = lmode[f];
      if (m != kItemsPos && m != kItemsAck) continue;
      const uint32_t hoff = m == kItemsPos ? (uint32_t)seg[lseg[f] + k]
                                           : 1u + ufc_codec::kAckPayloadHeader + UFC_ACK_GROUP_SIZE * k;
      uint32_t w[4];
      if (buf_ok) {
        const uint32_t rel = (uint32_t)(lstart[f] - span_lo) + delta + hoff;
        const uint32_t al = rel & ~3u, sh = rel & 3u;
        uint32_t x[5];
#pragma unroll
        for (int q = 0; q < 5; q++) x[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(al + 4 * q), 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) w[q] = __builtin_amdgcn_alignbyte(x[q + 1], x[q], sh);
      } else {
        const DevBytes rd{bytes + lstart[f] + hoff};
#pragma unroll
        for (int q = 0; q < 4; q++) w[q] = 0;
        // (only the bytes the header occupies: a datagram's hs <= 14, an ack group 9)
        const uint32_t nbytes = m == kItemsAck ? UFC_ACK_GROUP_SIZE : 14u;
        for (uint32_t c = 0; c < nbytes; c++) w[c >> 2] |= rd(c) << (8 * (c & 3));
      }
      auto h = [&](uint32_t c) -> uint32_t { return (w[c >> 2] >> (8 * (c & 3))) & 0xFFu; };
      ufc_item it{};
      if (m == kItemsPos) {
        uint32_t hs, dl;
        ufc_codec::datagram_size(h, hs, dl);
        ufc_codec::decode_datagram(h, hs, it);
        it.data_offset = hoff + hs;
      } else {
        ufc_codec::decode_ack_group(h, it);
      }
      store_item(items + g, it);
    }
    // Frames whose headers did not fit the slots: walked again, items stored directly.
    if (mode == kItemsWalk && (uint64_t)first < cap) {
      uint64_t aa;
      const uint32_t len = frame_len32(offsets, i, aa);
      const uint32_t room = (uint32_t)min((uint64_t)cnt, cap - first);
      ufc_frame_info info;
      ufc_codec::read_frame_to(DevBytes{bytes + aa}, len, valid[i] != 0, info, PackedSink{items + first}, room);
    }
  }
}

// =============================================================================================
// One-pass parse (the default): tiles of kFuseFrames consecutive frames, claimed in order from a
// ticket counter by workgroups of 256 threads (three per CU).  Per tile:
//   1. stage: the tile's bytes [offsets[f0], offsets[f0 + T]) are copied into LDS with coalesced
//      16-byte loads, up to kFuseData bytes (a frame not wholly inside the staged window is read
//      from global memory instead, byte by byte, as the three-pass walk does);
//   2. walk: one thread per frame runs the same read_frame_to as the host codec over the staged
//      bytes (LDS latency instead of an HBM round trip per datagram), recording each datagram
//      header's frame offset in LDS slots;
//   3. scan + decoupled look-back: the tile's item count is published (flag 1) at once, the global
//      first item found by walking back over the predecessors' published counts / prefixes, and
//      the tile's inclusive prefix published (flag 2); tiles are claimed in order, so every
//      predecessor belongs to a running workgroup;
//   4. emit: item-parallel over the tile, headers decoded from LDS, 24-byte records stored
//      consecutively; infos written once with item_first.  Frames with more than kPosSlots
//      datagrams or over 64 KiB are walked again from global memory by their own thread.
// Every byte of the batch is read once, coalesced, instead of the three-pass shape's two
// dependent-load walks over ~every line (walk + emit: 1.3 GB of scattered reads for 1.41 GB).
constexpr int kFuseThreads = 256;
constexpr int kFuseFrames = 32;              // frames per tile
constexpr uint32_t kFuseData = 46u * 1024u;  // staged bytes per tile (uflow frames: <= 1472 B)
constexpr uint32_t kFuseSpin = 1u << 22;     // look-back wait bound (s_sleep steps; never reached)
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kFlagMask = 3ull << 62;

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(3))) uint8_t l_u8;
typedef const __attribute__((address_space(3))) uint32_t l_u32;

struct LdsBytes {
  l_u8* p;
  __device__ uint32_t operator()(uint32_t i) const { return p[i]; }
};

// Walk sink: header offsets into LDS slots (slot k of tile frame f at k * kFuseFrames + f).
struct TilePosSink {
  static constexpr bool kDecode = false;
  uint16_t* slot;
  __device__ bool on() const { return true; }
  __device__ void operator()(uint32_t, const ufc_item&) const {}
  __device__ void header(uint32_t k, uint32_t off) const { slot[k * kFuseFrames] = (uint16_t)off; }
};

struct FuseLds {
  uint4 data[kFuseData / 16];
  uint16_t slots[kPosSlots * kFuseFrames];
  uint64_t off[kFuseFrames + 1];
  uint32_t first[kFuseFrames];
  uint8_t mode[kFuseFrames];
  uint8_t inlds[kFuseFrames];
  uint32_t tile;
  uint32_t agg;
  uint64_t excl;
};
static_assert(sizeof(FuseLds) * 3 <= 160 * 1024, "three workgroups per CU");

__global__ __launch_bounds__(kFuseThreads) void parse_fused_kernel(const uint8_t* bytes, const uint64_t* offsets,
                                                                   uint64_t n, const uint8_t* valid,
                                                                   ufc_frame_info* infos, ufc_item* items,
                                                                   uint64_t cap, uint64_t* items_used,
                                                                   uint32_t* ticket, uint64_t* state,
                                                                   uint32_t* err) {
  __shared__ FuseLds L;
  const uint32_t t = threadIdx.x;
  const uint64_t ntiles = (n + kFuseFrames - 1) / kFuseFrames;
  l_u8* const dl = (l_u8*)(const uint8_t*)L.data;
  for (;;) {
    if (t == 0) L.tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = L.tile;
    if ((uint64_t)tile >= ntiles) break;
    const uint64_t f0 = (uint64_t)tile * kFuseFrames;
    const uint32_t nb = (uint32_t)min((uint64_t)kFuseFrames, n - f0);
    if (t <= nb) L.off[t] = offsets[f0 + t];
    __syncthreads();

    // ---- 1. stage the tile's bytes (16-byte chunks from the aligned chunk of its first byte) ----
    const uint64_t a0 = L.off[0], an = L.off[nb];
    const uintptr_t s_addr = (uintptr_t)(bytes + a0);
    const uint32_t delta = (uint32_t)(s_addr & 15u);
    const uint64_t span = an >= a0 ? an - a0 : 0;
    const uint32_t staged = (uint32_t)min(span + delta, (uint64_t)kFuseData);  // bytes held, from the chunk start
    {  // every load issued before the first LDS write (chunks past the staged bytes: out of range, no request)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(s_addr - delta), 0, (int)staged, 0x00020000);
      const uint32_t nch = (staged + 15u) >> 4;
      constexpr int kPer = (kFuseData / 16 + kFuseThreads - 1) / kFuseThreads;
      u32x4v v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const uint32_t i = t + kFuseThreads * k;
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i < nch ? 16u * i : 0x80000000u), 0, 2);
      }
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const uint32_t i = t + kFuseThreads * k;
        if (i < nch) L.data[i] = make_uint4(v[k].x, v[k].y, v[k].z, v[k].w);
      }
    }
    __syncthreads();

    // ---- 2. walk: one thread per frame ----
    uint32_t cnt = 0;
    uint8_t mode = kItemsNone;
    ufc_frame_info info{};
    if (t < nb) {
      const uint64_t a = L.off[t], b = L.off[t + 1];
      const uint64_t len64 = b >= a ? b - a : 0;
      const uint32_t len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
      const uint64_t rel = a - a0 + delta;
      const bool in = a >= a0 && rel + len64 <= staged;
      const bool crc_ok = valid[f0 + t] != 0;
      const bool ok = in ? ufc_codec::read_frame_to(LdsBytes{dl + (uint32_t)rel}, len, crc_ok, info,
                                                    TilePosSink{L.slots + t}, kPosSlots)
                         : ufc_codec::read_frame_to(DevBytes{bytes + a}, len, crc_ok, info, TilePosSink{L.slots + t},
                                                    kPosSlots);
      cnt = ok ? info.item_count : 0u;
      if (cnt) {
        if (info.kind == UFC_FRAME_ACK)
          mode = kItemsAck;
        else if (cnt <= kPosSlots && len <= 0xFFFFu)
          mode = kItemsPos;
        else
          mode = kItemsWalk;
      }
      L.mode[t] = mode;
      L.inlds[t] = in ? 1 : 0;
    }

    // ---- 3. the tile's item scan (wave 0) and the decoupled look-back (thread 0) ----
    if (t < 64) {
      uint32_t x = t < nb ? cnt : 0u;
#pragma unroll
      for (int d = 1; d < kFuseFrames; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if ((int)(t & 63u) >= d) x += y;
      }
      if (t < kFuseFrames) L.first[t] = x - (t < nb ? cnt : 0u);  // exclusive
      if (t == kFuseFrames - 1) {
        const uint32_t agg = x;
        L.agg = agg;
        uint64_t excl = 0;
        if (tile == 0) {
          __hip_atomic_store(state + tile, kFlagIncl | (uint64_t)agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          __hip_atomic_store(state + tile, kFlagAgg | (uint64_t)agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          uint64_t j = tile;
          uint32_t spins = 0;
          while (j > 0) {
            const uint64_t s = __hip_atomic_load(state + j - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t fl = s & kFlagMask;
            if (fl == 0) {
              if (++spins > kFuseSpin) {  // (a predecessor that never publishes: flag it, do not hang)
                atomicOr(err, 1u);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
              continue;
            }
            excl += s & ~kFlagMask;
            if (fl == kFlagIncl) break;
            j--;
          }
          __hip_atomic_store(state + tile, kFlagIncl | (excl + agg), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        L.excl = excl;
        if (f0 + nb == n && items_used) *items_used = excl + agg;
      }
    }
    __syncthreads();
    const uint64_t excl = L.excl;
    const uint32_t agg = L.agg;
    if (t < nb) {
      info.item_first = (uint32_t)(excl + L.first[t]);
      infos[f0 + t] = info;
    }

    // ---- 4. emit ----
    if (items) {
      for (uint32_t q = t; q < agg && excl + q < cap; q += kFuseThreads) {
        uint32_t lo = 0, hi = nb - 1;  // owner: the last frame whose first item is <= q
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (L.first[mid] <= q)
            lo = mid;
          else
            hi = mid - 1;
        }
        const uint32_t f = lo, k = q - L.first[f];
        const uint8_t m = L.mode[f];
        if (m != kItemsPos && m != kItemsAck) continue;
        const uint32_t hoff = m == kItemsPos ? (uint32_t)L.slots[k * kFuseFrames + f]
                                             : 1u + ufc_codec::kAckPayloadHeader + UFC_ACK_GROUP_SIZE * k;
        uint32_t w[4];
        if (L.inlds[f]) {  // the header's 14 bytes from LDS: five aligned words, realigned
          const uint32_t p = (uint32_t)(L.off[f] - a0) + delta + hoff;
          const uint32_t al = p & ~3u, sh = p & 3u;
          uint32_t x[5];
#pragma unroll
          for (int i = 0; i < 5; i++) x[i] = (al + 4u * i < kFuseData) ? *(l_u32*)(dl + al + 4u * i) : 0u;
#pragma unroll
          for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], sh);
        } else {
          const DevBytes rd{bytes + L.off[f] + hoff};
#pragma unroll
          for (int i = 0; i < 4; i++) w[i] = 0;
          const uint32_t nbytes = m == kItemsAck ? UFC_ACK_GROUP_SIZE : 14u;
          for (uint32_t c = 0; c < nbytes; c++) w[c >> 2] |= rd(c) << (8 * (c & 3));
        }
        auto h = [&](uint32_t c) -> uint32_t { return (w[c >> 2] >> (8 * (c & 3))) & 0xFFu; };
        ufc_item it{};
        if (m == kItemsPos) {
          uint32_t hs, dlen;
          ufc_codec::datagram_size(h, hs, dlen);
          ufc_codec::decode_datagram(h, hs, it);
          it.data_offset = hoff + hs;
        } else {
          ufc_codec::decode_ack_group(h, it);
        }
        store_item(items + excl + q, it);
      }
      // frames whose headers did not fit the slots: walked again, items stored directly
      if (t < nb && mode == kItemsWalk && excl + L.first[t] < cap) {
        const uint64_t g0 = excl + L.first[t];
        const uint64_t a = L.off[t], b = L.off[t + 1];
        const uint32_t len = (uint32_t)min(b - a, (uint64_t)0xFFFFFFFFu);
        const uint32_t room = (uint32_t)min((uint64_t)cnt, cap - g0);
        ufc_frame_info again;
        ufc_codec::read_frame_to(DevBytes{bytes + a}, len, valid[f0 + t] != 0, again, PackedSink{items + g0}, room);
      }
    }
    __syncthreads();  // (LDS reused by the next tile)
  }
}

}  // namespace

namespace {
struct ParseLayout {  // the scratch of a parse of n frames (256-byte aligned parts)
  uint64_t counts, firsts, modes, cursor, bases, slots, temp, end, seg_cap;
  ParseLayout(uint64_t n, uint64_t items_cap, size_t temp_bytes) {
    auto up = [](uint64_t b) { return (b + 255) / 256 * 256; };
    const uint64_t blocks = (n + kParseThreads - 1) / kParseThreads;
    seg_cap = std::min<uint64_t>(n * kPosSlots, std::max<uint64_t>(items_cap, 1));  // u16 header slots
    counts = 0;
    firsts = counts + up(n * 4);
    modes = firsts + up(n * 4);
    cursor = modes + up(n);
    bases = cursor + 256;
    slots = bases + up(blocks * 4);
    temp = slots + up(seg_cap * 2);
    end = temp + up(temp_bytes);
  }
};
size_t scan_temp_bytes(uint64_t n) {
  size_t temp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return temp;
}
}  // namespace

// One-pass parse scratch: ticket and error words, then one look-back word per tile.
static uint64_t fused_scratch(uint64_t n) { return 256 + (n + kFuseFrames - 1) / kFuseFrames * 8; }

size_t parse_scratch_bytes(uint64_t n, uint64_t items_cap) {
  return std::max<uint64_t>(ParseLayout(n, items_cap, scan_temp_bytes(n)).end, fused_scratch(n));
}

hipError_t parse_batch(const ParseArgs& a, void* scratch, size_t scratch_bytes, hipStream_t stream) {
  const uint64_t n = a.n;
  if (a.kernel == kParseFused) {
    const uint64_t need = fused_scratch(n);
    if (need > scratch_bytes) return hipErrorInvalidValue;
    uint32_t* ticket = (uint32_t*)scratch;
    uint32_t* err = ticket + 1;
    uint64_t* state = (uint64_t*)((char*)scratch + 256);
    hipError_t e = hipMemsetAsync(scratch, 0, need, stream);
    if (e != hipSuccess) return e;
    const uint64_t ntiles = (n + kFuseFrames - 1) / kFuseFrames;
    const uint64_t grid = std::min<uint64_t>(ntiles, (uint64_t)std::max(1, a.ncu) * 3);
    parse_fused_kernel<<<(unsigned)grid, kFuseThreads, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, a.items,
                                                                   a.items_cap, a.items_used, ticket, state, err);
    return hipGetLastError();
  }
  const uint64_t blocks = (n + kParseThreads - 1) / kParseThreads;
  const ParseLayout lay(n, a.items_cap, scan_temp_bytes(n));
  if (lay.end > scratch_bytes) return hipErrorInvalidValue;
  char* s = (char*)scratch;
  uint32_t* counts = (uint32_t*)(s + lay.counts);
  uint32_t* firsts = (uint32_t*)(s + lay.firsts);
  uint8_t* modes = (uint8_t*)(s + lay.modes);
  uint32_t* cursor = (uint32_t*)(s + lay.cursor);
  uint32_t* bases = (uint32_t*)(s + lay.bases);
  uint16_t* pos_seg = (uint16_t*)(s + lay.slots);
  void* temp = s + lay.temp;
  size_t temp_bytes = lay.end - lay.temp;
  hipError_t e = hipMemsetAsync(cursor, 0, 4, stream);
  if (e != hipSuccess) return e;
  parse_walk_kernel<<<(unsigned)blocks, kParseThreads, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, counts,
                                                                    modes, pos_seg, cursor, bases, lay.seg_cap);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, firsts, (int)n, stream);
  if (e != hipSuccess) return e;
  parse_emit_kernel<<<(unsigned)blocks, kParseThreads, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, counts,
                                                                    firsts, modes, pos_seg, bases, a.items, a.items_cap,
                                                                    a.items_used);
  return hipGetLastError();
}

}  // namespace ufc_dev
