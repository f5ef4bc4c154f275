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
//   2. scan:  exclusive sum of the workgroups' item counts (hipcub) -> each workgroup's first item
//             (the emit adds the counts of the frames before a frame within its workgroup).
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
#include <cstdlib>

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

// Two per-frame counts scanned at once (each workgroup sum < 2^32: 256 frames x < 2^24), low and high halves.
typedef hipcub::BlockScan<uint64_t, kParseThreads> BlockScan2;

// Byte-aligned global views: the IR carries align 1, so the compiler never assumes 4- or 8-byte
// alignment when it combines or splits these loads; gfx950's unaligned access mode still makes each
// one a single global_load_dword / dwordx2.
typedef const __attribute__((address_space(1), aligned(1))) uint32_t g_u32_a1;
typedef const __attribute__((address_space(1), aligned(1))) uint64_t g_u64_a1;

struct DevBytes {
  const uint8_t* p;
  __device__ uint32_t operator()(uint32_t i) const {
    return *(const __attribute__((address_space(1))) uint8_t*)(p + i);
  }
  // one dword load at any byte address (gfx950's unaligned access mode; the codec guarantees the
  // four bytes lie inside the frame): one round trip and one address pass for a datagram's sizes
  __device__ uint32_t head3(uint32_t i) const {
    return *(g_u32_a1*)(p + i) & 0xFFFFFFu;
  }
};

// The walk's reader: the frame's first 8 bytes come from one load issued with the frame's other
// first reads (kind and the data header's fields), the rest as DevBytes.  (Round 4's 16-byte head,
// which also held the first datagram's size bytes, failed at random -- one data frame per ~200k, a
// different one each run -- and is gone: ADVICE r4, profiles/EXPERIMENTS.md "walk head" for the
// ISA comparison.)  head_byte keeps every shift amount in range.
struct DevBytesHead {
  const uint8_t* p;
  uint64_t w0;    // bytes 0..7, little-endian
  uint32_t held;  // bytes 0 .. held-1 in w0: 8 or 0
  __device__ static DevBytesHead load(const uint8_t* q, uint32_t len) {  // (any byte address: unaligned access mode)
    DevBytesHead r{q, 0ull, 0u};
    if (len >= 8) {
      r.w0 = *(g_u64_a1*)q;
      r.held = 8;
    }
    return r;
  }
  __device__ uint32_t held_byte(uint32_t i) const { return head_byte(w0, 0ull, i); }
  __device__ uint32_t operator()(uint32_t i) const {
    if (i < held) return held_byte(i);
    return *(const __attribute__((address_space(1))) uint8_t*)(p + i);
  }
  __device__ uint32_t head3(uint32_t i) const {
    if (i + 3 <= held) return held_byte(i) | (held_byte(i + 1) << 8) | (held_byte(i + 2) << 16);
    return *(g_u32_a1*)(p + i) & 0xFFFFFFu;
  }
};

// Items as three 8-byte stores each (ufc_item is 24 bytes, laid out as below).
static_assert(sizeof(ufc_item) == 24 && offsetof(ufc_item, channel_id) == 4 && offsetof(ufc_item, form) == 5 &&
                  offsetof(ufc_item, window_parent_lead) == 6 && offsetof(ufc_item, channel_parent_lead) == 8 &&
                  offsetof(ufc_item, fragment_id) == 10 && offsetof(ufc_item, fragment_id_last) == 12 &&
                  offsetof(ufc_item, flags) == 14 && offsetof(ufc_item, data_offset) == 16 &&
                  offsetof(ufc_item, data_len) == 20,
              "ufc_item layout");
template <bool NT = false>  // NT: non-temporal stores
__device__ __forceinline__ void store_item(ufc_item* p, const ufc_item& it) {
  typedef __attribute__((address_space(1))) uint64_t g_u64w;
  g_u64w* q = (g_u64w*)p;
  const uint64_t w0 = (uint64_t)it.id | ((uint64_t)it.channel_id << 32) | ((uint64_t)it.form << 40) |
                      ((uint64_t)it.window_parent_lead << 48);
  const uint64_t w1 = (uint64_t)it.channel_parent_lead | ((uint64_t)it.fragment_id << 16) |
                      ((uint64_t)it.fragment_id_last << 32) | ((uint64_t)it.flags << 48);
  const uint64_t w2 = (uint64_t)it.data_offset | ((uint64_t)it.data_len << 32);
  if constexpr (NT) {
    __builtin_nontemporal_store(w0, q);
    __builtin_nontemporal_store(w1, q + 1);
    __builtin_nontemporal_store(w2, q + 2);
  } else {
    q[0] = w0;
    q[1] = w1;
    q[2] = w2;
  }
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

// The walk with pooled header slots (round 3): kInlineSlots slots per frame in LDS, and the headers
// past them in a per-workgroup pool of linked LDS entries (offset | next << 16) taken one at a time
// with ds_add_rtn.  A frame averages ~15 datagrams, so 16 + a shared pool hold what 64 fixed slots per
// frame held, in a third of the LDS: more workgroups per CU and more frames walking at once (the walk
// is a dependent load chain per frame, bound by how many chains are in flight).  A frame that finds
// the pool full is walked again by the emit step, as one with more than kPosSlots datagrams.
constexpr uint32_t kInlineSlots = 16;
constexpr uint32_t kPoolSlots = 2048;
constexpr uint32_t kPoolNil = 0xFFFFu;

struct PoolSink {
  static constexpr bool kDecode = false;
  uint16_t* slot;     // this thread's inline slots (slot k at k * kParseThreads)
  uint32_t* pool;     // the workgroup's pool
  uint32_t* ctr;      // its allocation counter
  uint32_t* head;     // this thread's list (registers, through pointers: the sink is const)
  uint32_t* tail;
  bool* full;
  __device__ bool on() const { return true; }
  __device__ void operator()(uint32_t, const ufc_item&) const {}
  __device__ void header(uint32_t k, uint32_t off) const {
    if (k < kInlineSlots) {
      slot[k * kParseThreads] = (uint16_t)off;
      return;
    }
    if (*full) return;
    const uint32_t idx = atomicAdd(ctr, 1u);  // (LDS atomic)
    if (idx >= kPoolSlots) {
      *full = true;
      return;
    }
    pool[idx] = off | (kPoolNil << 16);
    if (k == kInlineSlots)
      *head = idx;
    else
      pool[*tail] = (pool[*tail] & 0xFFFFu) | (idx << 16);
    *tail = idx;
  }
};

__global__ __launch_bounds__(kParseThreads) void parse_walk_pool_kernel(const uint8_t* bytes, const uint64_t* offsets,
                                                                        uint64_t n, const uint8_t* valid,
                                                                        ufc_frame_info* infos, uint32_t* counts,
                                                                        uint8_t* modes, uint16_t* pos_seg,
                                                                        unsigned long long* seg_cursor, uint32_t* seg_base,
                                                                        uint64_t seg_cap, uint32_t* wg_counts) {
  __shared__ uint16_t slots[kInlineSlots * kParseThreads];
  __shared__ uint32_t pool[kPoolSlots];
  __shared__ typename BlockScan2::TempStorage scan_tmp;
  __shared__ uint32_t base_lds, pool_ctr;
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * kParseThreads + t;
  if (t == 0) pool_ctr = 0;
  __syncthreads();
  uint32_t npos = 0, head = kPoolNil, tail = kPoolNil;
  bool full = false;
  uint8_t mode = kItemsNone;
  uint32_t cnt_all = 0;
  if (i < n) {
    uint64_t a;
    const uint32_t len = frame_len32(offsets, i, a);
    ufc_frame_info info;
    const DevBytesHead rd = DevBytesHead::load(bytes + a, len);
    const bool ok = ufc_codec::read_frame_to(rd, len, valid[i] != 0, info,
                                             PoolSink{slots + t, pool, &pool_ctr, &head, &tail, &full}, kPosSlots);
    const uint32_t cnt = ok ? info.item_count : 0u;
    if (cnt) {
      if (info.kind == UFC_FRAME_ACK) {
        mode = kItemsAck;
      } else if (cnt <= kPosSlots && len <= 0xFFFFu && !full) {
        mode = kItemsPos;
        npos = cnt;
      } else {
        mode = kItemsWalk;
      }
    }
    info.item_first = 0;  // written by the emit step
    infos[i] = info;
    counts[i] = cnt;
    cnt_all = cnt;
  }
  // header slots (low half) and items (high half) of the workgroup's frames, one scan
  uint64_t lo2, total2;
  BlockScan2(scan_tmp).ExclusiveSum((uint64_t)npos | ((uint64_t)cnt_all << 32), lo2, total2);
  const uint32_t lo = (uint32_t)lo2, total = (uint32_t)total2;
  if (t == 0) wg_counts[blockIdx.x] = (uint32_t)(total2 >> 32);  // (scanned over the workgroups next)
  if (t == 0) {
    // (64-bit cursor: the sum of every workgroup's total may pass 2^32 long after the cap is reached)
    const unsigned long long b64 = total ? atomicAdd(seg_cursor, (unsigned long long)total) : 0ull;
    const uint32_t b = (total && b64 + total > seg_cap) ? 0xFFFFFFFFu : (uint32_t)b64;
    base_lds = b;
    seg_base[blockIdx.x] = b;
  }
  __syncthreads();
  const uint32_t base = base_lds;
  if (i < n) modes[i] = (mode == kItemsPos && base == 0xFFFFFFFFu) ? (uint8_t)kItemsWalk : mode;
  if (base != 0xFFFFFFFFu) {  // (each thread reads back only the slots and list it wrote)
    uint16_t* seg = pos_seg + base;
    const uint32_t ni = min(npos, kInlineSlots);
    for (uint32_t k = 0; k < ni; k++) seg[lo + k] = slots[k * kParseThreads + t];
    uint32_t idx = head;
    for (uint32_t k = kInlineSlots; k < npos; k++) {
      const uint32_t v = pool[idx];
      seg[lo + k] = (uint16_t)(v & 0xFFFFu);
      idx = v >> 16;
    }
  }
}

// The emit's header loads leave nothing behind for later (each line is read once, by neighbouring lanes
// of one instruction): non-temporal (buffer-load aux 2; the walk's loads stay default, measured slower).
constexpr int kEmitAux = 2;
template <int U, int X4, int AUX = 0, bool NTS = false>
__global__ __launch_bounds__(kParseThreads) void parse_emit_kernel(
    const uint8_t* bytes, const uint64_t* offsets, uint64_t n, const uint8_t* valid, ufc_frame_info* infos,
    const uint32_t* counts, const uint32_t* wg_firsts, const uint8_t* modes, const uint16_t* pos_seg,
    const uint32_t* seg_base, ufc_item* items, uint64_t cap, uint64_t* items_used) {
  __shared__ uint32_t lfirst[kParseThreads], lseg[kParseThreads];
  __shared__ uint64_t lstart[kParseThreads];
  __shared__ uint8_t lmode[kParseThreads];
  __shared__ uint32_t lend;
  __shared__ typename BlockScan2::TempStorage scan_tmp;
  const uint32_t t = threadIdx.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * kParseThreads, i = i0 + t;
  const uint32_t nb = (uint32_t)min((uint64_t)kParseThreads, n - i0);  // frames of this workgroup
  uint32_t cnt = 0;
  uint8_t mode = kItemsNone;
  uint64_t a = 0;
  if (i < n) {
    cnt = counts[i];
    mode = modes[i];
    a = offsets[i];
  }
  // each frame's first item (the workgroup's first from the scan over workgroups + the items of the
  // frames before it here) and its header slots' offset in the workgroup's segment, one scan
  uint64_t lo2;
  BlockScan2(scan_tmp).ExclusiveSum((uint64_t)(mode == kItemsPos ? cnt : 0u) | ((uint64_t)cnt << 32), lo2);
  const uint32_t lo = (uint32_t)lo2;
  const uint32_t first = wg_firsts[blockIdx.x] + (uint32_t)(lo2 >> 32);
  if (i < n) {
    infos[i].item_first = first;
    if (i == n - 1 && items_used) *items_used = (uint64_t)first + cnt;
  }
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
    // U items per thread per round (items g, g + 256, ...): every header load of the round is issued
    // before the first decode and store.  X4 = 2: one unaligned 16-byte load at the header itself
    // when all 16 bytes lie inside the workgroup's range (a header at the very end of the span takes
    // the X4 = 1 pair, so no header byte depends on how a straddling load is range-checked); X4 = 1:
    // an aligned 16-byte load + one dword; X4 = 0: five dwords.
    const uint64_t g_end = min((uint64_t)g1, cap);
    for (uint64_t gb = (uint64_t)g0 + t; gb < g_end; gb += (uint64_t)U * kParseThreads) {
      uint32_t hoff[U], fo[U], x[U][5];
      uint8_t mm[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t g = gb + (uint64_t)u * kParseThreads;
        mm[u] = kItemsNone;
        hoff[u] = fo[u] = 0;
        if (g < g_end) {
          uint32_t lo_f = 0, hi_f = nb - 1;  // owner: the last frame whose first item is <= g
          while (lo_f < hi_f) {
            const uint32_t mid = (lo_f + hi_f + 1) >> 1;
            if (lfirst[mid] <= (uint32_t)g)
              lo_f = mid;
            else
              hi_f = mid - 1;
          }
          const uint32_t f = lo_f, k = (uint32_t)g - lfirst[f];
          const uint8_t m = lmode[f];
          if (m == kItemsPos || m == kItemsAck) {
            mm[u] = m;
            fo[u] = f;
            hoff[u] = m == kItemsPos ? (uint32_t)seg[lseg[f] + k]
                                     : 1u + ufc_codec::kAckPayloadHeader + UFC_ACK_GROUP_SIZE * k;
          }
        }
      }
      if (buf_ok) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          if (mm[u] == kItemsNone) continue;
          const uint32_t ex = (uint32_t)(lstart[fo[u]] - span_lo) + delta + hoff[u];
          const uint32_t al = ex & ~3u;
          if (X4 == 2 && ex + 16 <= (uint32_t)range) {  // one unaligned 16-byte load at the header
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)ex, 0, AUX);
            x[u][0] = v.x, x[u][1] = v.y, x[u][2] = v.z, x[u][3] = v.w;
            x[u][4] = 0;
          } else if constexpr (X4 >= 1) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)al, 0, 0);
            x[u][0] = v.x, x[u][1] = v.y, x[u][2] = v.z, x[u][3] = v.w;
            x[u][4] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(al + 16), 0, 0);
          } else {
#pragma unroll
            for (int q = 0; q < 5; q++) x[u][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(al + 4 * q), 0, 0);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint8_t m = mm[u];
        if (m == kItemsNone) continue;
        const uint32_t f = fo[u];
        uint32_t w[4];
        if (buf_ok) {
          const uint32_t ex = (uint32_t)(lstart[f] - span_lo) + delta + hoff[u];
          const uint32_t sh = (X4 == 2 && ex + 16 <= (uint32_t)range) ? 0u : ex & 3u;
#pragma unroll
          for (int q = 0; q < 4; q++) w[q] = __builtin_amdgcn_alignbyte(x[u][q + 1], x[u][q], sh);
        } else {
          const DevBytes rd{bytes + lstart[f] + hoff[u]};
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
          it.data_offset = hoff[u] + hs;
        } else {
          ufc_codec::decode_ack_group(h, it);
        }
        store_item<NTS>(items + gb + (uint64_t)u * kParseThreads, it);
      }
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

}  // namespace

namespace {
struct ParseLayout {  // the scratch of a parse of n frames (256-byte aligned parts)
  uint64_t counts, wg_counts, wg_firsts, modes, cursor, bases, slots, temp, end, seg_cap;
  ParseLayout(uint64_t n, uint64_t items_cap, size_t temp_bytes) {
    auto up = [](uint64_t b) { return (b + 255) / 256 * 256; };
    const uint64_t blocks = (n + kParseThreads - 1) / kParseThreads;
    // u16 header slots; below 2^32 - 1 so that every segment fits 32-bit offsets and no segment base
    // can equal the overflow sentinel 0xFFFFFFFF (frames past the cap are walked again, kItemsWalk)
    seg_cap = std::min<uint64_t>(std::min<uint64_t>(n * kPosSlots, std::max<uint64_t>(items_cap, 1)),
                                 0xFFFFFFFEull - kSegWords);
    counts = 0;
    wg_counts = counts + up(n * 4);  // items per workgroup of 256 frames, then their exclusive sum
    wg_firsts = wg_counts + up(blocks * 4);
    modes = wg_firsts + up(blocks * 4);
    cursor = modes + up(n);
    bases = cursor + 256;
    slots = bases + up(blocks * 4);
    temp = slots + up(seg_cap * 2);
    end = temp + up(temp_bytes);
  }
};
size_t scan_temp_bytes(uint64_t n) {  // the scan over the workgroups' item counts
  const uint64_t blocks = (n + kParseThreads - 1) / kParseThreads;
  size_t temp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)blocks);
  return temp;
}
}  // namespace

size_t parse_scratch_bytes(uint64_t n, uint64_t items_cap) {
  return ParseLayout(n, items_cap, scan_temp_bytes(n)).end;
}

hipError_t parse_batch(const ParseArgs& a, void* scratch, size_t scratch_bytes, hipStream_t stream) {
  const uint64_t n = a.n;
  const uint64_t blocks = (n + kParseThreads - 1) / kParseThreads;
  const ParseLayout lay(n, a.items_cap, scan_temp_bytes(n));
  if (lay.end > scratch_bytes) return hipErrorInvalidValue;
  char* s = (char*)scratch;
  uint32_t* counts = (uint32_t*)(s + lay.counts);
  uint32_t* wg_counts = (uint32_t*)(s + lay.wg_counts);
  uint32_t* wg_firsts = (uint32_t*)(s + lay.wg_firsts);
  uint8_t* modes = (uint8_t*)(s + lay.modes);
  unsigned long long* cursor = (unsigned long long*)(s + lay.cursor);
  uint32_t* bases = (uint32_t*)(s + lay.bases);
  uint16_t* pos_seg = (uint16_t*)(s + lay.slots);
  void* temp = s + lay.temp;
  size_t temp_bytes = lay.end - lay.temp;
  hipError_t e = hipMemsetAsync(cursor, 0, 8, stream);
  if (e != hipSuccess) return e;
  parse_walk_pool_kernel<<<(unsigned)blocks, kParseThreads, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, counts,
                                                                         modes, pos_seg, cursor, bases, lay.seg_cap,
                                                                         wg_counts);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // each workgroup's first item (the emit adds the frames' own counts within the workgroup)
  e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, wg_counts, wg_firsts, (int)blocks, stream);
  if (e != hipSuccess) return e;
  // One item per thread per round, one non-temporal 16-byte load per header, non-temporal record
  // stores (the measured alternatives in profiles/EXPERIMENTS.md).  (A one-launch
  // parse -- walk, decoupled look-back scan and emit in one kernel -- measured 0.533 against 0.4206 ms
  // here, round 5.)
  parse_emit_kernel<1, 2, kEmitAux, true><<<(unsigned)blocks, kParseThreads, 0, stream>>>(
      a.bytes, a.offsets, n, a.valid, a.infos, counts, wg_firsts, modes, pos_seg, bases, a.items, a.items_cap,
      a.items_used);
  return hipGetLastError();
}

}  // namespace ufc_dev
