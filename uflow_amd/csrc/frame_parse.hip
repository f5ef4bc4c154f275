// frame_parse.hip -- batched Frame::read after the batched CRC gate, on device-resident frames
// (on-GPU datagram header parse/validation).
//
// One thread per frame runs the payload parse of frame_codec_core.hpp (restating
// src/frame/serial/mod.rs:54-434, 694-705) over the frame's bytes in HBM: only header bytes are
// read (a datagram header, then a jump over its payload), by independent byte loads the compiler
// issues together (a 16-byte chunk cache in registers measured slower: its per-lane misses
// diverge).  Items leave as three 8-byte stores each.  Three steps on the caller's stream:
//   1. count:  gate (the CRC kernel's valid flag) + parse -> item count per frame;
//   2. scan:   exclusive sum of the item counts (hipcub) -> each frame's first item;
//   3. fill:   parse again, write the frame's ufc_frame_info and its items (datagram / ack group
//              descriptors) at its first index; the total goes to *items_used.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstddef>

#include "frame_codec_core.hpp"
#include "frame_parse.hpp"

namespace ufc_dev {

namespace {

struct DevBytes {
  const uint8_t* p;
  __device__ uint32_t operator()(uint32_t i) const {
    return *(const __attribute__((address_space(1))) uint8_t*)(p + i);
  }
};

// Items as three 8-byte stores each (ufc_item is 24 bytes, laid out as below).
static_assert(sizeof(ufc_item) == 24 && offsetof(ufc_item, channel_id) == 4 && offsetof(ufc_item, form) == 5 &&
                  offsetof(ufc_item, window_parent_lead) == 6 && offsetof(ufc_item, channel_parent_lead) == 8 &&
                  offsetof(ufc_item, fragment_id) == 10 && offsetof(ufc_item, fragment_id_last) == 12 &&
                  offsetof(ufc_item, flags) == 14 && offsetof(ufc_item, data_offset) == 16 &&
                  offsetof(ufc_item, data_len) == 20,
              "ufc_item layout");
struct PackedSink {
  ufc_item* p;
  __device__ bool on() const { return p != nullptr; }
  __device__ void operator()(uint32_t k, const ufc_item& it) const {
    typedef __attribute__((address_space(1))) uint64_t g_u64w;
    g_u64w* q = (g_u64w*)((uint8_t*)(p + k));
    q[0] = (uint64_t)it.id | ((uint64_t)it.channel_id << 32) | ((uint64_t)it.form << 40) |
           ((uint64_t)it.window_parent_lead << 48);
    q[1] = (uint64_t)it.channel_parent_lead | ((uint64_t)it.fragment_id << 16) |
           ((uint64_t)it.fragment_id_last << 32) | ((uint64_t)it.flags << 48);
    q[2] = (uint64_t)it.data_offset | ((uint64_t)it.data_len << 32);
  }
};

__device__ __forceinline__ uint32_t frame_len32(const uint64_t* offsets, uint64_t i, uint64_t& a) {
  a = offsets[i];
  const uint64_t b = offsets[i + 1];
  const uint64_t len64 = b >= a ? b - a : 0;
  return len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
}

__global__ __launch_bounds__(256) void parse_count_kernel(const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                                          const uint8_t* valid, uint32_t* counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t a;
  const uint32_t len = frame_len32(offsets, i, a);
  ufc_frame_info info;
  const bool ok = ufc_codec::read_frame_to(DevBytes{bytes + a}, len, valid[i] != 0, info, PackedSink{nullptr}, 0);
  counts[i] = ok ? info.item_count : 0u;
}

__global__ __launch_bounds__(256) void parse_fill_kernel(const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                                         const uint8_t* valid, ufc_frame_info* infos,
                                                         const uint32_t* counts, const uint32_t* firsts,
                                                         ufc_item* items, uint64_t cap, uint64_t* items_used) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t first = firsts[i], cnt = counts[i];
  if (i == n - 1 && items_used) *items_used = (uint64_t)first + cnt;
  uint64_t a;
  const uint32_t len = frame_len32(offsets, i, a);
  const uint32_t room = (cnt == 0 || !items || (uint64_t)first >= cap) ? 0u : (uint32_t)min((uint64_t)cnt, cap - first);
  ufc_frame_info info;
  ufc_codec::read_frame_to(DevBytes{bytes + a}, len, valid[i] != 0, info, PackedSink{room ? items + first : nullptr},
                           room);
  info.item_first = first;
  infos[i] = info;
}

}  // namespace

size_t parse_scratch_bytes(uint64_t n) {
  size_t temp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return 2 * ((n * 4 + 255) / 256 * 256) + (temp + 255) / 256 * 256;
}

hipError_t parse_batch(const ParseArgs& a, void* scratch, size_t scratch_bytes, hipStream_t stream) {
  const uint64_t n = a.n;
  const size_t arr = (n * 4 + 255) / 256 * 256;
  uint32_t* counts = (uint32_t*)scratch;
  uint32_t* firsts = (uint32_t*)((char*)scratch + arr);
  void* temp = (char*)scratch + 2 * arr;
  size_t temp_bytes = scratch_bytes - 2 * arr;
  const unsigned grid = (unsigned)((n + 255) / 256);
  parse_count_kernel<<<grid, 256, 0, stream>>>(a.bytes, a.offsets, n, a.valid, counts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, firsts, (int)n, stream);
  if (e != hipSuccess) return e;
  parse_fill_kernel<<<grid, 256, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, counts, firsts, a.items,
                                              a.items_cap, a.items_used);
  return hipGetLastError();
}

}  // namespace ufc_dev
