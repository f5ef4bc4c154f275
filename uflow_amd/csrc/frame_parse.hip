// frame_parse.hip -- batched Frame::read after the batched CRC gate, on device-resident frames
// (on-GPU datagram header parse/validation).
//
// One thread per frame runs the payload parse of frame_codec_core.hpp (restating
// src/frame/serial/mod.rs:54-434, 694-705) over the frame's bytes in HBM: only header bytes are
// read (a datagram header, then a jump over its payload), so a frame costs a few dependent loads,
// not its length.  Three steps on the caller's stream:
//   1. count:  gate (the CRC kernel's valid flag) + parse -> ufc_frame_info, item count;
//   2. scan:   exclusive sum of the item counts (hipcub) -> each frame's first item;
//   3. fill:   accepted frames with items parse again and write their items (datagram / ack group
//              descriptors) at their first index; the total goes to *items_used.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

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

__global__ __launch_bounds__(256) void parse_count_kernel(const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                                          const uint8_t* valid, ufc_frame_info* infos,
                                                          uint32_t* counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = offsets[i], b = offsets[i + 1];
  const uint64_t len64 = b >= a ? b - a : 0;
  const uint32_t len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
  ufc_frame_info info;
  const bool ok = ufc_codec::read_frame(DevBytes{bytes + a}, len, valid[i] != 0, info, nullptr, 0);
  info.item_first = 0;
  infos[i] = info;
  counts[i] = ok ? info.item_count : 0u;
}

__global__ __launch_bounds__(256) void parse_fill_kernel(const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                                         ufc_frame_info* infos, const uint32_t* counts,
                                                         const uint32_t* firsts, ufc_item* items, uint64_t cap,
                                                         uint64_t* items_used) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t first = firsts[i], cnt = counts[i];
  infos[i].item_first = first;
  if (i == n - 1 && items_used) *items_used = (uint64_t)first + cnt;
  if (cnt == 0 || !items || (uint64_t)first >= cap) return;
  const uint64_t a = offsets[i];
  const uint32_t room = (uint32_t)min((uint64_t)cnt, cap - first);
  ufc_frame_info tmp;
  ufc_codec::read_frame(DevBytes{bytes + a}, (uint32_t)(offsets[i + 1] - a), true, tmp, items + first, room);
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
  parse_count_kernel<<<grid, 256, 0, stream>>>(a.bytes, a.offsets, n, a.valid, a.infos, counts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, firsts, (int)n, stream);
  if (e != hipSuccess) return e;
  parse_fill_kernel<<<grid, 256, 0, stream>>>(a.bytes, a.offsets, n, a.infos, counts, firsts, a.items, a.items_cap,
                                              a.items_used);
  return hipGetLastError();
}

}  // namespace ufc_dev
