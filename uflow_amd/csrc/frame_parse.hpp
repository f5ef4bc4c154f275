// frame_parse.hpp -- interface between the C-ABI layer and the GPU batch parse (frame_parse.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/uflow_frame_codec.h"

namespace ufc_dev {

// Byte i (0..15) of a frame's first 16 bytes held as two little-endian words (the parse walk's head,
// frame_parse.hip DevBytesHead): shift amounts always in range (host and device; tests/c/ubsan_helpers.hip).
__host__ __device__ __forceinline__ uint32_t head_byte(uint64_t w0, uint64_t w1, uint32_t i) {
  return (uint32_t)(((i & 15u) < 8 ? w0 : w1) >> (8 * (i & 7u))) & 0xFFu;
}

struct ParseArgs {
  const uint8_t* bytes;
  const uint64_t* offsets;
  uint64_t n;              // frames (< 2^31: one scan)
  const uint8_t* valid;    // the CRC gate's flags
  ufc_frame_info* infos;
  ufc_item* items;         // nullable
  uint64_t items_cap;
  uint64_t* items_used;    // device word, nullable
};

// Device scratch of a parse of n frames with room for at most items_cap items (item counts, first
// indices, modes, scan temporaries, and header slots for min(64 n, items_cap) datagrams: the walk's
// workgroups take their slot segments from a bump counter, and a workgroup that finds no room left
// leaves its frames to the emit step's re-walk).
size_t parse_scratch_bytes(uint64_t n, uint64_t items_cap);
hipError_t parse_batch(const ParseArgs& a, void* scratch, size_t scratch_bytes, hipStream_t stream);

}  // namespace ufc_dev
