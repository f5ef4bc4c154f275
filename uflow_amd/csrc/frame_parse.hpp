// frame_parse.hpp -- interface between the C-ABI layer and the GPU batch parse (frame_parse.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/uflow_frame_codec.h"

namespace ufc_dev {

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

// Device scratch of a parse of n frames (item counts, first indices, scan temporaries).
size_t parse_scratch_bytes(uint64_t n);
hipError_t parse_batch(const ParseArgs& a, void* scratch, size_t scratch_bytes, hipStream_t stream);

}  // namespace ufc_dev
