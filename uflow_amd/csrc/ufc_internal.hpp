// ufc_internal.hpp -- library-internal entry points shared by the C-ABI translation units
// (ufc_api.cpp, ufc_shard.cpp).  Not exported.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

struct ufc_ctx;

namespace ufc_internal {

constexpr uint64_t kMaxFrameLen = (uint64_t)1 << 30;  // per-frame limit of the 32-bit offsets math

// ufc_crc_batch_fixed with front_ok: the bytes before d_frames are readable (a later part of a
// larger batch), so the first frames need no edge handling.
int crc_fixed(ufc_ctx* ctx, const uint8_t* d_frames, size_t stride, size_t frame_len, size_t n, uint32_t* d_crc_out,
              uint8_t* d_valid_out, hipStream_t stream, bool front_ok);
int ctx_device(const ufc_ctx* ctx);
void note_hip_error(ufc_ctx* ctx, int e);
// A communicator on this context stalled (a peer missed the status agreement's deadline): an RCCL
// all-reduce stays pending on the device for good, so ufc_ctx_destroy must not free device memory
// (hipFree synchronizes the device and would wait for it).
void note_stall(ufc_ctx* ctx);

}  // namespace ufc_internal
