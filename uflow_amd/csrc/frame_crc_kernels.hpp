// frame_crc_kernels.hpp -- interface between the C-ABI layer and the HIP kernels.
#pragma once
#include <cstdint>

namespace ufc_dev {

constexpr int kModeVarlen = 1;  // frames from a CSR offsets array
constexpr int kModeSeal = 2;    // write the BE32 trailer instead of validating it
constexpr int kModeFreeze = 4;  // fixed-length frames whose block count is not a multiple of JC

constexpr int kBlockThreads = 1024;          // one workgroup per CU, 16 waves
constexpr int kLdsBytes = 131072 + 32768;    // chain tables + nibble tables

struct KernelParams {
  const uint8_t* bytes;       // batch base (fixed) or CSR byte buffer (varlen)
  uint8_t* wbytes;            // same buffer, writable (seal only)
  const uint64_t* offsets;    // varlen: n+1 offsets
  uint64_t stride;            // fixed: bytes between frame starts
  uint64_t frame_len;         // fixed: frame length
  uint64_t nframes;
  uint32_t* crc_out;          // nullable
  uint8_t* valid_out;         // nullable (validate mode)
  const uint32_t* chain_tab;  // device: 1024 words (A^256 byte tables)
  const uint32_t* nib_img;    // device: 8192 words (per-slot nibble tables, LDS image order)
  uint32_t G;                 // A^-4(~0)
  uint32_t* ctr;              // lean fixed kernel: per-workgroup claim counters (zero at launch)
  uint32_t front_ok;          // lean fixed kernel: the pad bytes before frame 0 are readable
  // Variable-length kernel: frames longer than its 13-line fast path (and in range) are left to a
  // second launch (frame_crc_long8_kernel): their indices go to defer_list (workgroup b's from entry
  // 64 * its first run on), workgroup b's count to defer_counts[b].  Null: they take the byte path.
  uint32_t* defer_list;
  uint32_t* defer_counts;
};

// Kernel entry for (JC 256-byte blocks per pipelined part, mode); nullptr if not instantiated.
const void* kernel_symbol(int jc, int mode);
bool config_available(int jc);
// Lean fixed-length kernel (frame_len >= 4, J = ceil((frame_len + 4) / 256) in 1..6); one
// workgroup per CU owning a contiguous range of 4-frame sets, spread over its waves by `sched`;
// `depth` sets in flight per wave.  Only the product configuration is instantiated (interleaved,
// 8 waves, depth 2); other arguments return nullptr.
constexpr int kLeanDepthDefault = 2;
// Results stay in registers until a wave's range is done: at most 16 * kLeanRuns sets per wave,
// i.e. a launch covers at most (waves in the grid) * 16 * kLeanRuns * 4 frames (host-chunked).
constexpr int kLeanRuns = 8;
// Runs of history per wave by wave count: 32 at 8 waves, kLeanRuns at 16 (register budget).
constexpr int lean_runs(int waves) { return waves == 8 ? 32 : kLeanRuns; }
constexpr int kLeanWavesDefault = 8;
// Schedules of a workgroup's contiguous set range over its waves: per-wave contiguous ranges,
// claimed one set at a time from a per-workgroup counter, or interleaved (wave i: lo + i + k*waves).
constexpr int kSchedRange = 0;
constexpr int kSchedClaim = 1;
constexpr int kSchedInterleave = 2;
constexpr int kLeanSchedDefault = kSchedInterleave;
const void* fixed_kernel_symbol(int J, bool seal, int depth, int sched, int waves);
constexpr int kRunFrames = 64;
// Variable-length kernel with 8 lanes per frame (frame_crc_varlen8.hip): CSR offsets (p.offsets,
// n + 1) or (start, end) pairs (p.offsets holds 2n words, p.frame_len the buffer length); each run of
// 64 frames ordered by piece count inside the kernel; 8-frame sets; A^128 chain tables and the
// 32-slot nibble image.  varlen8_waves(): the workgroup's waves (one workgroup per CU).
const void* varlen8_kernel_symbol(bool seal, bool pairs);
int varlen8_waves();
// The second launch over the frames the variable-length kernel deferred (p.defer_list / p.defer_counts of
// a first launch with the same p and `blocks` workgroups): one workgroup per first-launch workgroup,
// reading only its count when that is zero.
const void* long8_kernel_symbol(bool seal, bool pairs);
// Slot layout -> (start, end) pairs on the device: pairs[2i] = i * stride, pairs[2i+1] = i * stride
// + lens[i] (ufc_validate_host_slots_async).
int slots_to_pairs(const uint32_t* d_lens, uint64_t stride, uint64_t n, uint64_t* d_pairs, void* stream);
// Seal, second pass (fixed stride): write crc[i] big-endian at i * stride + frame_len - 4 for
// every frame, non-temporal (frame_len >= 4).  Returns a hipError_t.
int seal_scatter(uint8_t* bytes, uint64_t stride, uint64_t frame_len, uint64_t nframes, const uint32_t* crc,
                 void* stream);
// Read-only streaming ceiling (hbm_probe.hip): the first nbytes / 1024 KB of bytes as one contiguous
// stream, one workgroup of 8 waves per CU; XOR of the data into *sink.  Returns a hipError_t.
int read_stream(const uint8_t* bytes, uint64_t nbytes, uint32_t* sink, int ncu, void* stream);
// Claim-counter words per workgroup (the kernel uses the first two; one 128-byte line each).
constexpr int kCtrWordsPerBlock = 32;

}  // namespace ufc_dev
