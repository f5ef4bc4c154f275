// ufc_api.cpp -- C ABI of libuflowcrc.so (declared in include/uflow_frame_crc.h).
// Scalar host entry points mirror src/frame/serial/crc.rs:94-104 and the CRC gate / seal of
// src/frame/serial/mod.rs:463-470, 675-690; batched entry points launch the gfx950 kernels of
// frame_crc.hip.  Batched calls never fall back to the CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/uflow_frame_codec.h"
#include "../../include/uflow_frame_crc.h"
#include "crc_math.hpp"
#include "frame_crc_kernels.hpp"
#include "frame_parse.hpp"
#include "ufc_internal.hpp"

struct ufc_ctx {
  int device = -1;
  int ncu = 0;
  uint32_t* d_chain = nullptr;
  uint32_t* d_nib = nullptr;
  uint32_t* d_chain128 = nullptr;  // 8-lane varlen kernel: A^128 chain tables, 32-slot nibble image
  uint32_t* d_nib32 = nullptr;
  uint32_t G = 0;
  int last_hip_error = 0;
  std::atomic<int> stalled_comms{0};  // communicators of this context that stalled (ufc_internal::note_stall)
  // host-buffer path (ufc_validate_host_varlen): device staging, reused across calls
  uint8_t* d_stage = nullptr;
  size_t d_stage_cap = 0;
  uint64_t* d_off = nullptr;
  size_t d_off_cap = 0;  // entries
  uint32_t* d_crc = nullptr;
  uint8_t* d_valid = nullptr;
  size_t d_out_cap = 0;  // frames
  uint64_t* h_off_pinned = nullptr;
  size_t h_off_cap = 0;
  hipStream_t streams[2] = {nullptr, nullptr};
  // Claim counters of the lean fixed kernel: kCtrSlots slots of ncu * kCtrWordsPerBlock words,
  // zeroed at creation and reset by each launch's last wave; launches take slots round-robin, so
  // concurrent launches on different streams do not share counters (up to kCtrSlots in flight).
  uint32_t* d_ctr = nullptr;
  std::atomic<uint32_t> ctr_seq{0};
  // Kernel-selection options (ufc_ctx_set_option; A/B measurement and tests).
  int opt[UFC_OPT_COUNT_] = {};
  // Device scratch of the batch parse and of the sorted varlen mode, one grow-only buffer per
  // (kind, stream): work queued on different streams never shares scratch.
  struct Scratch {
    int kind;
    hipStream_t stream;
    void* p;
    size_t cap;
  };
  std::mutex scratch_mu;
  std::vector<Scratch> scratch;
};

constexpr uint32_t kCtrSlots = 64;

namespace {

enum ScratchKind { kScratchParse = 0, kScratchAsyncSlots = 2, kScratchSealCrc = 3, kScratchDeferList = 4, kScratchDeferCounts = 5 };

// The (kind, stream) scratch buffer of at least `need` bytes.  Growing waits for the work already
// queued on that stream (the only user of the old buffer) before freeing it.  *fresh (if given): the
// buffer was (re)allocated by this call.
hipError_t stream_scratch(ufc_ctx* ctx, int kind, hipStream_t stream, size_t need, void** out, bool* fresh = nullptr) {
  if (fresh) *fresh = false;
  std::lock_guard<std::mutex> lk(ctx->scratch_mu);
  ufc_ctx::Scratch* sc = nullptr;
  for (auto& x : ctx->scratch)
    if (x.kind == kind && x.stream == stream) sc = &x;
  if (!sc) {
    ctx->scratch.push_back({kind, stream, nullptr, 0});
    sc = &ctx->scratch.back();
  }
  if (sc->cap < need) {
    hipError_t e;
    if (sc->p) {
      if ((e = hipStreamSynchronize(stream)) != hipSuccess) return e;
      (void)hipFree(sc->p);
      sc->p = nullptr;
      sc->cap = 0;
    }
    if ((e = hipMalloc(&sc->p, need)) != hipSuccess) return e;
    sc->cap = need;
    if (fresh) *fresh = true;
  }
  *out = sc->p;
  return hipSuccess;
}

struct DeviceGuard {  // restores the caller's current device
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int hip_fail(ufc_ctx* ctx, hipError_t e) {
  if (ctx) ctx->last_hip_error = (int)e;
  return UFC_ERR_HIP;
}

struct Config {
  int jc;  // 256-byte blocks per pipelined part
};

int launch(ufc_ctx* ctx, Config cfg, int mode, ufc_dev::KernelParams& kp, hipStream_t stream) {
  const void* fn = ufc_dev::kernel_symbol(cfg.jc, mode);
  if (!fn) return UFC_ERR_INVALID_ARG;
  // A wave walks runs of 16 sets (64 frames); one 1024-thread workgroup per CU.
  const uint64_t nsets = (kp.nframes + 3) / 4;
  const uint64_t nruns = (nsets + 15) / 16;
  const uint64_t waves_per_block = ufc_dev::kBlockThreads / 64;
  uint64_t blocks = (nruns + waves_per_block - 1) / waves_per_block;
  if (blocks > (uint64_t)ctx->ncu) blocks = (uint64_t)ctx->ncu;
  if (blocks < 1) blocks = 1;
  kp.chain_tab = ctx->d_chain;
  kp.nib_img = ctx->d_nib;
  kp.G = ctx->G;
  void* args[] = {&kp};
  hipError_t e = hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(ufc_dev::kBlockThreads), args, 0, stream);
  if (e != hipSuccess) return hip_fail(ctx, e);
  return UFC_OK;
}

// Lean fixed-length kernel: J = blocks per frame when 4 <= frame_len and J <= 6, else 0.  The
// generic kernel stays reachable with UFC_OPT_FIXED_KERNEL = UFC_FIXED_GENERIC or a
// UFC_OPT_GENERIC_JC override (A/B measurement).  The batch must also hold a full 4-frame set
// past the edge sets (those whose first frames' pad bytes precede the buffer), which the kernel's
// out-of-range prefetches re-read.
int lean_fixed_blocks(const ufc_ctx* ctx, uint64_t frame_len, uint64_t stride, uint64_t n) {
  if (frame_len < 4) return 0;
  const uint64_t J = (frame_len + 4 + 255) / 256;
  if (J > 6 || stride >= (1ull << 28)) return 0;  // lane offsets (3 strides + 2 KiB) stay below 2^31
  const uint64_t pad = 256 * J - frame_len;
  const uint64_t s_edge = (pad + 4 * stride - 1) / (4 * stride);
  if (n / 4 <= s_edge) return 0;
  if (ctx->opt[UFC_OPT_FIXED_KERNEL] == UFC_FIXED_GENERIC || ctx->opt[UFC_OPT_GENERIC_JC] != 0) return 0;
  return (int)J;
}

// front_ok: the bytes before the batch's first frame are readable (a later part of a larger batch).
int launch_lean_fixed(ufc_ctx* ctx, int J, bool seal, ufc_dev::KernelParams& kp, hipStream_t stream,
                      bool front_ok = false) {
  const int depth = ufc_dev::kLeanDepthDefault, waves = ufc_dev::kLeanWavesDefault;
  const int sched = ufc_dev::kLeanSchedDefault;
  const void* fn = ufc_dev::fixed_kernel_symbol(J, seal, depth, sched, waves);
  if (!fn) return UFC_ERR_INVALID_ARG;
  kp.chain_tab = ctx->d_chain;
  kp.nib_img = ctx->d_nib;
  kp.G = ctx->G;
  // One 1024-thread workgroup per CU.  A launch covers at most `chunk` frames (32-bit set
  // indices; a wave's results mostly stay in registers until the end); every frame of a chunk
  // keeps its absolute address, and chunks after the first may read the pad bytes before them.
  const uint64_t waves_per_block = (uint64_t)waves;
  // (16 * kLeanRuns - 1 sets per wave: the static schedules' histories never overflow in the loop)
  const uint64_t chunk = (uint64_t)ctx->ncu * waves_per_block * (16 * ufc_dev::lean_runs(waves) - 1) * 4;
  const uint64_t total = kp.nframes;
  for (uint64_t f0 = 0, step = 0; f0 < total; f0 += step) {
    ufc_dev::KernelParams c = kp;
    c.nframes = std::min(chunk, total - f0);
    // Every launch needs a full set (see lean_fixed_blocks): never leave a final chunk of < 4 frames.
    if (total - f0 - c.nframes > 0 && total - f0 - c.nframes < 4) c.nframes -= 4;
    step = c.nframes;
    c.bytes = kp.bytes + f0 * kp.stride;
    if (kp.wbytes) c.wbytes = kp.wbytes + f0 * kp.stride;
    if (kp.crc_out) c.crc_out = kp.crc_out + f0;
    if (kp.valid_out) c.valid_out = kp.valid_out + f0;
    c.front_ok = (f0 > 0 || front_ok) ? 1u : 0u;
    // Claim counters: one slot of the ring per launch (zero on entry, reset by the kernel).
    const uint32_t slot = ctx->ctr_seq.fetch_add(1) % kCtrSlots;
    c.ctr = ctx->d_ctr + (size_t)slot * ctx->ncu * ufc_dev::kCtrWordsPerBlock;
    const uint64_t nsets = (c.nframes + 3) / 4;
    uint64_t blocks = (nsets + waves_per_block - 1) / waves_per_block;
    if (blocks > (uint64_t)ctx->ncu) blocks = (uint64_t)ctx->ncu;
    if (blocks < 1) blocks = 1;
    void* args[] = {&c};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)blocks), dim3((unsigned)(waves * 64)), args, 0, stream);
    if (e != hipSuccess) return hip_fail(ctx, e);
  }
  return UFC_OK;
}


// The sorted-runs kernel with 8 lanes per frame (frame_crc_varlen8.hip): one launch per chunk of
// < 2^29 frames, each run of 64 frames sorted by piece count inside the kernel.  Any buffer size:
// each set's loads are relative to its run's own base (a set whose frames lie 2 GB or more apart,
// possible with pairs, runs on the kernel's byte path).  Frames longer than its 13-line fast path are
// deferred by its byte path to a second launch on the same stream (frame_crc_long8_kernel): a per-stream
// list of frame indices (4 B per frame of a chunk) and per-workgroup counts (zeroed once when allocated;
// the second launch zeroes the counts it consumed).  A workgroup of the second launch with nothing
// deferred reads its count and returns.
int launch_varlen8(ufc_ctx* ctx, bool seal, bool pairs, ufc_dev::KernelParams& kp, hipStream_t stream) {
  const void* fn = ufc_dev::varlen8_kernel_symbol(seal, pairs);
  const void* fn_long = ufc_dev::long8_kernel_symbol(seal, pairs);
  if (!fn || !fn_long) return UFC_ERR_INVALID_ARG;
  const int waves = ufc_dev::varlen8_waves();
  kp.chain_tab = ctx->d_chain128;
  kp.nib_img = ctx->d_nib32;
  kp.G = ctx->G;
  const uint64_t chunk = (uint64_t)1 << 29;  // (32-bit set indices: 8 per run of 64 frames)
  const uint64_t total = kp.nframes;
  void* list = nullptr;
  void* counts = nullptr;
  bool fresh = false;
  hipError_t e;
  const uint64_t nmax = std::min(chunk, total);
  if ((e = stream_scratch(ctx, kScratchDeferList, stream, (size_t)(nmax + 64) * 4, &list)) != hipSuccess ||
      (e = stream_scratch(ctx, kScratchDeferCounts, stream, (size_t)ctx->ncu * 4, &counts, &fresh)) != hipSuccess)
    return hip_fail(ctx, e);
  if (fresh && (e = hipMemsetAsync(counts, 0, (size_t)ctx->ncu * 4, stream)) != hipSuccess) return hip_fail(ctx, e);
  for (uint64_t f0 = 0; f0 < total; f0 += chunk) {
    ufc_dev::KernelParams c = kp;
    c.nframes = std::min(chunk, total - f0);
    c.offsets = kp.offsets + (pairs ? 2 * f0 : f0);
    if (kp.crc_out) c.crc_out = kp.crc_out + f0;
    if (kp.valid_out) c.valid_out = kp.valid_out + f0;
    c.defer_list = (uint32_t*)list;
    c.defer_counts = (uint32_t*)counts;
    // one workgroup per CU, at least one run of 64 frames per wave
    const uint64_t nruns = (c.nframes + 63) / 64;
    uint64_t blocks = (nruns + waves - 1) / waves;
    if (blocks > (uint64_t)ctx->ncu) blocks = (uint64_t)ctx->ncu;
    if (blocks < 1) blocks = 1;
    void* args[] = {&c};
    if ((e = hipLaunchKernel(fn, dim3((unsigned)blocks), dim3((unsigned)(waves * 64)), args, 0, stream)) != hipSuccess)
      return hip_fail(ctx, e);
    uint32_t nb = (uint32_t)blocks;
    void* args_long[] = {&c, &nb};
    if ((e = hipLaunchKernel(fn_long, dim3((unsigned)blocks), dim3((unsigned)(waves * 64)), args_long, 0, stream)) !=
        hipSuccess)
      return hip_fail(ctx, e);
  }
  return UFC_OK;
}

// Kernel configuration and mode bits for a fixed frame length: J = 256-byte blocks per frame.
Config fixed_config(const ufc_ctx* ctx, uint64_t frame_len, int* freeze) {
  const uint64_t n = frame_len >= 4 ? frame_len - 4 : frame_len;
  const uint64_t J = (n + 8 + 255) / 256;  // virtual stream: G + n bytes + trailer, 256-B blocks
  Config c;
  const int jc = ctx->opt[UFC_OPT_GENERIC_JC];
  c.jc = ufc_dev::config_available(jc) ? jc : (J <= 6 ? (int)J : 6);
  // Without freeze the kernel assumes one part per set (JC == J); anything else runs in freeze mode.
  *freeze = ((uint64_t)c.jc == J) ? 0 : ufc_dev::kModeFreeze;
  return c;
}

Config varlen_config(const ufc_ctx* ctx) {
  const int jc = ctx->opt[UFC_OPT_GENERIC_JC];
  return Config{ufc_dev::config_available(jc) ? jc : 3};
}

// Variable-length batches: the sorted-runs 8-lane kernel; the generic kernel by option (CSR only).
int launch_varlen_any(ufc_ctx* ctx, bool seal, bool pairs, ufc_dev::KernelParams& kp, hipStream_t stream) {
  if (ctx->opt[UFC_OPT_VARLEN_KERNEL] == UFC_VARLEN_GENERIC && !pairs)
    return launch(ctx, varlen_config(ctx), ufc_dev::kModeVarlen | (seal ? ufc_dev::kModeSeal : 0), kp, stream);
  return launch_varlen8(ctx, seal, pairs, kp, stream);
}

using ufc_internal::kMaxFrameLen;

}  // namespace

extern "C" {

uint32_t ufc_crc32_compute(const uint8_t* data, size_t len) {
  if (!data) return 0;
  return ufc::host_extend(0u, data, len);
}

uint32_t ufc_crc32_extend(uint32_t initial_crc, const uint8_t* data, size_t len) {
  if (!data) return initial_crc;
  return ufc::host_extend(initial_crc, data, len);
}

int ufc_frame_validate(const uint8_t* frame, size_t len) {
  if (!frame || len < 5) return 0;
  const uint32_t c = ufc::host_extend(0u, frame, len - 4);
  const uint8_t* t = frame + len - 4;
  const uint32_t rx = ((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | (uint32_t)t[3];
  return c == rx ? 1 : 0;
}

int ufc_frame_seal(uint8_t* frame, size_t len) {
  if (!frame || len < 4) return UFC_ERR_INVALID_ARG;
  const uint32_t c = ufc::host_extend(0u, frame, len - 4);
  uint8_t* t = frame + len - 4;
  t[0] = (uint8_t)(c >> 24);
  t[1] = (uint8_t)(c >> 16);
  t[2] = (uint8_t)(c >> 8);
  t[3] = (uint8_t)c;
  return UFC_OK;
}

int ufc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* ufc_error_string(int code) {
  switch (code) {
    case UFC_OK: return "ok";
    case UFC_ERR_INVALID_ARG: return "invalid argument";
    case UFC_ERR_NO_DEVICE: return "no usable gfx950 (MI355X) device";
    case UFC_ERR_HIP: return "HIP runtime error (see ufc_ctx_last_hip_error)";
    case UFC_ERR_NOMEM: return "out of memory";
    case UFC_ERR_COMM: return "RCCL unavailable or failed (see ufc_comm_last_error)";
    case UFC_ERR_PEER: return "another rank rejected its part of this sharded call (nothing was transferred)";
    default: return "unknown error";
  }
}

int ufc_ctx_last_hip_error(const ufc_ctx* ctx) { return ctx ? ctx->last_hip_error : 0; }

int ufc_ctx_set_option(ufc_ctx* ctx, int option, int value) {
  if (!ctx || option < 0 || option >= UFC_OPT_COUNT_) return UFC_ERR_INVALID_ARG;
  switch (option) {
    case UFC_OPT_FIXED_KERNEL:
      if (value != UFC_FIXED_AUTO && value != UFC_FIXED_GENERIC) return UFC_ERR_INVALID_ARG;
      break;
    case UFC_OPT_VARLEN_KERNEL:
      if (value != UFC_VARLEN_AUTO && value != UFC_VARLEN_GENERIC && value != UFC_VARLEN_SORTED8)
        return UFC_ERR_INVALID_ARG;
      break;
    case UFC_OPT_GENERIC_JC:
      if (value != 0 && !ufc_dev::config_available(value)) return UFC_ERR_INVALID_ARG;
      break;
    case UFC_OPT_SEAL_KERNEL:
      if (value != UFC_SEAL_INLINE && value != UFC_SEAL_TWO_PASS) return UFC_ERR_INVALID_ARG;
      break;
    default: return UFC_ERR_INVALID_ARG;
  }
  ctx->opt[option] = value;
  return UFC_OK;
}

int ufc_ctx_get_option(const ufc_ctx* ctx, int option) {
  if (!ctx || option < 0 || option >= UFC_OPT_COUNT_) return UFC_ERR_INVALID_ARG;
  return ctx->opt[option];
}

int ufc_ctx_create(ufc_ctx** out, int device) {
  if (!out) return UFC_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return UFC_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return UFC_ERR_INVALID_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return UFC_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return UFC_ERR_NO_DEVICE;
  DeviceGuard g(device);
  ufc_ctx* ctx = new (std::nothrow) ufc_ctx();
  if (!ctx) return UFC_ERR_NOMEM;
  ctx->device = device;
  ctx->ncu = prop.multiProcessorCount;
  std::vector<uint32_t> chain(1024), nib(8192), chain128(1024), nib32(8192);
  ufc::build_chain_table(chain.data(), 256);
  ufc::build_nibble_image(nib.data());
  ufc::build_chain_table(chain128.data(), 128);
  ufc::build_nibble_image32(nib32.data());
  ctx->G = ufc::init_prefix_word();
  ctx->opt[UFC_OPT_SEAL_KERNEL] = UFC_SEAL_INLINE;  // (the other options default to 0)
  hipError_t e;
  if ((e = hipMalloc(&ctx->d_chain, chain.size() * 4)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_nib, nib.size() * 4)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_chain128, chain128.size() * 4)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_nib32, nib32.size() * 4)) != hipSuccess ||
      (e = hipMemcpy(ctx->d_chain, chain.data(), chain.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(ctx->d_nib, nib.data(), nib.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(ctx->d_chain128, chain128.data(), chain128.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(ctx->d_nib32, nib32.data(), nib32.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMalloc(&ctx->d_ctr, (size_t)kCtrSlots * ctx->ncu * ufc_dev::kCtrWordsPerBlock * 4)) != hipSuccess ||
      (e = hipMemset(ctx->d_ctr, 0, (size_t)kCtrSlots * ctx->ncu * ufc_dev::kCtrWordsPerBlock * 4)) != hipSuccess ||
      (e = hipDeviceSynchronize()) != hipSuccess) {
    ufc_ctx_destroy(ctx);
    return UFC_ERR_HIP;
  }
  // The kernels declare their 160 KiB of LDS statically: no dynamic-LDS attribute to set.
  *out = ctx;
  return UFC_OK;
}

int ufc_ctx_release_stream(ufc_ctx* ctx, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  DeviceGuard g(ctx->device);
  bool any = false;
  {
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    for (const auto& sc : ctx->scratch) any = any || sc.stream == (hipStream_t)stream;
  }
  if (!any) return UFC_OK;
  // The work queued on the stream may still use its scratch: wait for it without holding the lock,
  // so that scratch lookups of other streams go on meanwhile (the caller is retiring this stream and
  // queues nothing more on it).
  const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(ctx, e);
  std::vector<void*> dead;
  {
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    for (size_t i = 0; i < ctx->scratch.size();) {
      if (ctx->scratch[i].stream != (hipStream_t)stream) {
        i++;
        continue;
      }
      if (ctx->scratch[i].p) dead.push_back(ctx->scratch[i].p);
      ctx->scratch.erase(ctx->scratch.begin() + (long)i);
    }
  }
  for (void* p : dead) (void)hipFree(p);
  return UFC_OK;
}

int ufc_ctx_destroy(ufc_ctx* ctx) {
  if (!ctx) return UFC_OK;
  if (ctx->stalled_comms.load() > 0) {
    // A stalled communicator's all-reduce is still pending on the device (ufc_comm_set_timeout): every
    // hipFree / hipStreamDestroy below would synchronize with it and never return.  The device memory
    // and streams are left to process exit; the handle is gone.
    delete ctx;
    return UFC_ERR_COMM;
  }
  {
    DeviceGuard g(ctx->device >= 0 ? ctx->device : 0);
    if (ctx->d_chain) (void)hipFree(ctx->d_chain);
    if (ctx->d_nib) (void)hipFree(ctx->d_nib);
    if (ctx->d_chain128) (void)hipFree(ctx->d_chain128);
    if (ctx->d_nib32) (void)hipFree(ctx->d_nib32);
    if (ctx->d_ctr) (void)hipFree(ctx->d_ctr);
    for (auto& sc : ctx->scratch)
      if (sc.p) (void)hipFree(sc.p);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->d_off) (void)hipFree(ctx->d_off);
    if (ctx->d_crc) (void)hipFree(ctx->d_crc);
    if (ctx->d_valid) (void)hipFree(ctx->d_valid);
    if (ctx->h_off_pinned) (void)hipHostFree(ctx->h_off_pinned);
    for (hipStream_t& s : ctx->streams)
      if (s) (void)hipStreamDestroy(s);
  }
  delete ctx;
  return UFC_OK;
}

int ufc_hbm_read_probe(ufc_ctx* ctx, const uint8_t* d_buf, size_t bytes, uint32_t* d_sink, size_t* bytes_read,
                       void* stream) {
  if (!ctx || !d_sink || (bytes >= 1024 && !d_buf)) return UFC_ERR_INVALID_ARG;
  if (bytes_read) *bytes_read = bytes / 1024 * 1024;
  DeviceGuard g(ctx->device);
  const hipError_t e = (hipError_t)ufc_dev::read_stream(d_buf, bytes, d_sink, ctx->ncu, stream);
  return e == hipSuccess ? UFC_OK : hip_fail(ctx, e);
}

int ufc_crc_batch_fixed(ufc_ctx* ctx, const uint8_t* d_frames, size_t stride, size_t frame_len, size_t n,
                        uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream) {
  return ufc_internal::crc_fixed(ctx, d_frames, stride, frame_len, n, d_crc_out, d_valid_out, (hipStream_t)stream,
                                 false);
}

}  // extern "C"

int ufc_internal::ctx_device(const ufc_ctx* ctx) { return ctx ? ctx->device : -1; }

void ufc_internal::note_hip_error(ufc_ctx* ctx, int e) {
  if (ctx) ctx->last_hip_error = e;
}

void ufc_internal::note_stall(ufc_ctx* ctx) {
  if (ctx) ctx->stalled_comms.fetch_add(1);
}

int ufc_internal::crc_fixed(ufc_ctx* ctx, const uint8_t* d_frames, size_t stride, size_t frame_len, size_t n,
                            uint32_t* d_crc_out, uint8_t* d_valid_out, hipStream_t stream, bool front_ok) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_frames || stride < frame_len || frame_len > kMaxFrameLen || (!d_crc_out && !d_valid_out))
    return UFC_ERR_INVALID_ARG;
  int freeze;
  const Config cfg = fixed_config(ctx, frame_len, &freeze);
  int lean = lean_fixed_blocks(ctx, frame_len, stride, n);
  ufc_dev::KernelParams kp{};
  kp.bytes = d_frames;
  kp.stride = stride;
  kp.frame_len = frame_len;
  kp.nframes = n;
  kp.crc_out = d_crc_out;
  kp.valid_out = d_valid_out;
  DeviceGuard g(ctx->device);
  if (lean) return launch_lean_fixed(ctx, lean, false, kp, stream, front_ok);
  return launch(ctx, cfg, freeze, kp, stream);
}

extern "C" {

int ufc_crc_batch_varlen(ufc_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                         uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_bytes || !d_offsets || (!d_crc_out && !d_valid_out)) return UFC_ERR_INVALID_ARG;
  ufc_dev::KernelParams kp{};
  kp.bytes = d_bytes;
  kp.offsets = d_offsets;
  kp.nframes = n;
  kp.crc_out = d_crc_out;
  kp.valid_out = d_valid_out;
  DeviceGuard g(ctx->device);
  return launch_varlen_any(ctx, false, false, kp, (hipStream_t)stream);
}

int ufc_seal_batch_fixed(ufc_ctx* ctx, uint8_t* d_frames, size_t stride, size_t frame_len, size_t n,
                         uint32_t* d_crc_out, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_frames || stride < frame_len || frame_len < 4 || frame_len > kMaxFrameLen) return UFC_ERR_INVALID_ARG;
  int freeze;
  const Config cfg = fixed_config(ctx, frame_len, &freeze);
  ufc_dev::KernelParams kp{};
  kp.bytes = d_frames;
  kp.wbytes = d_frames;
  kp.stride = stride;
  kp.frame_len = frame_len;
  kp.nframes = n;
  kp.crc_out = d_crc_out;
  DeviceGuard g(ctx->device);
  if (const int lean = lean_fixed_blocks(ctx, frame_len, stride, n)) {
    // Default: the CRC kernel writes its trailers itself, each workgroup after its last read, in
    // frame order from the LDS-staged results with non-temporal stores (DESIGN.md section 5.3:
    // 0.2665 against 0.2795 ms for two passes, config 2's 1M x 1500 B).
    if (ctx->opt[UFC_OPT_SEAL_KERNEL] == UFC_SEAL_INLINE) return launch_lean_fixed(ctx, lean, true, kp, (hipStream_t)stream);
    // UFC_SEAL_TWO_PASS: the validate kernel's CRC words (into the caller's crc_out, or per-stream
    // scratch), then every trailer with non-temporal stores once the whole batch has been read.
    uint32_t* crc = d_crc_out;
    hipError_t e;
    if (!crc && (e = stream_scratch(ctx, kScratchSealCrc, (hipStream_t)stream, n * 4, (void**)&crc)) != hipSuccess)
      return hip_fail(ctx, e);
    kp.wbytes = nullptr;
    kp.crc_out = crc;
    if (const int r = launch_lean_fixed(ctx, lean, false, kp, (hipStream_t)stream)) return r;
    if ((e = (hipError_t)ufc_dev::seal_scatter(d_frames, stride, frame_len, n, crc, stream)) != hipSuccess)
      return hip_fail(ctx, e);
    return UFC_OK;
  }
  return launch(ctx, cfg, freeze | ufc_dev::kModeSeal, kp, (hipStream_t)stream);
}

int ufc_seal_batch_varlen(ufc_ctx* ctx, uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                          uint32_t* d_crc_out, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_bytes || !d_offsets) return UFC_ERR_INVALID_ARG;
  ufc_dev::KernelParams kp{};
  kp.bytes = d_bytes;
  kp.wbytes = d_bytes;
  kp.offsets = d_offsets;
  kp.nframes = n;
  kp.crc_out = d_crc_out;
  DeviceGuard g(ctx->device);
  return launch_varlen_any(ctx, true, false, kp, (hipStream_t)stream);
}

static int validate_host_varlen_impl(ufc_ctx* ctx, const uint8_t* h_bytes, const uint64_t* h_offsets, size_t n,
                                     uint32_t* h_crc_out, uint8_t* h_valid_out) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!h_bytes || !h_offsets || (!h_crc_out && !h_valid_out)) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (h_offsets[i + 1] < h_offsets[i]) return UFC_ERR_INVALID_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e;
  for (hipStream_t& s : ctx->streams)
    if (!s && (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return hip_fail(ctx, e);
  // Chunking: frames are split into chunks of at most kChunkBytes of frame data (or one frame);
  // chunk k uses staging slot k&1 on stream k&1, so H2D of chunk k+1 overlaps the CRC of chunk k.
  const size_t kChunkBytes = (size_t)64 << 20;
  const size_t kChunkFrames = (size_t)1 << 20;
  const uint64_t base = h_offsets[0];
  const uint64_t total = h_offsets[n] - base;
  size_t max_chunk_bytes = 0, max_chunk_frames = 0;
  std::vector<size_t> cuts;  // frame index boundaries
  cuts.push_back(0);
  while (cuts.back() < n) {
    size_t a = cuts.back(), b = a + 1;
    while (b < n && b - a < kChunkFrames && h_offsets[b + 1] - h_offsets[a] <= kChunkBytes) b++;
    const size_t cb = (size_t)(h_offsets[b] - h_offsets[a]);
    if (cb > max_chunk_bytes) max_chunk_bytes = cb;
    if (b - a > max_chunk_frames) max_chunk_frames = b - a;
    cuts.push_back(b);
  }
  (void)total;
  // Grow staging (2 slots each).
  if (ctx->d_stage_cap < 2 * max_chunk_bytes + 64) {
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    ctx->d_stage = nullptr;
    ctx->d_stage_cap = 0;
    if ((e = hipMalloc(&ctx->d_stage, 2 * max_chunk_bytes + 64)) != hipSuccess) return hip_fail(ctx, e);
    ctx->d_stage_cap = 2 * max_chunk_bytes + 64;
  }
  const size_t need_off = 2 * (max_chunk_frames + 1);
  if (ctx->d_off_cap < need_off) {
    if (ctx->d_off) (void)hipFree(ctx->d_off);
    if (ctx->h_off_pinned) (void)hipHostFree(ctx->h_off_pinned);
    ctx->d_off = nullptr;
    ctx->h_off_pinned = nullptr;
    ctx->d_off_cap = ctx->h_off_cap = 0;
    if ((e = hipMalloc(&ctx->d_off, need_off * 8)) != hipSuccess) return hip_fail(ctx, e);
    if ((e = hipHostMalloc(&ctx->h_off_pinned, need_off * 8, hipHostMallocDefault)) != hipSuccess)
      return hip_fail(ctx, e);
    ctx->d_off_cap = ctx->h_off_cap = need_off;
  }
  if (ctx->d_out_cap < 2 * max_chunk_frames) {
    if (ctx->d_crc) (void)hipFree(ctx->d_crc);
    if (ctx->d_valid) (void)hipFree(ctx->d_valid);
    ctx->d_crc = nullptr;
    ctx->d_valid = nullptr;
    ctx->d_out_cap = 0;
    if ((e = hipMalloc(&ctx->d_crc, 2 * max_chunk_frames * 4)) != hipSuccess) return hip_fail(ctx, e);
    if ((e = hipMalloc(&ctx->d_valid, 2 * max_chunk_frames)) != hipSuccess) return hip_fail(ctx, e);
    ctx->d_out_cap = 2 * max_chunk_frames;
  }
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    const int slot = (int)(k & 1);
    hipStream_t s = ctx->streams[slot];
    const size_t a = cuts[k], b = cuts[k + 1], nf = b - a;
    const uint64_t off0 = h_offsets[a];
    const size_t bytes = (size_t)(h_offsets[b] - off0);
    uint8_t* dst = ctx->d_stage + (size_t)slot * (max_chunk_bytes + 32);
    uint64_t* hoff = ctx->h_off_pinned + (size_t)slot * (max_chunk_frames + 1);
    uint64_t* doff = ctx->d_off + (size_t)slot * (max_chunk_frames + 1);
    uint32_t* dcrc = ctx->d_crc + (size_t)slot * max_chunk_frames;
    uint8_t* dval = ctx->d_valid + (size_t)slot * max_chunk_frames;
    // the pinned offsets slot may still be in use by the H2D of chunk k-2 on the same stream
    if (k >= 2 && (e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e);
    for (size_t i = 0; i <= nf; i++) hoff[i] = h_offsets[a + i] - off0;
    if (bytes && (e = hipMemcpyAsync(dst, h_bytes + off0, bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
      return hip_fail(ctx, e);
    if ((e = hipMemcpyAsync(doff, hoff, (nf + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e);
    ufc_dev::KernelParams kp{};
    kp.bytes = dst;
    kp.offsets = doff;
    kp.nframes = nf;
    kp.crc_out = dcrc;
    kp.valid_out = dval;
    int rc = launch_varlen_any(ctx, false, false, kp, s);
    if (rc != UFC_OK) return rc;
    if (h_crc_out && (e = hipMemcpyAsync(h_crc_out + a, dcrc, nf * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return hip_fail(ctx, e);
    if (h_valid_out && (e = hipMemcpyAsync(h_valid_out + a, dval, nf, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return hip_fail(ctx, e);
  }
  for (hipStream_t s : ctx->streams)
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e);
  return UFC_OK;
}

int ufc_crc_batch_pairs(ufc_ctx* ctx, const uint8_t* d_bytes, size_t bytes_len, const uint64_t* d_pairs, size_t n,
                        uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_bytes || !d_pairs || (!d_crc_out && !d_valid_out)) return UFC_ERR_INVALID_ARG;
  ufc_dev::KernelParams kp{};
  kp.bytes = d_bytes;
  kp.offsets = d_pairs;
  kp.frame_len = bytes_len;
  kp.nframes = n;
  kp.crc_out = d_crc_out;
  kp.valid_out = d_valid_out;
  DeviceGuard g(ctx->device);
  return launch_varlen_any(ctx, false, true, kp, (hipStream_t)stream);
}

static int validate_host_slots_impl(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens,
                                    size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!h_slots || !h_lens || slot_stride == 0 || (!h_crc_out && !h_valid_out)) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (h_lens[i] > slot_stride) return UFC_ERR_INVALID_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e;
  for (hipStream_t& s : ctx->streams)
    if (!s && (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return hip_fail(ctx, e);
  // Chunks of whole slots (<= 64 MB); chunk k on stream/slot k & 1, as ufc_validate_host_varlen.
  const size_t per = std::max<size_t>(1, std::min<size_t>((size_t)1 << 20, ((size_t)64 << 20) / slot_stride));
  const size_t cf = std::min(per, n);
  const size_t cb = cf * slot_stride;
  if (ctx->d_stage_cap < 2 * cb + 64) {
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    ctx->d_stage = nullptr;
    ctx->d_stage_cap = 0;
    if ((e = hipMalloc(&ctx->d_stage, 2 * cb + 64)) != hipSuccess) return hip_fail(ctx, e);
    ctx->d_stage_cap = 2 * cb + 64;
  }
  if (ctx->d_off_cap < 4 * cf) {
    if (ctx->d_off) (void)hipFree(ctx->d_off);
    if (ctx->h_off_pinned) (void)hipHostFree(ctx->h_off_pinned);
    ctx->d_off = nullptr;
    ctx->h_off_pinned = nullptr;
    ctx->d_off_cap = ctx->h_off_cap = 0;
    if ((e = hipMalloc(&ctx->d_off, 4 * cf * 8)) != hipSuccess) return hip_fail(ctx, e);
    if ((e = hipHostMalloc(&ctx->h_off_pinned, 4 * cf * 8, hipHostMallocDefault)) != hipSuccess) return hip_fail(ctx, e);
    ctx->d_off_cap = ctx->h_off_cap = 4 * cf;
  }
  if (ctx->d_out_cap < 2 * cf) {
    if (ctx->d_crc) (void)hipFree(ctx->d_crc);
    if (ctx->d_valid) (void)hipFree(ctx->d_valid);
    ctx->d_crc = nullptr;
    ctx->d_valid = nullptr;
    ctx->d_out_cap = 0;
    if ((e = hipMalloc(&ctx->d_crc, 2 * cf * 4)) != hipSuccess) return hip_fail(ctx, e);
    if ((e = hipMalloc(&ctx->d_valid, 2 * cf)) != hipSuccess) return hip_fail(ctx, e);
    ctx->d_out_cap = 2 * cf;
  }
  size_t k = 0;
  for (size_t a = 0; a < n; a += cf, k++) {
    const int slot = (int)(k & 1);
    hipStream_t s = ctx->streams[slot];
    const size_t nf = std::min(cf, n - a);
    uint8_t* dst = ctx->d_stage + (size_t)slot * (cb + 32);
    uint64_t* hp = ctx->h_off_pinned + (size_t)slot * 2 * cf;
    uint64_t* dp = ctx->d_off + (size_t)slot * 2 * cf;
    if (k >= 2 && (e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e);
    for (size_t i = 0; i < nf; i++) {
      hp[2 * i] = (uint64_t)i * slot_stride;
      hp[2 * i + 1] = (uint64_t)i * slot_stride + h_lens[a + i];
    }
    // the last slot only up to its datagram's end (the slab may end there)
    const size_t bytes = (nf - 1) * slot_stride + h_lens[a + nf - 1];
    if (bytes && (e = hipMemcpyAsync(dst, h_slots + a * slot_stride, bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
      return hip_fail(ctx, e);
    if ((e = hipMemcpyAsync(dp, hp, nf * 16, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e);
    uint32_t* dcrc = ctx->d_crc + (size_t)slot * cf;
    uint8_t* dval = ctx->d_valid + (size_t)slot * cf;
    int rc = ufc_crc_batch_pairs(ctx, dst, bytes, dp, nf, dcrc, dval, s);
    if (rc != UFC_OK) return rc;
    if (h_crc_out && (e = hipMemcpyAsync(h_crc_out + a, dcrc, nf * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return hip_fail(ctx, e);
    if (h_valid_out && (e = hipMemcpyAsync(h_valid_out + a, dval, nf, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return hip_fail(ctx, e);
  }
  for (hipStream_t s : ctx->streams)
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e);
  return UFC_OK;
}

// Staging of one asynchronous slots batch, in the (ctx, stream) scratch: the slots' bytes, the
// lengths, the pairs, the CRC words and the valid bytes, each 256-byte aligned.
static int validate_host_slots_async_impl(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride,
                                          const uint32_t* h_lens, size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out,
                                          hipStream_t stream) {
  if (!ctx || !stream) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!h_slots || !h_lens || slot_stride == 0 || (!h_crc_out && !h_valid_out)) return UFC_ERR_INVALID_ARG;
  if (n > (((size_t)1 << 31) - ((size_t)1 << 20)) / slot_stride) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (h_lens[i] > slot_stride) return UFC_ERR_INVALID_ARG;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t bytes = (n - 1) * slot_stride + h_lens[n - 1];  // the slab may end at the last datagram
  const size_t o_lens = up(bytes + 64), o_pairs = o_lens + up(4 * n), o_crc = o_pairs + up(16 * n),
               o_valid = o_crc + up(4 * n), need = o_valid + up(n);
  void* sp = nullptr;
  hipError_t e;
  if ((e = stream_scratch(ctx, kScratchAsyncSlots, stream, need, &sp)) != hipSuccess) return hip_fail(ctx, e);
  uint8_t* s = (uint8_t*)sp;
  uint32_t* d_lens = (uint32_t*)(s + o_lens);
  uint64_t* d_pairs = (uint64_t*)(s + o_pairs);
  uint32_t* d_crc = (uint32_t*)(s + o_crc);
  uint8_t* d_valid = s + o_valid;
  if ((e = hipMemcpyAsync(s, h_slots, bytes, hipMemcpyHostToDevice, stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_lens, h_lens, 4 * n, hipMemcpyHostToDevice, stream)) != hipSuccess)
    return hip_fail(ctx, e);
  if ((e = (hipError_t)ufc_dev::slots_to_pairs(d_lens, slot_stride, n, d_pairs, stream)) != hipSuccess)
    return hip_fail(ctx, e);
  const int rc = ufc_crc_batch_pairs(ctx, s, bytes, d_pairs, n, d_crc, d_valid, stream);
  if (rc != UFC_OK) return rc;
  if (h_crc_out && (e = hipMemcpyAsync(h_crc_out, d_crc, 4 * n, hipMemcpyDeviceToHost, stream)) != hipSuccess)
    return hip_fail(ctx, e);
  if (h_valid_out && (e = hipMemcpyAsync(h_valid_out, d_valid, n, hipMemcpyDeviceToHost, stream)) != hipSuccess)
    return hip_fail(ctx, e);
  return UFC_OK;
}

// After a failure part-way through a host-buffer call, copies of earlier chunks may still be
// queued on the context's streams (reading the caller's frames, writing its outputs): wait for
// them before returning, so that nothing touches the caller's buffers after the call.
static int drain_on_error(ufc_ctx* ctx, int rc) {
  if (rc != UFC_OK && ctx)
    for (hipStream_t s : ctx->streams)
      if (s) (void)hipStreamSynchronize(s);
  return rc;
}

int ufc_validate_host_varlen(ufc_ctx* ctx, const uint8_t* h_bytes, const uint64_t* h_offsets, size_t n,
                             uint32_t* h_crc_out, uint8_t* h_valid_out) {
  DeviceGuard g(ctx ? ctx->device : 0);
  return drain_on_error(ctx, validate_host_varlen_impl(ctx, h_bytes, h_offsets, n, h_crc_out, h_valid_out));
}

int ufc_validate_host_slots(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens,
                            size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out) {
  DeviceGuard g(ctx ? ctx->device : 0);
  return drain_on_error(ctx, validate_host_slots_impl(ctx, h_slots, slot_stride, h_lens, n, h_crc_out, h_valid_out));
}

int ufc_validate_host_slots_async(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens,
                                  size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out, void* stream) {
  DeviceGuard g(ctx ? ctx->device : 0);
  const int rc = validate_host_slots_async_impl(ctx, h_slots, slot_stride, h_lens, n, h_crc_out, h_valid_out,
                                                (hipStream_t)stream);
  // on error, nothing queued by this call may still touch the caller's buffers
  if (rc != UFC_OK && ctx && stream) (void)hipStreamSynchronize((hipStream_t)stream);
  return rc;
}

namespace {
void put_trailer(uint8_t* f, size_t len, uint32_t crc) {  // serial/mod.rs:466-470
  uint8_t* t = f + len - 4;
  t[0] = (uint8_t)(crc >> 24);
  t[1] = (uint8_t)(crc >> 16);
  t[2] = (uint8_t)(crc >> 8);
  t[3] = (uint8_t)crc;
}
}  // namespace

int ufc_seal_host_slots(ufc_ctx* ctx, uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens, size_t n,
                        uint32_t* h_crc_scratch) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;  // (an empty batch: nothing to do, whatever the pointers)
  if (!h_slots || !h_lens || !h_crc_scratch) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (h_lens[i] < 4) return UFC_ERR_INVALID_ARG;
  // The gate computes crc = compute(frame[..len-4]) whatever the trailer holds: that is the seal.
  const int rc = ufc_validate_host_slots(ctx, h_slots, slot_stride, h_lens, n, h_crc_scratch, nullptr);
  if (rc != UFC_OK) return rc;
  for (size_t i = 0; i < n; i++) put_trailer(h_slots + i * slot_stride, h_lens[i], h_crc_scratch[i]);
  return UFC_OK;
}

int ufc_seal_host_varlen(ufc_ctx* ctx, uint8_t* h_bytes, const uint64_t* h_offsets, size_t n,
                         uint32_t* h_crc_scratch) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;  // (an empty batch: nothing to do, whatever the pointers)
  if (!h_bytes || !h_offsets || !h_crc_scratch) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (h_offsets[i + 1] < h_offsets[i] + 4) return UFC_ERR_INVALID_ARG;
  const int rc = ufc_validate_host_varlen(ctx, h_bytes, h_offsets, n, h_crc_scratch, nullptr);
  if (rc != UFC_OK) return rc;
  for (size_t i = 0; i < n; i++) put_trailer(h_bytes + h_offsets[i], (size_t)(h_offsets[i + 1] - h_offsets[i]), h_crc_scratch[i]);
  return UFC_OK;
}

int ufc_parse_batch_varlen(ufc_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                           const uint8_t* d_valid, ufc_frame_info* d_infos, ufc_item* d_items, size_t items_cap,
                           uint64_t* d_items_used, void* stream) {
  if (!ctx) return UFC_ERR_INVALID_ARG;
  if (n == 0) return UFC_OK;
  if (!d_bytes || !d_offsets || !d_valid || !d_infos || n >= ((size_t)1 << 31)) return UFC_ERR_INVALID_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e;
  const size_t need = ufc_dev::parse_scratch_bytes(n, d_items ? (uint64_t)items_cap : 0);
  void* scratch = nullptr;  // this stream's own scratch (grows on the first or a larger batch only)
  if ((e = stream_scratch(ctx, kScratchParse, (hipStream_t)stream, need, &scratch)) != hipSuccess)
    return hip_fail(ctx, e);
  ufc_dev::ParseArgs a{d_bytes, d_offsets, (uint64_t)n, d_valid, d_infos, d_items, (uint64_t)(d_items ? items_cap : 0),
                       d_items_used};
  if ((e = ufc_dev::parse_batch(a, scratch, need, (hipStream_t)stream)) != hipSuccess) return hip_fail(ctx, e);
  return UFC_OK;
}

}  // extern "C"
