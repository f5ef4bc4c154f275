// ufc_shard.cpp -- multi-GPU entry points of libuflowcrc.so (include/uflow_frame_crc.h, "multi-GPU"):
// a batch of frames shards by frame index over the ranks (one process per GPU), every rank runs the
// batched gate on its own shard, and the only exchange is gathering the per-frame CRC words and
// valid flags into global frame order on the root over RCCL (xGMI point-to-point).
//
// Reference caller: the receive loop src/server/mod.rs:591-602 (Frame::read of every datagram),
// here for a batch spread over the GPUs of one node (SURVEY.md section 8(b) last line, 8(e)).
//
// RCCL is bound at run time (dlopen of librccl.so.1): the single-GPU entry points need no RCCL, and
// a process that already holds an RCCL (torch's) shares that one instead of loading a second copy.
// The gather is grouped ncclSend / ncclRecv (every shard straight to its global position on the
// root, no padding, no repacking), issued per chunk of the shard so that the transfer of chunk c
// overlaps the gate of chunk c + 1 when the caller gives a separate gather stream.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>

#include "../../include/uflow_frame_crc.h"
#include "ufc_internal.hpp"

namespace {

struct Rccl {
  bool ok = false;
  char err[256] = {0};
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // An RCCL already in the process (e.g. torch's, same soname) first; else the system one.
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("librccl.so", RTLD_NOW);
    if (!h) {
      std::snprintf(r.err, sizeof r.err, "%s", dlerror());
      return;
    }
    auto sym = [&](const char* name) { return dlsym(h, name); };
    r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.Send && r.Recv && r.GroupStart && r.GroupEnd;
  });
  return r;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

constexpr int kMaxChunks = 16;
// A chunk of the gather pipeline holds at most ~2^22 frames: one launch of the lean fixed kernel
// (ncu * 8 waves * 511 sets * 4 frames = 4.19M frames on 256 CUs).
constexpr int kChunkFramesLog2 = 22;

}  // namespace

struct ufc_comm {
  ufc_ctx* ctx = nullptr;
  int nranks = 0;
  int rank = 0;
  ncclComm_t nccl = nullptr;
  int last_nccl_error = 0;
  hipEvent_t ev[kMaxChunks] = {};
};

namespace {

// Contiguous shard of `rank`: frames [n r / W, n (r + 1) / W) (sizes differ by at most one).
void shard_of(uint64_t n, int nranks, int rank, uint64_t* first, uint64_t* count) {
  const unsigned __int128 lo = (unsigned __int128)n * (unsigned)rank / (unsigned)nranks;
  const unsigned __int128 hi = (unsigned __int128)n * (unsigned)(rank + 1) / (unsigned)nranks;
  *first = (uint64_t)lo;
  *count = (uint64_t)(hi - lo);
}

// Chunks of a shard: the same function of (n_total, nranks) on every rank, so that the root knows
// every sender's chunk sizes.  Chunk c of a shard of `count` frames: [count c / K, count (c+1) / K).
int chunks_for(uint64_t n_total, int nranks) {
  const uint64_t per = (n_total + nranks - 1) / nranks;
  const uint64_t k = (per + (1ull << kChunkFramesLog2) - 1) >> kChunkFramesLog2;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(kMaxChunks, k));
}

int nccl_fail(ufc_comm* comm, ncclResult_t r) {
  comm->last_nccl_error = (int)r;
  return UFC_ERR_COMM;
}

}  // namespace

extern "C" {

int ufc_shard_range(uint64_t n_total, int nranks, int rank, uint64_t* first, uint64_t* count) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return UFC_ERR_INVALID_ARG;
  shard_of(n_total, nranks, rank, first, count);
  return UFC_OK;
}

int ufc_shard_chunk(uint64_t n_total, int nranks, int rank, int chunk, uint64_t* first, uint64_t* count) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return UFC_ERR_INVALID_ARG;
  const int K = chunks_for(n_total, nranks);
  if (chunk < 0 || chunk >= K) return UFC_ERR_INVALID_ARG;
  uint64_t lo, cnt;
  shard_of(n_total, nranks, rank, &lo, &cnt);
  const uint64_t a = cnt * (uint64_t)chunk / K, b = cnt * (uint64_t)(chunk + 1) / K;
  *first = lo + a;
  *count = b - a;
  return K;
}

int ufc_comm_id_create(uint8_t id[UFC_COMM_ID_BYTES]) {
  if (!id) return UFC_ERR_INVALID_ARG;
  const Rccl& r = rccl();
  if (!r.ok) return UFC_ERR_COMM;
  ncclUniqueId u;
  static_assert(sizeof(u) == UFC_COMM_ID_BYTES, "ncclUniqueId size");
  if (r.GetUniqueId(&u) != ncclSuccess) return UFC_ERR_COMM;
  std::memcpy(id, &u, sizeof u);
  return UFC_OK;
}

int ufc_comm_create(ufc_comm** out, ufc_ctx* ctx, int nranks, int rank, const uint8_t id[UFC_COMM_ID_BYTES]) {
  if (!out) return UFC_ERR_INVALID_ARG;
  *out = nullptr;
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return UFC_ERR_INVALID_ARG;
  const Rccl& r = rccl();
  if (!r.ok) return UFC_ERR_COMM;
  ufc_comm* c = new (std::nothrow) ufc_comm();
  if (!c) return UFC_ERR_NOMEM;
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  DeviceGuard g(ufc_internal::ctx_device(ctx));
  for (hipEvent_t& e : c->ev) {
    const hipError_t he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (he != hipSuccess) {
      ufc_internal::note_hip_error(ctx, (int)he);
      ufc_comm_destroy(c);
      return UFC_ERR_HIP;
    }
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  const ncclResult_t nr = r.CommInitRank(&c->nccl, nranks, u, rank);  // collective over the ranks
  if (nr != ncclSuccess) {
    c->nccl = nullptr;
    ufc_comm_destroy(c);
    return UFC_ERR_COMM;
  }
  *out = c;
  return UFC_OK;
}

int ufc_comm_destroy(ufc_comm* comm) {
  if (!comm) return UFC_OK;
  {
    DeviceGuard g(ufc_internal::ctx_device(comm->ctx));
    if (comm->nccl) (void)rccl().CommDestroy(comm->nccl);
    for (hipEvent_t& e : comm->ev)
      if (e) (void)hipEventDestroy(e);
  }
  delete comm;
  return UFC_OK;
}

int ufc_comm_last_error(const ufc_comm* comm) { return comm ? comm->last_nccl_error : 0; }

int ufc_crc_sharded(ufc_comm* comm, const uint8_t* d_frames, size_t stride, size_t frame_len, uint64_t n_total,
                    uint32_t* d_crc_out, uint8_t* d_valid_out, int root, void* stream, void* gather_stream) {
  if (!comm) return UFC_ERR_INVALID_ARG;
  if (root < 0 || root >= comm->nranks || stride < frame_len || (!d_crc_out && !d_valid_out))
    return UFC_ERR_INVALID_ARG;
  uint64_t lo, cnt;
  shard_of(n_total, comm->nranks, comm->rank, &lo, &cnt);
  if (cnt && !d_frames) return UFC_ERR_INVALID_ARG;
  const Rccl& r = rccl();
  hipStream_t s = (hipStream_t)stream;
  hipStream_t gs = gather_stream ? (hipStream_t)gather_stream : s;
  const bool is_root = comm->rank == root;
  DeviceGuard g(ufc_internal::ctx_device(comm->ctx));
  const int K = chunks_for(n_total, comm->nranks);
  // This rank's results: on the root straight into their global position, elsewhere at the start
  // of the caller's (shard-sized) output.
  uint32_t* my_crc = d_crc_out ? d_crc_out + (is_root ? lo : 0) : nullptr;
  uint8_t* my_valid = d_valid_out ? d_valid_out + (is_root ? lo : 0) : nullptr;
  for (int c = 0; c < K; c++) {
    const uint64_t a = cnt * (uint64_t)c / K, b = cnt * (uint64_t)(c + 1) / K;
    if (b > a) {
      const int rc = ufc_internal::crc_fixed(comm->ctx, d_frames + a * stride, stride, frame_len, b - a,
                                             my_crc ? my_crc + a : nullptr, my_valid ? my_valid + a : nullptr, s,
                                             c > 0);
      if (rc != UFC_OK) return rc;
    }
    if (comm->nranks == 1) continue;
    if (gs != s) {
      hipError_t e = hipEventRecord(comm->ev[c], s);
      if (e == hipSuccess) e = hipStreamWaitEvent(gs, comm->ev[c], 0);
      if (e != hipSuccess) {
        ufc_internal::note_hip_error(comm->ctx, (int)e);
        return UFC_ERR_HIP;
      }
    }
    ncclResult_t nr = r.GroupStart();
    if (nr != ncclSuccess) return nccl_fail(comm, nr);
    if (is_root) {
      for (int p = 0; p < comm->nranks; p++) {
        if (p == root) continue;
        uint64_t plo, pcnt;
        shard_of(n_total, comm->nranks, p, &plo, &pcnt);
        const uint64_t pa = pcnt * (uint64_t)c / K, pb = pcnt * (uint64_t)(c + 1) / K;
        if (pb == pa) continue;
        if (d_crc_out && (nr = r.Recv(d_crc_out + plo + pa, pb - pa, ncclUint32, p, comm->nccl, gs)) != ncclSuccess)
          break;
        if (d_valid_out && (nr = r.Recv(d_valid_out + plo + pa, pb - pa, ncclUint8, p, comm->nccl, gs)) != ncclSuccess)
          break;
      }
    } else if (b > a) {
      if (my_crc) nr = r.Send(my_crc + a, b - a, ncclUint32, root, comm->nccl, gs);
      if (nr == ncclSuccess && my_valid) nr = r.Send(my_valid + a, b - a, ncclUint8, root, comm->nccl, gs);
    }
    const ncclResult_t ne = r.GroupEnd();
    if (nr != ncclSuccess) return nccl_fail(comm, nr);
    if (ne != ncclSuccess) return nccl_fail(comm, ne);
  }
  return UFC_OK;
}

}  // extern "C"
