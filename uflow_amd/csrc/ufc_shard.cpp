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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>

#include "../../include/uflow_frame_crc.h"
#include "ufc_internal.hpp"

namespace {

struct Rccl {
  bool ok = false;
  char err[256] = {0};
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
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
    r.CommAbort = (decltype(r.CommAbort))sym("ncclCommAbort");
    r.CommSplit = (decltype(r.CommSplit))sym("ncclCommSplit");
    r.CommGetAsyncError = (decltype(r.CommGetAsyncError))sym("ncclCommGetAsyncError");
    r.AllReduce = (decltype(r.AllReduce))sym("ncclAllReduce");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.CommAbort && r.CommSplit && r.CommGetAsyncError &&
           r.AllReduce && r.Send && r.Recv && r.GroupStart && r.GroupEnd;
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

// How long a sharded call waits for every peer to join its status agreement (ufc_comm_set_timeout).
constexpr int kDefaultTimeoutMs = 60000;

struct ufc_comm {
  ufc_ctx* ctx = nullptr;
  int nranks = 0;
  int rank = 0;
  ncclComm_t nccl = nullptr;
  // Status agreement before every gather (agree_status): a second communicator split from the first,
  // so that its one-word all-reduce never queues behind the data communicator's transfers, on a
  // stream of its own; the word goes through pinned host memory.
  ncclComm_t ctl = nullptr;
  hipStream_t ctl_stream = nullptr;
  int32_t* d_status = nullptr;
  int32_t* h_status = nullptr;  // [0] this rank's status, [1] the agreed (max over ranks)
  int last_nccl_error = 0;
  bool broken = false;   // aborted after a rank-local failure mid-gather, or stalled: every later call fails
  bool stalled = false;  // a peer missed the status agreement's deadline: the all-reduce is still pending
  int timeout_ms = kDefaultTimeoutMs;  // the status agreement's deadline (0: wait for ever)
  hipEvent_t ev[kMaxChunks] = {};
};

namespace {

uint64_t mul_div(uint64_t a, uint64_t b, uint64_t c) { return (uint64_t)((unsigned __int128)a * b / c); }

// Contiguous shard of `rank`: frames [n r / W, n (r + 1) / W) (sizes differ by at most one).
void shard_of(uint64_t n, int nranks, int rank, uint64_t* first, uint64_t* count) {
  const uint64_t lo = mul_div(n, (unsigned)rank, (unsigned)nranks);
  const uint64_t hi = mul_div(n, (unsigned)(rank + 1), (unsigned)nranks);
  *first = lo;
  *count = hi - lo;
}

bool bounds_ok(const uint64_t* bounds, int nranks) {
  if (!bounds || nranks < 1 || nranks > UFC_MAX_RANKS || bounds[0] != 0) return false;
  for (int r = 0; r < nranks; r++)
    if (bounds[r + 1] < bounds[r]) return false;
  return true;
}

// Chunks per shard: the same function of the bounds on every rank, so that the root knows every
// sender's chunk sizes.
int nchunks_of(const uint64_t* bounds, int nranks) {
  uint64_t per = 0;
  for (int r = 0; r < nranks; r++) per = std::max(per, bounds[r + 1] - bounds[r]);
  const uint64_t k = (per >> kChunkFramesLog2) + ((per & ((1ull << kChunkFramesLog2) - 1)) ? 1 : 0);
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(kMaxChunks, k));
}

// The plan of one chunk (include/uflow_frame_crc.h, ufc_shard_gather_plan); returns the op count.
int plan_chunk(const uint64_t* bounds, int nranks, int rank, int root, int K, int c, ufc_xfer* ops, int max_ops) {
  int k = 0;
  auto push = [&](int op, int peer, uint64_t src, uint64_t dst, uint64_t count) {
    if (ops && k < max_ops) ops[k] = ufc_xfer{op, peer, src, dst, count};
    k++;
  };
  const uint64_t cnt = bounds[rank + 1] - bounds[rank];
  const uint64_t a = mul_div(cnt, (unsigned)c, (unsigned)K), b = mul_div(cnt, (unsigned)(c + 1), (unsigned)K);
  const bool is_root = rank == root;
  if (b > a) push(UFC_OP_GATE, rank, a, (is_root ? bounds[rank] : 0) + a, b - a);
  if (nranks == 1) return k;
  if (is_root) {
    for (int p = 0; p < nranks; p++) {
      if (p == root) continue;
      const uint64_t pc = bounds[p + 1] - bounds[p];
      const uint64_t pa = mul_div(pc, (unsigned)c, (unsigned)K), pb = mul_div(pc, (unsigned)(c + 1), (unsigned)K);
      if (pb > pa) push(UFC_OP_RECV, p, pa, bounds[p] + pa, pb - pa);
    }
  } else if (b > a) {
    push(UFC_OP_SEND, root, a, bounds[rank] + a, b - a);
  }
  return k;
}

int nccl_fail(ufc_comm* comm, ncclResult_t r) {
  comm->last_nccl_error = (int)r;
  return UFC_ERR_COMM;
}

// A failure only this rank sees, after the gather may have begun: abort the communicator so that no
// later call queues transfers the peers cannot match.
int abort_comm(ufc_comm* comm, int rc) {
  if (comm->nccl && !comm->broken) (void)rccl().CommAbort(comm->nccl);
  if (comm->ctl && !comm->broken) (void)rccl().CommAbort(comm->ctl);
  comm->nccl = nullptr;
  comm->ctl = nullptr;
  comm->broken = true;
  return rc;
}

// Every rank's verdict on its own arguments, agreed before any transfer is queued: a one-word
// max-all-reduce on the control communicator, read back through pinned memory.  A rank-local failure
// (a missing shard pointer) then fails the call on every rank -- UFC_ERR_PEER on the others -- and
// the communicator stays usable.  The host waits here for every peer to make the call (so every
// sharded call blocks its thread until then), polling the stream and the control communicator's
// asynchronous error, up to the communicator's deadline (ufc_comm_set_timeout).  A peer that has not
// joined by then fails the call with UFC_ERR_COMM and leaves the communicator stalled: nothing is
// aborted (ncclCommAbort measured not to return while the peer's side of the all-reduce is missing),
// the pending all-reduce and its buffers stay as they are, every later call returns UFC_ERR_COMM, the
// context records the stall (ufc_ctx_destroy then leaves the device memory to process exit), and the
// caller ends the process.
//
// Two rounds: the status all-reduce, then a one-word commit all-reduce.  A rank whose
// deadline passes in round 1 never enqueues round 2.  A peer that joins later completes round 1 against
// the stalled rank's pending all-reduce -- and would otherwise go on to queue its gather against a rank
// that is gone -- but its round 2 then finds no partner: it stalls at its own deadline and fails with
// UFC_ERR_COMM too.  So a late peer fails like the early one instead of hanging in its gather.  (Once
// every rank has finished round 1 they are all present; round 2 only misses its deadline on a rank if a
// peer dies in between.)
// UFC_SHARD_TRACE=1: progress of the status agreement on stderr (diagnosing a peer that never joins).
bool shard_trace() {
  static const bool on = [] {
    const char* t = std::getenv("UFC_SHARD_TRACE");
    return t && *t && *t != '0';
  }();
  return on;
}
#define UFC_TRACE(...)                                        \
  do {                                                        \
    if (shard_trace()) {                                      \
      std::fprintf(stderr, "[ufc_shard rank %d] ", comm->rank); \
      std::fprintf(stderr, __VA_ARGS__);                      \
      std::fprintf(stderr, "\n");                             \
      std::fflush(stderr);                                    \
    }                                                         \
  } while (0)

// Mark the communicator stalled (and its context: ufc_ctx_destroy must not wait for the device).
int stall(ufc_comm* comm) {
  comm->stalled = true;
  comm->broken = true;
  ufc_internal::note_stall(comm->ctx);
  return UFC_ERR_COMM;
}

// One round: word `in` of this rank -> max over the ranks into comm->h_status[1], waiting up to the
// deadline.  UFC_OK, or an error (the communicator aborted or stalled).
int ctl_round(ufc_comm* comm, int32_t in, int round) {
  const Rccl& r = rccl();
  comm->h_status[0] = in;
  comm->h_status[1] = -1;
  hipError_t e = hipMemcpyAsync(comm->d_status, comm->h_status, 4, hipMemcpyHostToDevice, comm->ctl_stream);
  if (e != hipSuccess) {
    ufc_internal::note_hip_error(comm->ctx, (int)e);
    return abort_comm(comm, UFC_ERR_HIP);
  }
  const ncclResult_t nr = r.AllReduce(comm->d_status, comm->d_status, 1, ncclInt32, ncclMax, comm->ctl,
                                      comm->ctl_stream);
  if (nr != ncclSuccess) return abort_comm(comm, nccl_fail(comm, nr));
  UFC_TRACE("agree_status: round %d all-reduce enqueued", round);
  if ((e = hipMemcpyAsync(comm->h_status + 1, comm->d_status, 4, hipMemcpyDeviceToHost, comm->ctl_stream)) !=
      hipSuccess) {
    ufc_internal::note_hip_error(comm->ctx, (int)e);
    return abort_comm(comm, UFC_ERR_HIP);
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; spin++) {
    e = hipStreamQuery(comm->ctl_stream);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) {
      ufc_internal::note_hip_error(comm->ctx, (int)e);
      return abort_comm(comm, UFC_ERR_HIP);
    }
    ncclResult_t ae = ncclSuccess;
    if (r.CommGetAsyncError(comm->ctl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
      return abort_comm(comm, nccl_fail(comm, ae));
    if (comm->timeout_ms > 0 && (spin & 63) == 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(comm->timeout_ms)) {
      if (hipStreamQuery(comm->ctl_stream) == hipSuccess) break;  // (done meanwhile)
      UFC_TRACE("agree_status: round %d, no answer from every peer in %d ms: stalled", round, comm->timeout_ms);
      return stall(comm);
    }
    if (spin > 1000) std::this_thread::sleep_for(std::chrono::microseconds(spin > 20000 ? 1000 : 20));
  }
  return UFC_OK;
}

int agree_status(ufc_comm* comm, int local_rc) {
  if (comm->nranks == 1) return local_rc;
  DeviceGuard g(ufc_internal::ctx_device(comm->ctx));  // (the control stream's device, whatever the caller's)
  UFC_TRACE("agree_status: local %d, enqueueing", local_rc);
  if (const int rc = ctl_round(comm, local_rc != UFC_OK ? 1 : 0, 1)) return rc;
  const int32_t agreed = comm->h_status[1];
  UFC_TRACE("agree_status: agreed %d", agreed);
  if (const int rc = ctl_round(comm, 0, 2)) return rc;  // commit: every rank got through round 1
  UFC_TRACE("agree_status: committed");
  if (local_rc != UFC_OK) return local_rc;
  return agreed != 0 ? UFC_ERR_PEER : UFC_OK;
}

// The gate of one chunk's frames, results into the rank's outputs at `dst`.
using GateFn = int (*)(const void* args, uint64_t src, uint64_t count, uint32_t* crc, uint8_t* valid,
                       hipStream_t s, bool front_ok);

struct FixedArgs {
  ufc_ctx* ctx;
  const uint8_t* frames;
  size_t stride, frame_len;
};
int gate_fixed(const void* p, uint64_t src, uint64_t count, uint32_t* crc, uint8_t* valid, hipStream_t s,
               bool front_ok) {
  const FixedArgs& a = *(const FixedArgs*)p;
  return ufc_internal::crc_fixed(a.ctx, a.frames + src * a.stride, a.stride, a.frame_len, count, crc, valid, s,
                                 front_ok);
}

struct VarlenArgs {
  ufc_ctx* ctx;
  const uint8_t* bytes;
  const uint64_t* offsets;
};
int gate_varlen(const void* p, uint64_t src, uint64_t count, uint32_t* crc, uint8_t* valid, hipStream_t s, bool) {
  const VarlenArgs& a = *(const VarlenArgs*)p;
  return ufc_crc_batch_varlen(a.ctx, a.bytes, a.offsets + src, count, crc, valid, (void*)s);
}

// The chunked gate + gather of one rank, executing ufc_shard_gather_plan chunk by chunk.
int run_sharded(ufc_comm* comm, const uint64_t* bounds, GateFn gate, const void* gargs, uint32_t* d_crc_out,
                uint8_t* d_valid_out, int root, hipStream_t s, hipStream_t gs) {
  const Rccl& r = rccl();
  const int W = comm->nranks;
  const int K = nchunks_of(bounds, W);
  DeviceGuard g(ufc_internal::ctx_device(comm->ctx));
  ufc_xfer ops[UFC_MAX_RANKS + 1];
  for (int c = 0; c < K; c++) {
    const int nops = plan_chunk(bounds, W, comm->rank, root, K, c, ops, UFC_MAX_RANKS + 1);
    bool xfer = false;
    for (int i = 0; i < nops; i++) {
      const ufc_xfer& o = ops[i];
      if (o.op != UFC_OP_GATE) {
        xfer = true;
        continue;
      }
      const int rc = gate(gargs, o.src, o.count, d_crc_out ? d_crc_out + o.dst : nullptr,
                          d_valid_out ? d_valid_out + o.dst : nullptr, s, c > 0);
      if (rc != UFC_OK) return W > 1 ? abort_comm(comm, rc) : rc;
    }
    if (!xfer) continue;  // (one rank, or nothing of this chunk to move)
    if (gs != s) {
      hipError_t e = hipEventRecord(comm->ev[c], s);
      if (e == hipSuccess) e = hipStreamWaitEvent(gs, comm->ev[c], 0);
      if (e != hipSuccess) {
        ufc_internal::note_hip_error(comm->ctx, (int)e);
        return abort_comm(comm, UFC_ERR_HIP);
      }
    }
    ncclResult_t nr = r.GroupStart();
    if (nr != ncclSuccess) return abort_comm(comm, nccl_fail(comm, nr));
    for (int i = 0; i < nops && nr == ncclSuccess; i++) {
      const ufc_xfer& o = ops[i];
      if (o.op == UFC_OP_SEND) {
        if (d_crc_out) nr = r.Send(d_crc_out + o.src, o.count, ncclUint32, o.peer, comm->nccl, gs);
        if (nr == ncclSuccess && d_valid_out)
          nr = r.Send(d_valid_out + o.src, o.count, ncclUint8, o.peer, comm->nccl, gs);
      } else if (o.op == UFC_OP_RECV) {
        if (d_crc_out) nr = r.Recv(d_crc_out + o.dst, o.count, ncclUint32, o.peer, comm->nccl, gs);
        if (nr == ncclSuccess && d_valid_out)
          nr = r.Recv(d_valid_out + o.dst, o.count, ncclUint8, o.peer, comm->nccl, gs);
      }
    }
    const ncclResult_t ne = r.GroupEnd();
    if (nr != ncclSuccess) return abort_comm(comm, nccl_fail(comm, nr));
    if (ne != ncclSuccess) return abort_comm(comm, nccl_fail(comm, ne));
  }
  return UFC_OK;
}

// Checks every rank makes alike (same arguments on every rank by contract): a failure here happens
// on every rank before any transfer.
int check_common(ufc_comm* comm, int root, bool any_out) {
  if (!comm) return UFC_ERR_INVALID_ARG;
  if (comm->broken) return UFC_ERR_COMM;
  if (root < 0 || root >= comm->nranks || !any_out) return UFC_ERR_INVALID_ARG;
  return UFC_OK;
}

}  // namespace

extern "C" {

int ufc_shard_range(uint64_t n_total, int nranks, int rank, uint64_t* first, uint64_t* count) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return UFC_ERR_INVALID_ARG;
  shard_of(n_total, nranks, rank, first, count);
  return UFC_OK;
}

int ufc_shard_bounds_fixed(uint64_t n_total, int nranks, uint64_t* bounds) {
  if (!bounds || nranks < 1 || nranks > UFC_MAX_RANKS) return UFC_ERR_INVALID_ARG;
  for (int r = 0; r <= nranks; r++) bounds[r] = mul_div(n_total, (unsigned)r, (unsigned)nranks);
  return UFC_OK;
}

int ufc_shard_bounds_varlen(const uint64_t* h_offsets, uint64_t n_total, int nranks, uint64_t* bounds) {
  if (!h_offsets || !bounds || nranks < 1 || nranks > UFC_MAX_RANKS) return UFC_ERR_INVALID_ARG;
  const uint64_t base = h_offsets[0];
  if (h_offsets[n_total] < base) return UFC_ERR_INVALID_ARG;
  const uint64_t B = h_offsets[n_total] - base;
  bounds[0] = 0;
  bounds[nranks] = n_total;
  for (int r = 1; r < nranks; r++) {
    // First frame starting at or past byte r B / W of the batch (lower_bound over offsets[0..n]).
    const uint64_t target = base + mul_div(B, (unsigned)r, (unsigned)nranks);
    const uint64_t* it = std::lower_bound(h_offsets, h_offsets + n_total + 1, target);
    bounds[r] = std::min<uint64_t>((uint64_t)(it - h_offsets), n_total);
    if (bounds[r] < bounds[r - 1]) return UFC_ERR_INVALID_ARG;  // offsets not sorted
  }
  return UFC_OK;
}

int ufc_shard_nchunks(const uint64_t* bounds, int nranks) {
  if (!bounds_ok(bounds, nranks)) return UFC_ERR_INVALID_ARG;
  return nchunks_of(bounds, nranks);
}

int ufc_shard_gather_plan(const uint64_t* bounds, int nranks, int rank, int root, int chunk, ufc_xfer* ops,
                          int max_ops) {
  if (!bounds_ok(bounds, nranks) || rank < 0 || rank >= nranks || root < 0 || root >= nranks || max_ops < 0 ||
      (max_ops > 0 && !ops))
    return UFC_ERR_INVALID_ARG;
  const int K = nchunks_of(bounds, nranks);
  if (chunk < 0 || chunk >= K) return UFC_ERR_INVALID_ARG;
  return plan_chunk(bounds, nranks, rank, root, K, chunk, ops, max_ops);
}

int ufc_shard_chunk(uint64_t n_total, int nranks, int rank, int chunk, uint64_t* first, uint64_t* count) {
  if (nranks < 1 || nranks > UFC_MAX_RANKS || rank < 0 || rank >= nranks || !first || !count)
    return UFC_ERR_INVALID_ARG;
  uint64_t bounds[UFC_MAX_RANKS + 1];
  (void)ufc_shard_bounds_fixed(n_total, nranks, bounds);
  const int K = nchunks_of(bounds, nranks);
  if (chunk < 0 || chunk >= K) return UFC_ERR_INVALID_ARG;
  const uint64_t cnt = bounds[rank + 1] - bounds[rank];
  const uint64_t a = mul_div(cnt, (unsigned)chunk, (unsigned)K), b = mul_div(cnt, (unsigned)(chunk + 1), (unsigned)K);
  *first = bounds[rank] + a;
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
  if (!ctx || !id || nranks < 1 || nranks > UFC_MAX_RANKS || rank < 0 || rank >= nranks) return UFC_ERR_INVALID_ARG;
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
  hipError_t he = hipStreamCreateWithFlags(&c->ctl_stream, hipStreamNonBlocking);
  if (he == hipSuccess) he = hipMalloc(&c->d_status, 4);
  if (he == hipSuccess) he = hipHostMalloc(&c->h_status, 8, hipHostMallocDefault);
  if (he != hipSuccess) {
    ufc_internal::note_hip_error(ctx, (int)he);
    ufc_comm_destroy(c);
    return UFC_ERR_HIP;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclResult_t nr = r.CommInitRank(&c->nccl, nranks, u, rank);  // collective over the ranks
  if (nr != ncclSuccess) {
    c->nccl = nullptr;
    c->last_nccl_error = (int)nr;
    ufc_comm_destroy(c);
    return UFC_ERR_COMM;
  }
  if ((nr = r.CommSplit(c->nccl, 0, rank, &c->ctl, nullptr)) != ncclSuccess) {  // collective too
    c->ctl = nullptr;
    c->last_nccl_error = (int)nr;
    ufc_comm_destroy(c);
    return UFC_ERR_COMM;
  }
  // Connect the control communicator now, while every rank is here: RCCL sets a communicator's
  // connections up at its first collective, inside the enqueueing call (blocking the host until the
  // peers join), so the first sharded call would otherwise pay for it.
  if (nranks > 1) {
    c->h_status[0] = 0;
    he = hipMemcpyAsync(c->d_status, c->h_status, 4, hipMemcpyHostToDevice, c->ctl_stream);
    if (he == hipSuccess) {
      if ((nr = r.AllReduce(c->d_status, c->d_status, 1, ncclInt32, ncclMax, c->ctl, c->ctl_stream)) != ncclSuccess) {
        c->last_nccl_error = (int)nr;
        ufc_comm_destroy(c);
        return UFC_ERR_COMM;
      }
      he = hipStreamSynchronize(c->ctl_stream);
    }
    if (he != hipSuccess) {
      ufc_internal::note_hip_error(ctx, (int)he);
      ufc_comm_destroy(c);
      return UFC_ERR_HIP;
    }
  }
  *out = c;
  return UFC_OK;
}

int ufc_comm_destroy(ufc_comm* comm) {
  if (!comm) return UFC_OK;
  if (comm->stalled) {
    // The status all-reduce is still pending on the control stream (a peer never joined): destroying
    // the communicators, the stream or the status words could wait for it or free what it writes.
    // Everything is left to process exit; the handle is gone.
    delete comm;
    return UFC_ERR_COMM;
  }
  {
    DeviceGuard g(ufc_internal::ctx_device(comm->ctx));
    if (comm->ctl) (void)rccl().CommDestroy(comm->ctl);
    if (comm->nccl) (void)rccl().CommDestroy(comm->nccl);
    for (hipEvent_t& e : comm->ev)
      if (e) (void)hipEventDestroy(e);
    if (comm->ctl_stream) (void)hipStreamDestroy(comm->ctl_stream);
    if (comm->d_status) (void)hipFree(comm->d_status);
    if (comm->h_status) (void)hipHostFree(comm->h_status);
  }
  delete comm;
  return UFC_OK;
}

int ufc_comm_set_timeout(ufc_comm* comm, int timeout_ms) {
  if (!comm || timeout_ms < 0) return UFC_ERR_INVALID_ARG;
  comm->timeout_ms = timeout_ms;
  return UFC_OK;
}

int ufc_comm_last_error(const ufc_comm* comm) { return comm ? comm->last_nccl_error : 0; }


int ufc_crc_sharded(ufc_comm* comm, const uint8_t* d_frames, size_t stride, size_t frame_len, uint64_t n_total,
                    uint32_t* d_crc_out, uint8_t* d_valid_out, int root, void* stream, void* gather_stream) {
  if (const int rc = check_common(comm, root, d_crc_out || d_valid_out)) return rc;
  if (stride < frame_len || frame_len > ufc_internal::kMaxFrameLen) return UFC_ERR_INVALID_ARG;
  uint64_t bounds[UFC_MAX_RANKS + 1];
  (void)ufc_shard_bounds_fixed(n_total, comm->nranks, bounds);
  const uint64_t cnt = bounds[comm->rank + 1] - bounds[comm->rank];
  // Rank-local: this rank's frames.  Agreed with the peers before any transfer, so the call fails on
  // every rank (UFC_ERR_PEER on the others) and nothing is left queued.
  if (const int rc = agree_status(comm, cnt && !d_frames ? UFC_ERR_INVALID_ARG : UFC_OK)) return rc;
  const FixedArgs args{comm->ctx, d_frames, stride, frame_len};
  hipStream_t s = (hipStream_t)stream;
  return run_sharded(comm, bounds, gate_fixed, &args, d_crc_out, d_valid_out, root, s,
                     gather_stream ? (hipStream_t)gather_stream : s);
}

int ufc_crc_sharded_varlen(ufc_comm* comm, const uint8_t* d_bytes, const uint64_t* d_offsets, const uint64_t* bounds,
                           uint32_t* d_crc_out, uint8_t* d_valid_out, int root, void* stream, void* gather_stream) {
  if (const int rc = check_common(comm, root, d_crc_out || d_valid_out)) return rc;
  if (!bounds_ok(bounds, comm->nranks)) return UFC_ERR_INVALID_ARG;
  const uint64_t cnt = bounds[comm->rank + 1] - bounds[comm->rank];
  if (const int rc = agree_status(comm, cnt && (!d_bytes || !d_offsets) ? UFC_ERR_INVALID_ARG : UFC_OK)) return rc;
  const VarlenArgs args{comm->ctx, d_bytes, d_offsets};
  hipStream_t s = (hipStream_t)stream;
  return run_sharded(comm, bounds, gate_varlen, &args, d_crc_out, d_valid_out, root, s,
                     gather_stream ? (hipStream_t)gather_stream : s);
}

}  // extern "C"
