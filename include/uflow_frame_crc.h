/*
 * uflow_frame_crc.h -- C ABI of libuflowcrc.so, the MI355X-native drop-in for uflow's
 * per-frame CRC-32 (polynomial 0x132c00699, reflected 0x9960034C) in src/frame.
 *
 * Reference (lowquark/uflow v0.7.1, Rust) interfaces each entry point replaces:
 *   ufc_crc32_compute      <- src/frame/serial/crc.rs:102-104  `pub fn compute(data: &[u8]) -> u32`
 *   ufc_crc32_extend       <- src/frame/serial/crc.rs:94-100   `pub fn extend(initial_crc: u32, data: &[u8]) -> u32`
 *   ufc_frame_validate     <- src/frame/serial/mod.rs:675-690  the CRC gate of `Frame::read`
 *   ufc_frame_seal         <- src/frame/serial/mod.rs:463-470 (every fixed-size write_*) and
 *                             src/frame/serial/build.rs:151-159 (DataFrameBuilder/AckFrameBuilder::build)
 *   ufc_crc_batch_fixed /  <- many calls of the gate above, one per received datagram
 *   ufc_crc_batch_varlen      (src/server/mod.rs:597-601, src/client/mod.rs:618-622), batched on the GPU
 *   ufc_seal_batch_fixed / <- many calls of the seal above, one per emitted frame
 *   ufc_seal_batch_varlen     (src/half_connection/emit.rs:114-125, 205-211), batched on the GPU
 *   ufc_crc_batch_pairs       the gate over frames given as (start, end) pairs (any gapped layout)
 *   ufc_validate_host_varlen  the same gate for frames that start and end in host memory
 *   ufc_validate_host_slots   (a UDP receive buffer): H2D copy + GPU CRC + D2H copy; _slots takes the
 *                             recvmmsg layout (fixed-size slots + lengths) of the receive loops
 *   ufc_seal_host_slots /     a flush's frames sealed in one batch before sendmmsg (the builders'
 *   ufc_seal_host_varlen      build(), build.rs:151-159, for every frame of half_connection/emit.rs)
 *   ufc_crc_sharded           the gate over a batch sharded across the GPUs of a node (one process
 *                             per GPU), CRC words + valid flags gathered to a root over RCCL
 *
 * Conventions (mirroring the reference):
 *   - All buffers are caller-owned; nothing is retained after a call returns (device calls:
 *     after the work queued on `stream` completes).
 *   - A CRC mismatch is data (valid = 0), never an error -- exactly like `Frame::read`
 *     returning None.  Errors are negative return codes for invalid arguments or HIP failures.
 *   - Batch semantics per frame i of length len_i:
 *         crc_out[i]   = compute(frame_i[0 .. len_i-4])      (compute(frame_i) when len_i < 4)
 *         valid_out[i] = len_i >= 5 && crc_out[i] == BE32(frame_i[len_i-4 .. len_i])
 *     and the seal writes BE32(compute(frame_i[0 .. len_i-4])) into frame_i[len_i-4 .. len_i].
 *   - An empty batch (n = 0) is nothing to do: every batch entry point returns UFC_OK for it with
 *     a valid context, whatever its buffer pointers (an empty Vec's may be dangling or NULL).
 *   - Device entry points are asynchronous on `stream` (a hipStream_t, or NULL for the null
 *     stream), allocate nothing per call, and never fall back to the CPU: without a usable
 *     MI355X (gfx950) device ufc_ctx_create fails with UFC_ERR_NO_DEVICE.
 *   - One ufc_ctx per device.  Device launches on different streams of one context are safe while
 *     fewer than 64 are in flight (each takes a claim-counter slot); device scratch (batch parse,
 *     sorted varlen mode, the CRC words of a fixed seal called without d_crc_out) is kept per
 *     stream and grows only on a stream's first or a larger batch.  The host-buffer calls (ufc_validate_host_*,
 *     ufc_seal_host_*) use the context's own streams and staging, one host thread at a time per
 *     context; they are synchronous and, on error too, return only once no copy touches the
 *     caller's buffers.  The scalar host functions are reentrant.
 */
#ifndef UFLOW_FRAME_CRC_H
#define UFLOW_FRAME_CRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UFC_OK 0
#define UFC_ERR_INVALID_ARG (-1)
#define UFC_ERR_NO_DEVICE (-2)
#define UFC_ERR_HIP (-3)
#define UFC_ERR_NOMEM (-4)
#define UFC_ERR_COMM (-5) /* RCCL missing or failed (multi-GPU entry points; see ufc_comm_last_error) */
#define UFC_ERR_PEER (-6) /* multi-GPU: another rank rejected its part of this call; nothing was transferred */

/* Frame constants from the reference (src/frame/serial/mod.rs:11-13, src/lib.rs:286-294). */
#define UFC_FRAME_CRC_SIZE 4
#define UFC_FRAME_OVERHEAD 5
#define UFC_MAX_FRAME_SIZE 1472

/* ---- scalar host entry points (bit-exact with crc.rs; drop-in for the Rust functions) ---- */
uint32_t ufc_crc32_compute(const uint8_t* data, size_t len);
uint32_t ufc_crc32_extend(uint32_t initial_crc, const uint8_t* data, size_t len);
/* 1 if the frame passes Frame::read's length + CRC gate, 0 if Frame::read would return None there. */
int ufc_frame_validate(const uint8_t* frame, size_t len);
/* Writes BE32(compute(frame[..len-4])) into frame[len-4..len]; UFC_ERR_INVALID_ARG if len < 4. */
int ufc_frame_seal(uint8_t* frame, size_t len);

/* ---- device context ---- */
typedef struct ufc_ctx ufc_ctx;
int ufc_device_count(void);
int ufc_ctx_create(ufc_ctx** out, int device);
/* UFC_OK; UFC_ERR_COMM when a communicator created on this context stalled (ufc_comm_set_timeout):
 * its RCCL all-reduce stays pending on the device, so the context's device memory and streams are
 * left to process exit (freeing them would wait for the device for ever); the handle is freed. */
int ufc_ctx_destroy(ufc_ctx* ctx);
/* Device scratch is kept per (context, stream) and grows only (batch parse: 14 B per frame + 2 B per
 * header slot, min(64 n, items_cap) slots; fixed seal without d_crc_out: 4 B per frame; asynchronous
 * host slots: the batch's slot bytes + 13 B per datagram; variable-length gates and seals: the list of
 * frames over 13 lines (1532 B) handed to their second launch, 4 B per frame of the largest launch
 * (< 2^29 frames) + 256 B, and 4 B per CU of counts).  A caller that retires a stream releases its scratch
 * here, BEFORE destroying the stream: waits for the work queued on it, then frees its buffers. */
int ufc_ctx_release_stream(ufc_ctx* ctx, void* stream);
const char* ufc_error_string(int code);
/* Last HIP error code seen by this context (0 if none). */
int ufc_ctx_last_hip_error(const ufc_ctx* ctx);

/* Kernel-selection options of a context (A/B measurement and tests; the defaults are the measured
 * fastest).  Results never depend on them.  Set between calls, not while work is queued.  Values
 * marked (removed) name kernels of earlier rounds that were measured slower and deleted;
 * ufc_ctx_set_option rejects them (UFC_ERR_INVALID_ARG).  Numbers are never reused. */
#define UFC_OPT_FIXED_KERNEL 0   /* fixed-stride batches: */
#define UFC_FIXED_AUTO 0         /*   lean kernel when eligible (default) */
#define UFC_FIXED_GENERIC 1      /*   the generic kernel */
#define UFC_FIXED_CLAIM16 2      /*   (removed) lean kernel, claimed schedule at 16 waves (round-1 default) */
#define UFC_OPT_VARLEN_KERNEL 1  /* CSR / pairs batches: */
#define UFC_VARLEN_AUTO 0        /*   the default: UFC_VARLEN_SORTED8 */
#define UFC_VARLEN_GENERIC 1     /*   the generic kernel (CSR only; pairs take the default) */
#define UFC_VARLEN_SORTED 2      /*   (removed) round-1 kernel on frames sorted by block count within runs of 64 */
#define UFC_VARLEN_BLOCKED8 3    /*   (removed) round-1 kernel, static blocked schedule at 8 waves */
#define UFC_VARLEN_CLAIM16 4     /*   (removed) round-1 kernel, claimed sets at 16 waves (round-1 default) */
#define UFC_VARLEN_BLOCKSTREAM 5 /*   (removed) the block-stream kernel */
#define UFC_VARLEN_SORTED8 6     /*   runs of 64 sorted in the kernel, 8-frame sets of 8 lanes per frame */
#define UFC_VARLEN_STREAM 7      /*   (removed) the byte-balanced stream kernel */
#define UFC_OPT_GENERIC_JC 2     /* 0 = auto, else 1..6: blocks per pipelined part of the generic kernel */
#define UFC_OPT_SEAL_KERNEL 3    /* fixed-stride seals: */
#define UFC_SEAL_INLINE 0        /*   the CRC kernel writes each workgroup's trailers after its reads (default; the
                                  *   numbers of round 4's header, kept: ufc_ctx_create sets the default explicitly) */
#define UFC_SEAL_TWO_PASS 1      /*   validate kernel's CRC words, then a non-temporal trailer pass (the round-3 default) */
#define UFC_OPT_COUNT_ 4
int ufc_ctx_set_option(ufc_ctx* ctx, int option, int value);
int ufc_ctx_get_option(const ufc_ctx* ctx, int option);

/* ---- batched, device-resident ---- */
/* Frame i occupies d_frames[i*stride .. i*stride + frame_len); stride >= frame_len.
 * d_crc_out (n words) and d_valid_out (n bytes) are each nullable, not both. */
int ufc_crc_batch_fixed(ufc_ctx* ctx, const uint8_t* d_frames, size_t stride, size_t frame_len, size_t n,
                        uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream);
/* Frame i occupies d_bytes[d_offsets[i] .. d_offsets[i+1]) (CSR, n+1 offsets, nondecreasing). */
int ufc_crc_batch_varlen(ufc_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                         uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream);
/* In-place seal of every frame (frame_len >= 4); d_crc_out nullable.  Fixed stride: one kernel whose
 * workgroups write their trailers after their reads (UFC_SEAL_INLINE, default), or two (the CRC words,
 * then every trailer with non-temporal stores: UFC_SEAL_TWO_PASS); UFC_OPT_SEAL_KERNEL. */
int ufc_seal_batch_fixed(ufc_ctx* ctx, uint8_t* d_frames, size_t stride, size_t frame_len, size_t n,
                         uint32_t* d_crc_out, void* stream);
int ufc_seal_batch_varlen(ufc_ctx* ctx, uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                          uint32_t* d_crc_out, void* stream);

/* Frame i occupies d_bytes[d_pairs[2i] .. d_pairs[2i+1]) (start <= end <= bytes_len): any
 * gapped layout, e.g. datagrams received into fixed-size slots.  Validate only. */
int ufc_crc_batch_pairs(ufc_ctx* ctx, const uint8_t* d_bytes, size_t bytes_len, const uint64_t* d_pairs, size_t n,
                        uint32_t* d_crc_out, uint8_t* d_valid_out, void* stream);

/* Measurement context, not part of the CRC path: reads the first
 * floor(bytes / 1024) KiB of d_buf as one plain contiguous stream (the access pattern an HBM read
 * bandwidth ceiling is measured with) and XORs the data into *d_sink.  *bytes_read receives the byte
 * count read.  bench.py times it beside the gate and reports roofline.ceiling_GBs. */
int ufc_hbm_read_probe(ufc_ctx* ctx, const uint8_t* d_buf, size_t bytes, uint32_t* d_sink, size_t* bytes_read,
                       void* stream);

/* ---- host buffers in, host buffers out (the receive path of SURVEY.md config 5) ----
 * Copies the frames through pinned staging buffers owned by the context, runs the batched
 * gate on the device and copies crc/valid back; synchronous.  h_offsets as above. */
int ufc_validate_host_varlen(ufc_ctx* ctx, const uint8_t* h_bytes, const uint64_t* h_offsets, size_t n,
                             uint32_t* h_crc_out, uint8_t* h_valid_out);
/* The batched receive loop's layout: datagram i was received (recvmmsg) into the slot
 * h_slots[i*slot_stride ..] and is h_lens[i] <= slot_stride bytes long.  Same staging as above;
 * no host-side compaction. */
int ufc_validate_host_slots(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens,
                            size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out);
/* Asynchronous form for a receive loop that overlaps its next recvmmsg with this batch's gate
 * (src/server/mod.rs:591-602): the H2D copies of the slots and lengths, the kernel and the D2H
 * copies are queued on `stream` (a hipStream_t, not NULL) and the call returns.  The four host
 * buffers must stay valid, the slots and lengths unmodified, until that work has completed
 * (hipStreamSynchronize or an event); pinned memory (hipHostMalloc) keeps the copies asynchronous.
 * Device staging is per (context, stream): batches on different streams may be in flight at once,
 * from different threads (one host thread per stream).  n * slot_stride < 2^31 - 2^20. */
int ufc_validate_host_slots_async(ufc_ctx* ctx, const uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens,
                                  size_t n, uint32_t* h_crc_out, uint8_t* h_valid_out, void* stream);
/* The send side (a flush's frames laid out by the builders with zero trailers):
 * CRC of every frame on the GPU (H2D of the frames, D2H of 4 B per frame), then the BE32 trailers
 * are written into the host buffer.  h_crc_scratch: n words (receives the CRCs).  Lengths >= 4. */
int ufc_seal_host_slots(ufc_ctx* ctx, uint8_t* h_slots, size_t slot_stride, const uint32_t* h_lens, size_t n,
                        uint32_t* h_crc_scratch);
int ufc_seal_host_varlen(ufc_ctx* ctx, uint8_t* h_bytes, const uint64_t* h_offsets, size_t n, uint32_t* h_crc_scratch);

/* ---- multi-GPU: one process per GPU, frames sharded by index, RCCL gather to a root ----
 * Replaces, for a batch spread over the GPUs of one node, the receive loop's per-datagram gate
 * (src/server/mod.rs:591-602 -> Frame::read, serial/mod.rs:675-690).  Rank r owns the frames
 * [bounds[r], bounds[r+1]) of a batch of n_total frames:
 *   fixed length     ufc_shard_bounds_fixed: [n_total r / nranks, n_total (r+1) / nranks)
 *   variable length  ufc_shard_bounds_varlen: split by bytes, a binary search of r * bytes / nranks
 *                    in the batch's offsets.
 * The only exchange is the per-frame CRC word and valid flag of every frame, gathered into global
 * frame order on the root over RCCL (xGMI point-to-point).  RCCL is loaded at run time
 * (librccl.so.1); without it the comm calls return UFC_ERR_COMM. */
#define UFC_COMM_ID_BYTES 128
#define UFC_MAX_RANKS 64
typedef struct ufc_comm ufc_comm;
int ufc_shard_range(uint64_t n_total, int nranks, int rank, uint64_t* first, uint64_t* count);
/* The gather pipeline's chunk `chunk` of rank `rank`'s shard: global frames [*first, *first + *count).
 * Returns the number of chunks every shard of the batch is split into (1..16: one per <= 2^22 frames
 * of a shard), or UFC_ERR_INVALID_ARG. */
int ufc_shard_chunk(uint64_t n_total, int nranks, int rank, int chunk, uint64_t* first, uint64_t* count);
/* Shard boundaries, bounds[0 .. nranks] (bounds[0] = 0, bounds[nranks] = n_total, nondecreasing).
 * _varlen: h_offsets[0 .. n_total] of the whole CSR batch (nondecreasing); bounds[r] = the first
 * frame i with h_offsets[i] - h_offsets[0] >= r * B / nranks, B = h_offsets[n_total] - h_offsets[0]. */
int ufc_shard_bounds_fixed(uint64_t n_total, int nranks, uint64_t* bounds);
int ufc_shard_bounds_varlen(const uint64_t* h_offsets, uint64_t n_total, int nranks, uint64_t* bounds);
/* The gather schedule, a pure function of (bounds, rank, root): the same on every rank, no device.
 * Every shard is split into the same number of chunks K = ufc_shard_nchunks(bounds, nranks) (1..16,
 * one per <= 2^22 frames of the largest shard); chunk c of a shard of `cnt` frames is its local frames
 * [cnt c / K, cnt (c+1) / K).  Per chunk, in order, a rank performs its plan's operations:
 *   UFC_OP_GATE  the batched gate over its local frames [src, src + count), results into its own
 *                outputs at [dst, dst + count) (the root: global positions; others: shard-local)
 *   UFC_OP_SEND  (non-root) its outputs [src, src + count) to `peer` (= root), landing at global dst
 *   UFC_OP_RECV  (root) `peer`'s outputs [src, src + count) into its own outputs [dst, dst + count)
 * All SEND/RECV of one chunk form one RCCL group.  Returns the number of operations of chunk `chunk`
 * (writing at most max_ops of them; ops may be NULL to query), or UFC_ERR_INVALID_ARG. */
#define UFC_OP_GATE 0
#define UFC_OP_SEND 1
#define UFC_OP_RECV 2
typedef struct ufc_xfer {
  int32_t op;
  int32_t peer;
  uint64_t src;
  uint64_t dst;
  uint64_t count;
} ufc_xfer;
int ufc_shard_nchunks(const uint64_t* bounds, int nranks);
int ufc_shard_gather_plan(const uint64_t* bounds, int nranks, int rank, int root, int chunk, ufc_xfer* ops,
                          int max_ops);
/* On one rank: a fresh communicator id (ncclGetUniqueId), handed to every rank out of band. */
int ufc_comm_id_create(uint8_t id[UFC_COMM_ID_BYTES]);
/* Collective over the nranks processes (one per GPU, each with its own ufc_ctx). */
int ufc_comm_create(ufc_comm** out, ufc_ctx* ctx, int nranks, int rank, const uint8_t id[UFC_COMM_ID_BYTES]);
/* UFC_ERR_COMM for a stalled communicator (see ufc_comm_set_timeout): its RCCL state is left to
 * process exit, the handle is freed. */
int ufc_comm_destroy(ufc_comm* comm);
/* How long a sharded call waits for every peer to join it (its status agreement, see ufc_crc_sharded),
 * in ms; 0 = for ever; default 60000.  Replaces the caller-side supervision a plain RCCL collective
 * needs (server/mod.rs:591-602's loop cannot wait for ever on a dead peer). */
int ufc_comm_set_timeout(ufc_comm* comm, int timeout_ms);
/* Last RCCL result code seen by this communicator (0 if none). */
int ufc_comm_last_error(const ufc_comm* comm);
/* Collective: the batched gate on this rank's shard, then the gather to `root`.
 *   d_frames     this rank's shard (frame k of the shard at d_frames + k * stride, stride >= frame_len)
 *   d_crc_out    root: n_total words in global frame order; other ranks: their shard's words
 *   d_valid_out  likewise, bytes; either output may be NULL, identically on every rank
 *   stream       the gate runs here (the root's own shard is complete when it is)
 *   gather_stream  the RCCL transfers run here, each chunk of the shard after its gate, so that the
 *                transfer of one chunk overlaps the gate of the next; NULL = `stream`.  The root's
 *                output is complete once both streams are; a sender's output may be rewritten
 *                once gather_stream has passed this call.
 * One host thread per communicator at a time; every rank must make the same calls in the same
 * order with the same n_total, stride, frame_len, root and output nullness.  Arguments that every
 * rank sees alike are checked before any transfer, so a bad call fails on every rank.  Arguments
 * only this rank can check (its shard pointers) are agreed before any transfer with a one-word
 * all-reduce on a second communicator: a rank that rejects its part returns UFC_ERR_INVALID_ARG,
 * every other rank UFC_ERR_PEER, nothing is queued and the communicator stays usable.  That
 * agreement blocks the calling host thread until every peer has made the call: a sharded call is
 * asynchronous on `stream` only from then on.  A peer that has not made it within the communicator's
 * deadline (ufc_comm_set_timeout; crashed, or calling something else) fails the call with
 * UFC_ERR_COMM without aborting anything (ncclCommAbort measured not to return while the peer has not
 * joined, on the socket transport): the communicator is then stalled, every later call returns
 * UFC_ERR_COMM, and the caller should end the process with an error.  The agreement takes two rounds
 * (status, then commit), so a peer that makes the call after the deadline has passed on another rank
 * fails with UFC_ERR_COMM at its own deadline too, instead of queueing a gather nobody answers.  A failure that only this rank
 * sees after the gather has begun (a HIP launch error) aborts the communicator (ncclCommAbort) and
 * marks it unusable (later calls return UFC_ERR_COMM): the peers' transfers then fail or stall, and
 * the caller must tear down every rank's communicator. */
int ufc_crc_sharded(ufc_comm* comm, const uint8_t* d_frames, size_t stride, size_t frame_len, uint64_t n_total,
                    uint32_t* d_crc_out, uint8_t* d_valid_out, int root, void* stream, void* gather_stream);
/* Variable-length form: rank r's shard is the frames [bounds[r], bounds[r+1]) (ufc_shard_bounds_varlen
 * of the whole batch, the same array on every rank), given as a CSR batch of its own: frame k of the
 * shard occupies d_bytes[d_offsets[k] .. d_offsets[k+1]), k < bounds[r+1] - bounds[r] (offsets relative
 * to d_bytes, e.g. the batch's offsets minus the shard's first offset).  Outputs, streams and error
 * behaviour as ufc_crc_sharded. */
int ufc_crc_sharded_varlen(ufc_comm* comm, const uint8_t* d_bytes, const uint64_t* d_offsets, const uint64_t* bounds,
                           uint32_t* d_crc_out, uint8_t* d_valid_out, int root, void* stream, void* gather_stream);

#ifdef __cplusplus
}
#endif

#endif /* UFLOW_FRAME_CRC_H */
