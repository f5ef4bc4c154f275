/*
 * oracle/crc_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of uflow's frame CRC (reference crate `uflow` v0.7.1, Rust),
 * used as the parity checker for the HIP path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product (libuflowcrc.so)
 * never links, calls or falls back to it.
 *
 * The reference is Rust and cannot be compiled in this image (no cargo/rustc), so there
 * is no oracle/_ref build.  Parity is pinned instead by the reference's own data:
 *   - the 256-entry PARTIAL_RESULTS table literal (src/frame/serial/crc.rs:59-92), which
 *     tests/golden/partial_results.json holds and which this file regenerates from the
 *     polynomial and compares (ufo_table_matches);
 *   - the known-answer test crc("123456789") == 0x11A6F2A3 (crc.rs:135-138);
 *   - crc([0]) != 0 (crc.rs:130-132) and table == bit-serial for any init (crc.rs:141-147).
 *
 * Function-by-function citations are given at each definition.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#define UFO_POLY_REFLECTED 0x9960034Cu /* crc.rs:50 (0x132c00699 bit-reversed, x^32 dropped) */

/* crc.rs:44-57  `fn extend_slow(initial_crc, data)` -- the bit-serial definition. */
uint32_t ufo_extend_slow(uint32_t initial_crc, const uint8_t* data, size_t len) {
  uint32_t reg = ~initial_crc;
  for (size_t i = 0; i < len; i++) {
    reg ^= (uint32_t)data[i];
    for (int b = 0; b < 8; b++) reg = (reg & 1u) ? (reg >> 1) ^ UFO_POLY_REFLECTED : (reg >> 1);
  }
  return ~reg;
}

static uint32_t g_table[256];
static int g_table_ready = 0;

/* crc.rs:59-92 `static PARTIAL_RESULTS: [u32; 256]` -- entry i == extend_slow(0, [i])
 * (the commented-out generator at crc.rs:111-126 prints exactly this). */
void ufo_table(uint32_t out[256]) {
  for (int i = 0; i < 256; i++) {
    uint8_t b = (uint8_t)i;
    out[i] = ufo_extend_slow(0, &b, 1);
  }
}

static void ensure_table(void) {
  if (!g_table_ready) { ufo_table(g_table); g_table_ready = 1; }
}

/* Returns 1 iff the regenerated table equals the 256 literals passed in
 * (the fixture copy of crc.rs:59-92). */
int ufo_table_matches(const uint32_t lit[256]) {
  ensure_table();
  for (int i = 0; i < 256; i++) if (g_table[i] != lit[i]) return 0;
  return 1;
}

/* crc.rs:94-100 `pub fn extend(initial_crc, data)`:
 *   for byte: crc = (crc >> 8) ^ PARTIAL_RESULTS[(crc as u8 ^ byte) as usize]           */
uint32_t ufo_extend(uint32_t initial_crc, const uint8_t* data, size_t len) {
  ensure_table();
  uint32_t crc = initial_crc;
  for (size_t i = 0; i < len; i++) crc = (crc >> 8) ^ g_table[(uint8_t)((uint8_t)crc ^ data[i])];
  return crc;
}

/* crc.rs:102-104 `pub fn compute(data) = extend(INITIAL_CRC, data)`, INITIAL_CRC = 0 (crc.rs:41). */
uint32_t ufo_compute(const uint8_t* data, size_t len) { return ufo_extend(0u, data, len); }

/* src/frame/serial/mod.rs:675-690 -- the CRC gate of `Frame::read`:
 *   len < 5 -> None; crc = BE32(frame[len-4..len]); compute(frame[..len-4]) != crc -> None.
 * Returns 1 when the frame passes the gate, 0 when Frame::read would return None there.
 * *crc_out (nullable) receives compute(frame[..len-4]) (or compute(frame) when len < 4). */
int ufo_frame_validate(const uint8_t* frame, size_t len, uint32_t* crc_out) {
  uint32_t c;
  if (len < 4) {
    c = ufo_compute(frame, len);
    if (crc_out) *crc_out = c;
    return 0;
  }
  c = ufo_compute(frame, len - 4);
  if (crc_out) *crc_out = c;
  if (len < 5) return 0;
  uint32_t rx = ((uint32_t)frame[len - 4] << 24) | ((uint32_t)frame[len - 3] << 16) |
                ((uint32_t)frame[len - 2] << 8) | (uint32_t)frame[len - 1];
  return c == rx ? 1 : 0;
}

/* src/frame/serial/mod.rs:463-470 (every fixed-size write_*) and build.rs:151-159:
 * crc = compute(frame[..len-4]); frame[len-4..len] = crc big-endian.  len >= 4. */
uint32_t ufo_frame_seal(uint8_t* frame, size_t len) {
  if (len < 4) return 0;
  uint32_t c = ufo_compute(frame, len - 4);
  frame[len - 4] = (uint8_t)(c >> 24);
  frame[len - 3] = (uint8_t)(c >> 16);
  frame[len - 2] = (uint8_t)(c >> 8);
  frame[len - 1] = (uint8_t)c;
  return c;
}

/* Batched forms of the two functions above (the same per-frame semantics, looped). */
void ufo_validate_fixed(const uint8_t* frames, size_t stride, size_t frame_len, size_t n,
                        uint32_t* crc_out, uint8_t* valid_out) {
  for (size_t i = 0; i < n; i++) {
    uint32_t c;
    int v = ufo_frame_validate(frames + i * stride, frame_len, &c);
    if (crc_out) crc_out[i] = c;
    if (valid_out) valid_out[i] = (uint8_t)v;
  }
}

void ufo_validate_varlen(const uint8_t* bytes, const uint64_t* offsets, size_t n,
                         uint32_t* crc_out, uint8_t* valid_out) {
  for (size_t i = 0; i < n; i++) {
    uint32_t c;
    int v = ufo_frame_validate(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), &c);
    if (crc_out) crc_out[i] = c;
    if (valid_out) valid_out[i] = (uint8_t)v;
  }
}

void ufo_seal_fixed(uint8_t* frames, size_t stride, size_t frame_len, size_t n) {
  for (size_t i = 0; i < n; i++) ufo_frame_seal(frames + i * stride, frame_len);
}

void ufo_seal_varlen(uint8_t* bytes, const uint64_t* offsets, size_t n) {
  for (size_t i = 0; i < n; i++) ufo_frame_seal(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}

/* Multi-threaded CPU baseline: the same bytewise loop (crc.rs:94-100) over a fixed-stride
 * batch, frames partitioned contiguously over `nthreads` pthreads.  Used only by
 * bench.py's cpu_baseline leg. */
typedef struct {
  const uint8_t* frames; size_t stride, frame_len, lo, hi; uint32_t* crc_out; uint8_t* valid_out;
} ufo_job;

static void* ufo_worker(void* p) {
  ufo_job* j = (ufo_job*)p;
  ufo_validate_fixed(j->frames + j->lo * j->stride, j->stride, j->frame_len, j->hi - j->lo,
                     j->crc_out ? j->crc_out + j->lo : NULL, j->valid_out ? j->valid_out + j->lo : NULL);
  return NULL;
}

int ufo_validate_fixed_mt(const uint8_t* frames, size_t stride, size_t frame_len, size_t n,
                          uint32_t* crc_out, uint8_t* valid_out, int nthreads) {
  ensure_table();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ufo_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t].frames = frames; jobs[t].stride = stride; jobs[t].frame_len = frame_len;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads; jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    jobs[t].crc_out = crc_out; jobs[t].valid_out = valid_out;
  }
  int started = 1;
  for (int t = 1; t < nthreads; t++, started++)
    if (pthread_create(&th[t], NULL, ufo_worker, &jobs[t]) != 0) break;
  ufo_worker(&jobs[0]);
  for (int t = 1; t < started; t++) pthread_join(th[t], NULL);
  for (int t = started; t < nthreads; t++) ufo_worker(&jobs[t]);
  return 0;
}

/* The same loops over a CSR batch and the seals, frames partitioned contiguously over
 * `nthreads` pthreads (full-size parity checks in tests/ and the config-3 CPU baseline). */
typedef struct {
  int op; /* 0 validate varlen, 1 seal fixed, 2 seal varlen */
  uint8_t* bytes; const uint64_t* offsets; size_t stride, frame_len, lo, hi;
  uint32_t* crc_out; uint8_t* valid_out;
} ufo_job2;

static void* ufo_worker2(void* p) {
  ufo_job2* j = (ufo_job2*)p;
  if (j->op == 0) {
    ufo_validate_varlen(j->bytes, j->offsets + j->lo, j->hi - j->lo, j->crc_out ? j->crc_out + j->lo : NULL,
                        j->valid_out ? j->valid_out + j->lo : NULL);
  } else if (j->op == 1) {
    ufo_seal_fixed(j->bytes + j->lo * j->stride, j->stride, j->frame_len, j->hi - j->lo);
  } else {
    ufo_seal_varlen(j->bytes, j->offsets + j->lo, j->hi - j->lo);
  }
  return NULL;
}

static int ufo_run2(ufo_job2 proto, size_t n, int nthreads) {
  ensure_table();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ufo_job2 jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = proto;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
  }
  int started = 1;
  for (int t = 1; t < nthreads; t++, started++)
    if (pthread_create(&th[t], NULL, ufo_worker2, &jobs[t]) != 0) break;
  ufo_worker2(&jobs[0]);
  for (int t = 1; t < started; t++) pthread_join(th[t], NULL);
  if (started != nthreads) { /* finish the ranges whose thread did not start */
    for (int t = started; t < nthreads; t++) ufo_worker2(&jobs[t]);
  }
  return 0;
}

int ufo_validate_varlen_mt(const uint8_t* bytes, const uint64_t* offsets, size_t n, uint32_t* crc_out,
                           uint8_t* valid_out, int nthreads) {
  ufo_job2 j = {0, (uint8_t*)bytes, offsets, 0, 0, 0, 0, crc_out, valid_out};
  return ufo_run2(j, n, nthreads);
}

int ufo_seal_fixed_mt(uint8_t* frames, size_t stride, size_t frame_len, size_t n, int nthreads) {
  ufo_job2 j = {1, frames, NULL, stride, frame_len, 0, 0, NULL, NULL};
  return ufo_run2(j, n, nthreads);
}

int ufo_seal_varlen_mt(uint8_t* bytes, const uint64_t* offsets, size_t n, int nthreads) {
  ufo_job2 j = {2, bytes, offsets, 0, 0, 0, 0, NULL, NULL};
  return ufo_run2(j, n, nthreads);
}

/* ---------------------------------------------------------------------------------------
 * Restated fixed-frame encoders, used to generate the wire-format golden fixtures of the
 * reference's fixed-value tests (src/frame/serial/mod.rs:760-925).  Each writes into `out`
 * (caller-sized) and returns the frame length.
 * ------------------------------------------------------------------------------------- */
static size_t put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
  return 4;
}

/* serial/mod.rs:437-473, MAX_FRAME_SIZE = 1500 - 28 = 1472 (lib.rs:286-294). */
size_t ufo_write_handshake_syn(uint8_t* out, uint8_t version, uint32_t nonce, uint32_t max_receive_rate,
                               uint32_t max_packet_size, uint32_t max_receive_alloc) {
  const size_t len = 1472;
  memset(out, 0, len);
  out[0] = 0; out[1] = version;
  put_be32(out + 2, nonce); put_be32(out + 6, max_receive_rate);
  put_be32(out + 10, max_packet_size); put_be32(out + 14, max_receive_alloc);
  ufo_frame_seal(out, len);
  return len;
}

/* serial/mod.rs:475-514 */
size_t ufo_write_handshake_syn_ack(uint8_t* out, uint32_t nonce_ack, uint32_t nonce, uint32_t max_receive_rate,
                                   uint32_t max_packet_size, uint32_t max_receive_alloc) {
  const size_t len = 25;
  memset(out, 0, len);
  out[0] = 1;
  put_be32(out + 1, nonce_ack); put_be32(out + 5, nonce); put_be32(out + 9, max_receive_rate);
  put_be32(out + 13, max_packet_size); put_be32(out + 17, max_receive_alloc);
  ufo_frame_seal(out, len);
  return len;
}

/* serial/mod.rs:516-539 */
size_t ufo_write_handshake_ack(uint8_t* out, uint32_t nonce_ack) {
  memset(out, 0, 9);
  out[0] = 2; put_be32(out + 1, nonce_ack);
  ufo_frame_seal(out, 9);
  return 9;
}

/* serial/mod.rs:541-569 ; error: 0 Version, 1 Config, 2 ServerFull */
size_t ufo_write_handshake_error(uint8_t* out, uint32_t nonce_ack, uint8_t error) {
  memset(out, 0, 10);
  out[0] = 3; put_be32(out + 1, nonce_ack); out[5] = error;
  ufo_frame_seal(out, 10);
  return 10;
}

/* serial/mod.rs:571-611 ; id 4 = Disconnect, 5 = DisconnectAck */
size_t ufo_write_disconnect(uint8_t* out, int ack) {
  memset(out, 0, 5);
  out[0] = ack ? 5 : 4;
  ufo_frame_seal(out, 5);
  return 5;
}

/* serial/mod.rs:623-657 ; has_* select the Option fields */
size_t ufo_write_sync(uint8_t* out, int has_frame_id, uint32_t next_frame_id, int has_packet_id,
                      uint32_t next_packet_id) {
  memset(out, 0, 14);
  out[0] = 11;
  out[1] = (uint8_t)((has_frame_id ? 1 : 0) | (has_packet_id ? 2 : 0));
  put_be32(out + 2, has_frame_id ? next_frame_id : 0);
  put_be32(out + 6, has_packet_id ? next_packet_id : 0);
  ufo_frame_seal(out, 14);
  return 14;
}
