/* C (not C++) caller of libuflowcrc.so on the GPU: what a Rust `extern "C"` block over the
 * reference's host buffers would do.  No HIP in the caller: the frames live in
 * host memory and the host-buffer entry points stage them to the device.
 *   - a flush: variable-length frames (5..1472 B, src/lib.rs:294) laid out with zero trailers,
 *     sealed on the GPU (ufc_seal_host_varlen; build.rs:151-159), every frame then checked by the
 *     scalar host gate (ufc_frame_validate; serial/mod.rs:675-690);
 *   - a receive batch: the same frames with one bit flipped in every 7th, gated on the GPU
 *     (ufc_validate_host_varlen, and ufc_validate_host_slots in recvmmsg layout); CRC words and valid
 *     flags vs the scalar host entry points frame by frame.
 * Built with gcc and run by tests/test_gpu_c_caller.py on the GPU box.  Prints "c gpu ok". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "uflow_frame_crc.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                     \
    }                                                              \
  } while (0)

static uint64_t rng = 0x5EED0C0Cull;
static uint32_t next(void) {
  rng = rng * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(rng >> 33);
}

int main(void) {
  const size_t n = 200000, slot = 1472;
  uint64_t* off = malloc((n + 1) * sizeof *off);
  uint32_t* lens = malloc(n * sizeof *lens);
  off[0] = 0;
  for (size_t i = 0; i < n; i++) {
    lens[i] = 5 + next() % 1468;
    off[i + 1] = off[i] + lens[i];
  }
  uint8_t* bytes = malloc(off[n]);
  for (uint64_t b = 0; b < off[n]; b++) bytes[b] = (uint8_t)next();
  for (size_t i = 0; i < n; i++) memset(bytes + off[i + 1] - 4, 0, 4);  /* the builders' zero trailers */

  ufc_ctx* ctx = NULL;
  int rc = ufc_ctx_create(&ctx, 0);
  CHECK(rc == UFC_OK);
  if (rc != UFC_OK) return 1;

  /* the send side: seal on the GPU, check with the scalar host gate */
  uint32_t* crc = malloc(n * sizeof *crc);
  CHECK(ufc_seal_host_varlen(ctx, bytes, off, n, crc) == UFC_OK);
  size_t sealed_ok = 0;
  for (size_t i = 0; i < n; i++) {
    const uint8_t* f = bytes + off[i];
    sealed_ok += ufc_frame_validate(f, lens[i]) == 1 &&
                 crc[i] == ufc_crc32_compute(f, lens[i] - 4);
  }
  CHECK(sealed_ok == n);

  /* the receive side: flip a bit in every 7th frame, gate on the GPU (CSR and slot layouts) */
  for (size_t i = 0; i < n; i += 7) bytes[off[i] + next() % lens[i]] ^= (uint8_t)(1u << (next() % 8));
  uint8_t* valid = malloc(n);
  CHECK(ufc_validate_host_varlen(ctx, bytes, off, n, crc, valid) == UFC_OK);
  uint8_t* slots = calloc(n, slot);
  for (size_t i = 0; i < n; i++) memcpy(slots + i * slot, bytes + off[i], lens[i]);
  uint32_t* crc2 = malloc(n * sizeof *crc2);
  uint8_t* valid2 = malloc(n);
  CHECK(ufc_validate_host_slots(ctx, slots, slot, lens, n, crc2, valid2) == UFC_OK);
  size_t agree = 0, nvalid = 0;
  for (size_t i = 0; i < n; i++) {
    const uint8_t* f = bytes + off[i];
    const int v = ufc_frame_validate(f, lens[i]);
    const uint32_t c = ufc_crc32_compute(f, lens[i] - 4);
    agree += valid[i] == v && crc[i] == c && valid2[i] == v && crc2[i] == c;
    nvalid += v;
  }
  CHECK(agree == n);
  CHECK(nvalid < n && nvalid >= n - (n + 6) / 7);  /* every flipped frame is rejected */
  CHECK(ufc_ctx_destroy(ctx) == UFC_OK);
  free(off); free(lens); free(bytes); free(crc); free(valid); free(slots); free(crc2); free(valid2);
  if (fails) return 1;
  printf("c gpu ok: %zu frames sealed and gated through the C ABI, %zu valid\n", n, nvalid);
  return 0;
}
