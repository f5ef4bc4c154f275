/* C (not C++) caller of libuflowcrc.so on the GPU: what a Rust `extern "C"` block over the
 * reference's host buffers would do.  No HIP in the caller: the frames live in
 * host memory and the host-buffer entry points stage them to the device.  Every result is compared
 * with the CPU oracle's (oracle/crc_oracle.c), which tests/test_gpu_c_caller.py computes and hands
 * over in a file -- not with the library's own host path:
 *   - a flush: variable-length frames (5..1472 B, src/lib.rs:294) laid out with zero trailers,
 *     sealed on the GPU (ufc_seal_host_varlen; build.rs:151-159): the CRC words and every sealed byte
 *     equal the oracle's seal of the same frames;
 *   - a receive batch: the sealed frames with the file's bit flips applied, gated on the GPU
 *     (ufc_validate_host_varlen, and ufc_validate_host_slots in recvmmsg layout): CRC words and valid
 *     flags equal the oracle's gate (serial/mod.rs:675-690) frame by frame.
 * File (little-endian): u64 n, u64 nbytes, u64 nflips; u64 offsets[n + 1]; u8 bytes[nbytes] (zero
 * trailers); u8 sealed[nbytes] (the oracle's seal); u32 seal_crc[n]; u64 flip_at[nflips]; u8
 * flip_mask[nflips]; u32 crc[n]; u8 valid[n] (the oracle's gate after the flips).
 * Usage: c_abi_gpu <file>.  Prints "c gpu ok". */
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

static void* take(FILE* f, size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "short file\n");
    exit(2);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s <oracle file>\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint64_t* hdr = take(f, 3 * sizeof(uint64_t));
  const size_t n = (size_t)hdr[0], nbytes = (size_t)hdr[1], nflips = (size_t)hdr[2];
  uint64_t* off = take(f, (n + 1) * sizeof *off);
  uint8_t* bytes = take(f, nbytes);
  uint8_t* o_sealed = take(f, nbytes);
  uint32_t* o_seal_crc = take(f, n * sizeof *o_seal_crc);
  uint64_t* flip_at = take(f, nflips * sizeof *flip_at);
  uint8_t* flip_mask = take(f, nflips);
  uint32_t* o_crc = take(f, n * sizeof *o_crc);
  uint8_t* o_valid = take(f, n);
  fclose(f);
  CHECK(off[0] == 0 && off[n] == nbytes);

  ufc_ctx* ctx = NULL;
  int rc = ufc_ctx_create(&ctx, 0);
  CHECK(rc == UFC_OK);
  if (rc != UFC_OK) return 1;

  /* the send side: seal on the GPU; the CRC words and every byte as the oracle's seal */
  uint32_t* crc = malloc(n * sizeof *crc);
  CHECK(ufc_seal_host_varlen(ctx, bytes, off, n, crc) == UFC_OK);
  CHECK(memcmp(crc, o_seal_crc, n * sizeof *crc) == 0);
  CHECK(memcmp(bytes, o_sealed, nbytes) == 0);

  /* the receive side: the file's bit flips, then the gate on the GPU (CSR and slot layouts) */
  for (size_t k = 0; k < nflips; k++) bytes[flip_at[k]] ^= flip_mask[k];
  uint8_t* valid = malloc(n);
  CHECK(ufc_validate_host_varlen(ctx, bytes, off, n, crc, valid) == UFC_OK);
  const size_t slot = 1472;
  uint8_t* slots = calloc(n, slot);
  uint32_t* lens = malloc(n * sizeof *lens);
  for (size_t i = 0; i < n; i++) {
    lens[i] = (uint32_t)(off[i + 1] - off[i]);
    memcpy(slots + i * slot, bytes + off[i], lens[i]);
  }
  uint32_t* crc2 = malloc(n * sizeof *crc2);
  uint8_t* valid2 = malloc(n);
  CHECK(ufc_validate_host_slots(ctx, slots, slot, lens, n, crc2, valid2) == UFC_OK);
  size_t agree = 0, nvalid = 0;
  for (size_t i = 0; i < n; i++) {
    agree += crc[i] == o_crc[i] && valid[i] == o_valid[i] && crc2[i] == o_crc[i] && valid2[i] == o_valid[i];
    nvalid += o_valid[i];
  }
  CHECK(agree == n);
  CHECK(nvalid < n);
  CHECK(ufc_ctx_destroy(ctx) == UFC_OK);
  free(hdr); free(off); free(bytes); free(o_sealed); free(o_seal_crc); free(flip_at); free(flip_mask);
  free(o_crc); free(o_valid); free(crc); free(valid); free(slots); free(lens); free(crc2); free(valid2);
  if (fails) return 1;
  printf("c gpu ok: %zu frames sealed and gated through the C ABI, equal to the oracle's; %zu valid\n", n, nvalid);
  return 0;
}
