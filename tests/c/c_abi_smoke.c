/* C (not C++) caller of libuflowcrc.so: the headers compile as C99 and the host entry points --
 * the drop-ins for crc::compute / crc::extend (src/frame/serial/crc.rs:94-104), the Frame::read
 * CRC gate (serial/mod.rs:675-690), the seal (serial/mod.rs:463-470) and the DataFrameBuilder
 * (build.rs:47-162) -- behave as the reference's tests require.  No GPU needed: a missing
 * device must make ufc_ctx_create fail cleanly (UFC_ERR_NO_DEVICE), never fall back to the CPU.
 * Built and run by tests/test_native_cpu.py with gcc. */
#include <stdio.h>
#include <string.h>

#include "uflow_frame_codec.h"
#include "uflow_frame_crc.h"

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                \
    }                                                         \
  } while (0)

int main(void) {
  const char* kat = "123456789";
  CHECK(ufc_crc32_compute((const uint8_t*)kat, 9) == 0x11A6F2A3u); /* crc.rs:135-138 */
  const uint8_t zero = 0;
  CHECK(ufc_crc32_compute(&zero, 1) != 0); /* crc.rs:130-132 */
  CHECK(ufc_crc32_extend(ufc_crc32_compute((const uint8_t*)kat, 4), (const uint8_t*)kat + 4, 5) == 0x11A6F2A3u);

  /* a data frame with one datagram, built, sealed, validated; a flipped bit is rejected */
  uint8_t buf[1472], payload[100];
  for (int i = 0; i < 100; i++) payload[i] = (uint8_t)(i * 7 + 1);
  ufc_builder b;
  CHECK(ufc_data_frame_builder_init(&b, buf, sizeof buf, 0x12345, 1) == UFC_OK);
  ufc_datagram_ref d;
  memset(&d, 0, sizeof d);
  d.sequence_id = 77;
  d.channel_id = 3;
  d.data = payload;
  d.data_len = 100;
  CHECK(ufc_data_frame_builder_add(&b, &d) == UFC_OK);
  const size_t len = ufc_builder_build(&b, 1);
  CHECK(len > 5 && len < sizeof buf);
  CHECK(ufc_frame_validate(buf, len) == 1);
  ufc_frame_info info;
  ufc_item items[4];
  CHECK(ufc_frame_read(buf, len, &info, items, 4) == 1);
  CHECK(info.kind == UFC_FRAME_DATA && info.item_count == 1 && items[0].data_len == 100);
  buf[10] ^= 0x20;
  CHECK(ufc_frame_validate(buf, len) == 0);
  buf[10] ^= 0x20;
  /* the seal of a frame with a zero trailer reproduces the builder's trailer */
  uint8_t copy[1472];
  memcpy(copy, buf, len);
  memset(copy + len - 4, 0, 4);
  CHECK(ufc_frame_seal(copy, len) == UFC_OK && memcmp(copy, buf, len) == 0);
  /* too short for the gate (serial/mod.rs:676-678) */
  CHECK(ufc_frame_validate(buf, 4) == 0);

  /* no silent CPU fallback for the batched path */
  ufc_ctx* ctx = NULL;
  const int rc = ufc_ctx_create(&ctx, 0);
  if (ufc_device_count() == 0) CHECK(rc == UFC_ERR_NO_DEVICE && ctx == NULL);
  if (ctx) ufc_ctx_destroy(ctx);
  CHECK(ufc_error_string(UFC_ERR_INVALID_ARG) != NULL);
  CHECK(ufc_error_string(UFC_ERR_COMM) != NULL);

  /* NULL buffers are argument errors, never crashes (no context here either way) */
  uint32_t scratch[4];
  CHECK(ufc_seal_host_slots(NULL, NULL, 1472, NULL, 4, scratch) == UFC_ERR_INVALID_ARG);
  CHECK(ufc_seal_host_varlen(NULL, NULL, NULL, 4, scratch) == UFC_ERR_INVALID_ARG);
  CHECK(ufc_validate_host_slots_async(NULL, NULL, 1472, NULL, 4, scratch, NULL, NULL) == UFC_ERR_INVALID_ARG);
  CHECK(ufc_ctx_set_option(NULL, UFC_OPT_FIXED_KERNEL, UFC_FIXED_AUTO) == UFC_ERR_INVALID_ARG);

  /* multi-GPU layout: config 4 (100M frames over 8 GPUs) -> 12.5M frames per rank, 3 chunks */
  uint64_t first = 0, count = 0;
  CHECK(ufc_shard_range(100000000u, 8, 3, &first, &count) == UFC_OK && first == 37500000u && count == 12500000u);
  CHECK(ufc_shard_chunk(100000000u, 8, 3, 2, &first, &count) == 3 && first + count == 50000000u);
  CHECK(ufc_shard_range(10, 2, 2, &first, &count) == UFC_ERR_INVALID_ARG);
  ufc_comm* comm = NULL;
  uint8_t id[UFC_COMM_ID_BYTES] = {0};
  CHECK(ufc_comm_create(&comm, NULL, 2, 0, id) == UFC_ERR_INVALID_ARG && comm == NULL);
  CHECK(ufc_crc_sharded(NULL, NULL, 1500, 1500, 10, NULL, NULL, 0, NULL, NULL) == UFC_ERR_INVALID_ARG);

  if (fails) return 1;
  printf("c abi ok\n");
  return 0;
}
