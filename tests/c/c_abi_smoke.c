/* C (not C++) caller of libuflowcrc.so: the headers compile as C99 and the host entry points --
 * the drop-ins for crc::compute / crc::extend (src/frame/serial/crc.rs:94-104), the Frame::read
 * CRC gate (serial/mod.rs:675-690), the seal (serial/mod.rs:463-470) and the DataFrameBuilder
 * (build.rs:47-162) -- behave as the reference's tests require.  No GPU needed: a missing
 * device must make ufc_ctx_create fail cleanly (UFC_ERR_NO_DEVICE), never fall back to the CPU.
 * Built and run by tests/test_native_cpu.py with gcc. */
#include <stdio.h>
#include <stdlib.h>
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

/* The multi-GPU gather plan (ufc_shard_gather_plan), checked as a whole for one batch: every rank
 * gates its shard exactly once in order, every SEND is matched by the root's RECV of the same chunk
 * (same peer, count, source and destination), and the root's outputs are covered exactly once. */
typedef struct {
  uint64_t a, b;
} span;
static int span_cmp(const void* x, const void* y) {
  const span* p = (const span*)x;
  const span* q = (const span*)y;
  return p->a < q->a ? -1 : p->a > q->a;
}
static void check_plan(const uint64_t* bounds, int W, int root) {
  const uint64_t n = bounds[W];
  const int K = ufc_shard_nchunks(bounds, W);
  CHECK(K >= 1 && K <= 16);
  static span cover[64 * 16 + 16];
  int ncover = 0;
  uint64_t gated[64] = {0};
  for (int c = 0; c < K; c++) {
    ufc_xfer root_ops[UFC_MAX_RANKS + 1];
    const int nroot = ufc_shard_gather_plan(bounds, W, root, root, c, root_ops, UFC_MAX_RANKS + 1);
    CHECK(nroot >= 0 && nroot <= W);
    CHECK(ufc_shard_gather_plan(bounds, W, root, root, c, NULL, 0) == nroot);
    for (int r = 0; r < W; r++) {
      ufc_xfer ops[UFC_MAX_RANKS + 1];
      const int m = ufc_shard_gather_plan(bounds, W, r, root, c, ops, UFC_MAX_RANKS + 1);
      CHECK(m >= 0 && m <= (r == root ? W : 2));
      for (int i = 0; i < m; i++) {
        const ufc_xfer* o = &ops[i];
        if (o->op == UFC_OP_GATE) {
          CHECK(o->peer == r && o->src == gated[r] && o->count > 0);
          CHECK(o->dst == (r == root ? bounds[r] : 0) + o->src);
          gated[r] += o->count;
          if (r == root) cover[ncover++] = (span){o->dst, o->dst + o->count};
        } else if (o->op == UFC_OP_SEND) {
          CHECK(r != root && o->peer == root && o->count > 0 && o->dst == bounds[r] + o->src);
          CHECK(i > 0 && ops[i - 1].op == UFC_OP_GATE && ops[i - 1].src == o->src && ops[i - 1].count == o->count);
          int matched = 0;
          for (int j = 0; j < nroot; j++) {
            const ufc_xfer* q = &root_ops[j];
            if (q->op == UFC_OP_RECV && q->peer == r)
              matched += q->src == o->src && q->dst == o->dst && q->count == o->count;
          }
          CHECK(matched == 1);
          cover[ncover++] = (span){o->dst, o->dst + o->count};
        } else {
          CHECK(o->op == UFC_OP_RECV && r == root && o->peer != root);
        }
      }
    }
  }
  for (int r = 0; r < W; r++) CHECK(gated[r] == bounds[r + 1] - bounds[r]);
  qsort(cover, ncover, sizeof(span), span_cmp);
  uint64_t at = 0;
  for (int i = 0; i < ncover; i++) {
    CHECK(cover[i].a == at && cover[i].b > cover[i].a);
    at = cover[i].b;
  }
  CHECK(at == n);
}

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
  {
    const int worlds[3] = {2, 3, 8};
    const uint64_t sizes[4] = {0, 5, 1000000u, 100000000u};
    for (int wi = 0; wi < 3; wi++)
      for (int si = 0; si < 4; si++)
        for (int root = 0; root < worlds[wi]; root += worlds[wi] - 1) {
          uint64_t bounds[UFC_MAX_RANKS + 1];
          CHECK(ufc_shard_bounds_fixed(sizes[si], worlds[wi], bounds) == UFC_OK);
          for (int r = 0; r < worlds[wi]; r++) {
            uint64_t f, c;
            CHECK(ufc_shard_range(sizes[si], worlds[wi], r, &f, &c) == UFC_OK && f == bounds[r] && f + c == bounds[r + 1]);
          }
          check_plan(bounds, worlds[wi], root);
        }
    /* config 4: 12.5M frames per rank over 8 GPUs -> 3 chunks of <= 2^22 frames */
    uint64_t b8[9];
    CHECK(ufc_shard_bounds_fixed(100000000u, 8, b8) == UFC_OK && ufc_shard_nchunks(b8, 8) == 3);
    /* variable length: split by bytes (binary search on the offsets) */
    static uint64_t off[100001];
    off[0] = 0;
    for (int i = 0; i < 100000; i++) off[i + 1] = off[i] + 64 + (uint64_t)((i * 2654435761u) % 1437u);
    for (int wi = 0; wi < 3; wi++) {
      const int W = worlds[wi];
      uint64_t bv[UFC_MAX_RANKS + 1];
      CHECK(ufc_shard_bounds_varlen(off, 100000, W, bv) == UFC_OK && bv[0] == 0 && bv[W] == 100000);
      for (int r = 1; r < W; r++) { /* first frame starting at or past r / W of the bytes */
        const uint64_t t = off[100000] * (uint64_t)r / (uint64_t)W;
        CHECK(off[bv[r]] >= t && off[bv[r] - 1] < t);
      }
      check_plan(bv, W, 0);
      check_plan(bv, W, W - 1);
    }
    uint64_t bad[3] = {0, 5, 4};
    CHECK(ufc_shard_nchunks(bad, 2) == UFC_ERR_INVALID_ARG);
    CHECK(ufc_shard_gather_plan(b8, 8, 8, 0, 0, NULL, 0) == UFC_ERR_INVALID_ARG);
    CHECK(ufc_shard_gather_plan(b8, 8, 0, 0, 3, NULL, 0) == UFC_ERR_INVALID_ARG);
  }
  ufc_comm* comm = NULL;
  uint8_t id[UFC_COMM_ID_BYTES] = {0};
  CHECK(ufc_comm_create(&comm, NULL, 2, 0, id) == UFC_ERR_INVALID_ARG && comm == NULL);
  CHECK(ufc_crc_sharded(NULL, NULL, 1500, 1500, 10, NULL, NULL, 0, NULL, NULL) == UFC_ERR_INVALID_ARG);
  CHECK(ufc_crc_sharded_varlen(NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, NULL) == UFC_ERR_INVALID_ARG);

  if (fails) return 1;
  printf("c abi ok\n");
  return 0;
}
