// ubsan_helpers.hip -- the kernels' mask and shift helpers as host code under UBSan
// (-fsanitize=undefined -fno-sanitize-recover=all, tests/test_ubsan_helpers.py), each over its
// whole argument range and against a byte-wise restatement: an out-of-range shift amount in any arm,
// selected or not, stops the run ("a mechanical guard against out-of-range shifts").
//   fix_word, front_fix, data_mask, data_mask_bits, frame_word_mask, rot_nibble_key  (frame_crc_dev.hpp)
//   head_byte                                                        (frame_parse.hpp)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../uflow_amd/csrc/frame_crc_dev.hpp"
#include "../../uflow_amd/csrc/frame_parse.hpp"

using namespace ufc_dev;

static int g_fail = 0;
#define CHECK(c, ...)                  \
  do {                                 \
    if (!(c)) {                        \
      if (g_fail++ < 20) {             \
        std::printf("FAIL: " __VA_ARGS__); \
        std::printf("\n");             \
      }                                \
    }                                  \
  } while (0)

static uint32_t rng_state = 0x5EED1234u;
static uint32_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return rng_state;
}

// The virtual stream's byte at frame offset fo: data at fo >= 0, G's byte fo + 4 at [-4, 0), zero below.
static uint8_t stream_byte(uint8_t data, int fo, uint32_t G) {
  if (fo >= 0) return data;
  if (fo >= -4) return (uint8_t)(G >> (8 * (fo + 4)));
  return 0;
}

int main() {
  const uint32_t Gs[] = {0x4474BF9Bu, 0xFFFFFFFFu, 0x01020304u, 0u};
  long checks = 0;
  for (uint32_t G : Gs) {
    // fix_word: every frame offset o of the word's first byte, -300..300
    for (int o = -300; o <= 300; o++)
      for (int r = 0; r < 8; r++) {
        const uint32_t v = r == 0 ? 0u : (r == 1 ? ~0u : rnd());
        const uint32_t got = fix_word(v, o, G);
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want |= (uint32_t)stream_byte((uint8_t)(v >> (8 * k)), o + k, G) << (8 * k);
        CHECK(got == want, "fix_word(%08x, %d, %08x) = %08x, want %08x", v, o, G, got, want);
        checks++;
      }
    // front_fix: p = bytes of the lane's 16 before the frame, -260..260
    for (int p = -260; p <= 260; p++)
      for (int r = 0; r < 8; r++) {
        const uint4 x = make_uint4(rnd(), rnd(), rnd(), r == 0 ? 0u : rnd());
        const uint4 got = front_fix(x, p, G);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, gs[4] = {got.x, got.y, got.z, got.w};
        for (int w = 0; w < 4; w++) {
          uint32_t want = 0;
          for (int k = 0; k < 4; k++) {
            const int byte = 4 * w + k;
            const int fo = p > 20 ? byte - 20 - 4 : byte - (p < 0 ? 0 : p);  // (p >= 20: all before G)
            want |= (uint32_t)stream_byte((uint8_t)(xs[w] >> (8 * k)), fo, G) << (8 * k);
          }
          CHECK(gs[w] == want, "front_fix(p=%d, G=%08x) word %d = %08x, want %08x", p, G, w, gs[w], want);
        }
        checks++;
      }
  }
  // data_mask: lb = bytes of the word before the data's end, -300..300
  for (int lb = -300; lb <= 300; lb++) {
    uint32_t want = 0;
    for (int k = 0; k < 4; k++)
      if (k < lb) want |= 0xFFu << (8 * k);
    CHECK(data_mask(lb) == want, "data_mask(%d) = %08x, want %08x", lb, data_mask(lb), want);
    checks++;
  }
  // data_mask_bits: b = 8 lb (any int; the varlen gate passes 8 lim - 32 k): the same mask
  for (int lb = -1000; lb <= 1000; lb++) {
    const int b = 8 * lb;
    CHECK(data_mask_bits(b) == data_mask(lb), "data_mask_bits(%d) = %08x, want %08x", b, data_mask_bits(b), data_mask(lb));
    checks++;
  }
  for (int b : {-2147483647 - 1, -2147483647, 2147483647, 33, 31, -1})
    CHECK(data_mask_bits(b) == (b >= 32 ? ~0u : (b <= 0 ? 0u : ~(0xFFFFFFFFu << b))), "data_mask_bits(%d)", b);
  // frame_word_mask: ob = frame offset of the word's first byte, every frame length 0..2100
  for (uint32_t len = 0; len <= 2100; len++)
    for (int ob = -300; ob <= 2400; ob++) {
      uint32_t want = 0;
      for (int k = 0; k < 4; k++)
        if (ob + k >= 0 && ob + k < (int)len) want |= 0xFFu << (8 * k);
      CHECK(frame_word_mask(ob, len) == want, "frame_word_mask(%d, %u) = %08x, want %08x", ob, len,
            frame_word_mask(ob, len), want);
      checks++;
    }
  for (uint32_t len : {0xFFFFFFFFu, 0x80000000u, 0x7FFFFFFFu})
    for (int ob = -300; ob <= 300; ob++) {
      uint32_t want = 0;
      for (int k = 0; k < 4; k++)
        if (ob + k >= 0) want |= 0xFFu << (8 * k);
      CHECK(frame_word_mask(ob, len) == want, "frame_word_mask(%d, %u)", ob, len);
      checks++;
    }
  // rot_nibble_key: column of nibble step i = (4 col + ((i + u) & 3) + 31 - e) & 31, and the 32 lanes of
  // a half-wave (4 groups, group g with rot = g, any e per group) read 32 distinct columns in every step
  for (uint32_t e = 0; e < 32; e++)
    for (uint32_t rot = 0; rot < 4; rot++) {
      const uint32_t u = (rot - (31u - e)) & 3u;
      for (uint32_t col = 0; col < 8; col++) {
        const uint32_t key = rot_nibble_key(col, u, e);
        for (uint32_t i = 0; i < 4; i++) {
          const uint32_t c = ((key >> (8 * i)) & 0xFFu) / 4u;
          CHECK(((key >> (8 * i)) & 3u) == 0u, "rot_nibble_key byte not a multiple of 4");
          CHECK(c == ((4 * col + ((i + u) & 3) + 31 - e) & 31u), "rot_nibble_key(col %u, u %u, e %u) step %u", col, u, e, i);
          CHECK((c & 3u) == ((i + rot) & 3u), "rot_nibble_key: column %u of group %u, step %u, not in its bank class", c, rot, i);
          checks++;
        }
      }
    }
  for (uint32_t e0 = 0; e0 < 32; e0 += 3)
    for (uint32_t e1 = 0; e1 < 32; e1 += 5)
      for (uint32_t i = 0; i < 4; i++) {
        uint64_t seen = 0;
        const uint32_t es[4] = {e0, e1, (e0 + 7) & 31u, (e1 * 3 + 1) & 31u};
        for (uint32_t g = 0; g < 4; g++)
          for (uint32_t col = 0; col < 8; col++) {
            const uint32_t u = (g - (31u - es[g])) & 3u;
            seen |= 1ull << (((rot_nibble_key(col, u, es[g]) >> (8 * i)) & 0xFFu) / 4u);
          }
        CHECK(seen == 0xFFFFFFFFull, "half-wave columns not distinct (e %u %u, step %u)", e0, e1, i);
        checks++;
      }
  // head_byte: bytes 0..15 of a frame's first 16 bytes from two little-endian words
  for (int r = 0; r < 1000; r++) {
    uint8_t b[16];
    uint64_t w0 = 0, w1 = 0;
    for (int k = 0; k < 16; k++) {
      b[k] = (uint8_t)rnd();
      if (k < 8) w0 |= (uint64_t)b[k] << (8 * k);
      else w1 |= (uint64_t)b[k] << (8 * (k - 8));
    }
    for (uint32_t i = 0; i < 64; i++) {
      CHECK(head_byte(w0, w1, i) == b[i & 15u], "head_byte(%u)", i);
      checks++;
    }
  }
  std::printf("%s: %ld checks, %d failures\n", g_fail ? "FAILED" : "ok", checks, g_fail);
  return g_fail ? 1 : 0;
}
