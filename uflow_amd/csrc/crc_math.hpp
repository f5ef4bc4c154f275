// crc_math.hpp -- host-side GF(2) arithmetic for uflow's frame CRC-32 (product code).
//
// The reference CRC (src/frame/serial/crc.rs) is a reflected table-driven CRC-32 with
// polynomial 0x132c00699 (reflected form 0x9960034C, crc.rs:50), INITIAL_CRC = 0 (crc.rs:41)
// and the init/xorout complement folded into its table PARTIAL_RESULTS (crc.rs:59-92):
//     extend(c, data): for byte b: c = (c >> 8) ^ T[(c ^ b) & 0xff]          (crc.rs:94-100)
// In the register domain (reg = ~crc, crc.rs:45 / :56) the same loop is linear over GF(2):
//     reg = (reg >> 8) ^ L[(reg ^ b) & 0xff],   L[i] = step8(i),  T[i] = 0xFF000000 ^ L[i ^ 0xff]
// Everything below works in that linear register domain.  A^n denotes "advance the register
// over n zero bytes", a linear map; A^4 is the slice-by-4 word step.
#pragma once
#include <cstdint>
#include <cstddef>

namespace ufc {

constexpr uint32_t kPolyReflected = 0x9960034Cu;  // crc.rs:50

struct HostTables {
  uint32_t lin[8][256];   // slice-by-8 linear tables; lin[0] = L (one byte step)
  uint32_t ref[256];      // PARTIAL_RESULTS (crc.rs:59-92), regenerated from the polynomial
};

// Built once, thread-safe (C++11 static init).
const HostTables& host_tables();

// A^n(v): advance the linear register v over n zero bytes.  O(log n) via GF(2) matrix powers.
uint32_t advance(uint32_t v, uint64_t nbytes);

// G = A^-4(0xFFFFFFFF): four bytes that, processed from register 0, leave the register at ~0.
// Prefixing a frame's CRC bytes with G folds the reference's init (~0) into plain linear CRC.
uint32_t init_prefix_word();

// Host scalar CRC with the reference's semantics (slice-by-8 in the register domain).
uint32_t host_extend(uint32_t initial_crc, const uint8_t* data, size_t len);

// Device table images (layouts documented in frame_crc.hip):
//   chain[k*256 + e] = A^nbytes(e << 8k)                    k = 0..3, e = 0..255   (1024 words)
//   nib[(k*16 + e)*64 + c] = A^(4(63 - s))(e << 4k),  s = ((c & 31) << 1) | (c >> 5)  (8192 words)
//   nib32[(k*16 + e)*64 + c] = A^(4(31 - c))(e << 4k) for c < 32 (8-lane frames, 32 slots);
//     columns 40 + 3 g + (t - 1), g = 0..3, t = 1..3: A^-t(e << 4k) (bytes past a frame's end); 0 else
void build_chain_table(uint32_t out[1024], uint64_t nbytes);
void build_nibble_image(uint32_t out[8192]);
void build_nibble_image32(uint32_t out[8192]);
// A^-nbytes(v): the register before nbytes zero bytes that leave it at v.
uint32_t retreat(uint32_t v, uint64_t nbytes);

}  // namespace ufc
