// crc_math.cpp -- see crc_math.hpp.  Product code (host side of libuflowcrc.so).
#include "crc_math.hpp"

#include <cstring>

namespace ufc {
namespace {

struct Mat {  // 32x32 GF(2) matrix stored by columns: col[i] = M * e_i
  uint32_t col[32];
};

uint32_t mat_vec(const Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; i++, v >>= 1)
    if (v & 1u) r ^= m.col[i];
  return r;
}

Mat mat_mul(const Mat& a, const Mat& b) {  // a * b
  Mat r;
  for (int i = 0; i < 32; i++) r.col[i] = mat_vec(a, b.col[i]);
  return r;
}

struct Powers {
  Mat p[64];  // p[k] = A^(2^k) (byte-advance matrix powers)
  Powers() {
    const HostTables& t = host_tables();
    Mat a;  // A = one zero-byte step
    for (int i = 0; i < 32; i++) {
      uint32_t v = 1u << i;
      a.col[i] = (v >> 8) ^ t.lin[0][v & 0xff];
    }
    p[0] = a;
    for (int k = 1; k < 64; k++) p[k] = mat_mul(p[k - 1], p[k - 1]);
  }
};

const Powers& powers() {
  static const Powers pw;
  return pw;
}

HostTables make_tables() {
  HostTables t;
  for (int i = 0; i < 256; i++) {
    uint32_t v = (uint32_t)i;
    for (int b = 0; b < 8; b++) v = (v & 1u) ? (v >> 1) ^ kPolyReflected : (v >> 1);
    t.lin[0][i] = v;
  }
  for (int k = 1; k < 8; k++)
    for (int i = 0; i < 256; i++) {
      uint32_t v = t.lin[k - 1][i];
      t.lin[k][i] = (v >> 8) ^ t.lin[0][v & 0xff];
    }
  for (int i = 0; i < 256; i++) t.ref[i] = 0xFF000000u ^ t.lin[0][i ^ 0xff];
  return t;
}

}  // namespace

const HostTables& host_tables() {
  static const HostTables t = make_tables();
  return t;
}

uint32_t advance(uint32_t v, uint64_t nbytes) {
  const Powers& pw = powers();
  for (int k = 0; nbytes; k++, nbytes >>= 1)
    if (nbytes & 1u) v = mat_vec(pw.p[k], v);
  return v;
}

uint32_t init_prefix_word() {
  // Solve A^4 x = 0xFFFFFFFF by Gaussian elimination over GF(2).
  uint32_t cols[32];
  for (int i = 0; i < 32; i++) cols[i] = advance(1u << i, 4);
  // Augmented rows: row r = (bits of equation r over the 32 unknowns, rhs bit)
  uint64_t rows[32];
  for (int r = 0; r < 32; r++) {
    uint64_t row = 0;
    for (int c = 0; c < 32; c++) row |= (uint64_t)((cols[c] >> r) & 1u) << c;
    row |= (uint64_t)1 << 32;  // rhs bit of 0xFFFFFFFF
    rows[r] = row;
  }
  int pivcol[32];
  int r = 0;
  for (int c = 0; c < 32 && r < 32; c++) {
    int p = -1;
    for (int i = r; i < 32; i++)
      if ((rows[i] >> c) & 1u) { p = i; break; }
    if (p < 0) continue;
    uint64_t tmp = rows[r]; rows[r] = rows[p]; rows[p] = tmp;
    for (int i = 0; i < 32; i++)
      if (i != r && ((rows[i] >> c) & 1u)) rows[i] ^= rows[r];
    pivcol[r] = c;
    r++;
  }
  uint32_t x = 0;
  for (int i = 0; i < r; i++) x |= (uint32_t)((rows[i] >> 32) & 1u) << pivcol[i];
  return x;
}

uint32_t host_extend(uint32_t initial_crc, const uint8_t* data, size_t len) {
  const HostTables& t = host_tables();
  uint32_t reg = ~initial_crc;
  while (len >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, data, 4);
    std::memcpy(&hi, data + 4, 4);
    lo ^= reg;
    reg = t.lin[7][lo & 0xff] ^ t.lin[6][(lo >> 8) & 0xff] ^ t.lin[5][(lo >> 16) & 0xff] ^ t.lin[4][lo >> 24] ^
          t.lin[3][hi & 0xff] ^ t.lin[2][(hi >> 8) & 0xff] ^ t.lin[1][(hi >> 16) & 0xff] ^ t.lin[0][hi >> 24];
    data += 8;
    len -= 8;
  }
  while (len--) reg = (reg >> 8) ^ t.lin[0][(reg ^ *data++) & 0xff];
  return ~reg;
}

void build_chain_table(uint32_t out[1024], uint64_t nbytes) {
  for (int k = 0; k < 4; k++)
    for (int e = 0; e < 256; e++) out[k * 256 + e] = advance((uint32_t)e << (8 * k), nbytes);
}

void build_nibble_image(uint32_t out[8192]) {
  for (int c = 0; c < 64; c++) {
    const int s = ((c & 31) << 1) | (c >> 5);
    for (int k = 0; k < 8; k++)
      for (int e = 0; e < 16; e++)
        out[(k * 16 + e) * 64 + c] = advance((uint32_t)e << (4 * k), (uint64_t)4 * (63 - s));
  }
}

// The inverse of A^nbytes (GF(2) Gauss-Jordan on the 32 columns), applied to v.
uint32_t retreat(uint32_t v, uint64_t nbytes) {
  uint32_t cols[32];
  for (int i = 0; i < 32; i++) cols[i] = advance(1u << i, nbytes);
  // rows of [M | I]: row r = bits r of the columns (M part) and e_r (identity part)
  uint64_t rows[32];
  for (int r = 0; r < 32; r++) {
    uint64_t row = (uint64_t)1 << (32 + r);
    for (int c = 0; c < 32; c++) row |= (uint64_t)((cols[c] >> r) & 1u) << c;
    rows[r] = row;
  }
  for (int c = 0; c < 32; c++) {
    int piv = -1;
    for (int r = c; r < 32; r++)
      if ((rows[r] >> c) & 1u) { piv = r; break; }
    if (piv < 0) return 0;  // (A is invertible: not reached)
    const uint64_t t = rows[c]; rows[c] = rows[piv]; rows[piv] = t;
    for (int r = 0; r < 32; r++)
      if (r != c && ((rows[r] >> c) & 1u)) rows[r] ^= rows[c];
  }
  // rows[r] = [e_r | row r of M^-1]: x = M^-1 v, x_r = parity(rowinv_r & v)
  uint32_t x = 0;
  for (int r = 0; r < 32; r++) x |= (uint32_t)(__builtin_popcount((uint32_t)(rows[r] >> 32) & v) & 1) << r;
  return x;
}

void build_nibble_image32(uint32_t out[8192]) {
  for (int c = 0; c < 64; c++)
    for (int k = 0; k < 8; k++)
      for (int e = 0; e < 16; e++) {
        uint32_t v = 0;
        if (c < 32) {
          v = advance((uint32_t)e << (4 * k), (uint64_t)4 * (31 - c));
        } else if (k >= 2 && k <= 4) {  // A^-t (t = k - 1 bytes) of nibble (c - 32) & 7 alone: column
          // 32 + l belongs to lane l of a half-wave, which looks up its own nibble (rows 0..31 of
          // columns 32..39 hold the front-fix table, row 127 of column 63 the run counter)
          v = retreat((uint32_t)e << (4 * ((c - 32) & 7)), (uint64_t)(k - 1));
        }
        out[(k * 16 + e) * 64 + c] = v;
      }
}

}  // namespace ufc
