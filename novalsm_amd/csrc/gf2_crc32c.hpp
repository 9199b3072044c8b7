// GF(2) linear algebra for CRC-32C (Castagnoli, reflected poly 0x82F63B78).
//
// The CRC register update is linear over GF(2): advancing a raw register by k
// zero bytes is a fixed 32x32 bit-matrix M_k, and processing data D from
// register l equals M_|D|(l) xor raw(D).  Every table the engine uses is one
// such operator split into four byte-indexed tables (op(x) = T0[x&255] ^
// T1[x>>8&255] ^ T2[x>>16&255] ^ T3[x>>24]):
//   * the reference's kStrideExtensionTable0..3 (util/crc32c.cc:107-453) are
//     exactly M_16 split this way; the HIP main loop uses M_S
//     for its own stride S = 16 * lanes-per-unit;
//   * kByteExtensionTable (util/crc32c.cc:20-105) is the one-byte step.
// Nothing here is copied from the reference: tables are generated from the
// polynomial at start-up.
#pragma once
#include <cstddef>
#include <cstdint>

namespace nova {
namespace gf2 {

constexpr uint32_t kPoly = 0x82F63B78u;

// A linear map on the 32-bit register, stored by columns: col[i] = M(1 << i).
struct Lin {
  uint32_t col[32];
  uint32_t operator()(uint32_t x) const {
    uint32_t r = 0;
    for (int i = 0; i < 32; i++)
      if (x >> i & 1u) r ^= col[i];
    return r;
  }
};

inline uint32_t byte_step_bitwise(uint32_t l) {  // one zero byte, bit by bit
  for (int b = 0; b < 8; b++) l = (l >> 1) ^ (kPoly & (0u - (l & 1u)));
  return l;
}

inline Lin identity() {
  Lin m;
  for (int i = 0; i < 32; i++) m.col[i] = 1u << i;
  return m;
}

// M_1: the register advanced through one zero byte.
inline Lin zero_byte() {
  Lin m;
  for (int i = 0; i < 32; i++) m.col[i] = byte_step_bitwise(1u << i);
  return m;
}

// (a o b)(x) = a(b(x))
inline Lin compose(const Lin& a, const Lin& b) {
  Lin m;
  for (int i = 0; i < 32; i++) m.col[i] = a(b.col[i]);
  return m;
}

inline Lin power(Lin base, uint64_t e) {
  Lin r = identity();
  while (e) {
    if (e & 1) r = compose(r, base);
    base = compose(base, base);
    e >>= 1;
  }
  return r;
}

// Gauss-Jordan inverse over GF(2).  M_1 is invertible because x is a unit
// modulo the CRC polynomial (it has a non-zero constant term).
inline Lin inverse(const Lin& m) {
  // rows[r] bit c = M[r][c]; augment with identity.
  uint32_t a[32], inv[32];
  for (int r = 0; r < 32; r++) {
    a[r] = 0;
    for (int c = 0; c < 32; c++) a[r] |= ((m.col[c] >> r) & 1u) << c;
    inv[r] = 1u << r;
  }
  for (int c = 0; c < 32; c++) {
    int p = c;
    while (p < 32 && !((a[p] >> c) & 1u)) p++;
    if (p == 32) return identity();  // singular: cannot happen for M_k
    uint32_t t = a[p]; a[p] = a[c]; a[c] = t;
    t = inv[p]; inv[p] = inv[c]; inv[c] = t;
    for (int r = 0; r < 32; r++)
      if (r != c && ((a[r] >> c) & 1u)) { a[r] ^= a[c]; inv[r] ^= inv[c]; }
  }
  Lin out;
  for (int c = 0; c < 32; c++) {
    out.col[c] = 0;
    for (int r = 0; r < 32; r++) out.col[c] |= ((inv[r] >> c) & 1u) << r;
  }
  return out;
}

// Split an operator into four byte tables: out[k][b] = M(b << 8k).
inline void byte_tables(const Lin& m, uint32_t out[4][256]) {
  for (int k = 0; k < 4; k++)
    for (uint32_t b = 0; b < 256; b++) out[k][b] = m(b << (8 * k));
}

// M_n for arbitrary n via square-and-multiply on M_1 (host only; O(32*log n)).
inline Lin shift_bytes(uint64_t n) { return power(zero_byte(), n); }

}  // namespace gf2
}  // namespace nova
