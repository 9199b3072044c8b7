// Host side of the drop-in: leveldb::crc32c::{Extend} (util/crc32c.cc:487-588)
// and the scalar C-ABI.  Single-block calls stay on the host CPU: a 4 KiB
// block costs ~1.4 us on one core, far below a kernel launch.
// Batches go to the GPU (crc32c_device.hip) and never come back here.
//
// Implementation: the SSE4.2 `crc32` instruction computes exactly CRC-32C
// (same reflected polynomial) -- the role Google crc32c plays behind the
// reference's port::AcceleratedCRC32C hook (port/port_stdcxx.h:179-189) --
// three independent chains at a time on buffers of >= 768 bytes.  A portable
// slicing-by-8 path (tables generated from the polynomial) covers hosts
// without it.
#include <cstring>
#include <mutex>

#include "../../include/nova_crc32c.h"
#include "../../include/nova_crc32c.hpp"
#include "gf2_crc32c.hpp"

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

namespace {

struct Slice8 {
  uint32_t t[8][256];
  Slice8() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int b = 0; b < 8; b++) c = (c >> 1) ^ (nova::gf2::kPoly & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (int k = 1; k < 8; k++)
      for (uint32_t i = 0; i < 256; i++) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xff];
  }
};

const Slice8& slice8() {
  static const Slice8 s;
  return s;
}

uint32_t raw_portable(uint32_t l, const uint8_t* p, size_t n) {
  const Slice8& s = slice8();
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    l = s.t[0][(l ^ *p++) & 0xff] ^ (l >> 8);
    n--;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);  // little-endian host
    std::memcpy(&hi, p + 4, 4);
    lo ^= l;
    l = s.t[7][lo & 0xff] ^ s.t[6][(lo >> 8) & 0xff] ^ s.t[5][(lo >> 16) & 0xff] ^
        s.t[4][lo >> 24] ^ s.t[3][hi & 0xff] ^ s.t[2][(hi >> 8) & 0xff] ^
        s.t[1][(hi >> 16) & 0xff] ^ s.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) l = s.t[0][(l ^ *p++) & 0xff] ^ (l >> 8);
  return l;
}

#if defined(__x86_64__)
// One dependent `crc32` chain retires 8 bytes per instruction latency (3
// cycles), a third of the instruction's throughput.  Long buffers therefore
// run three independent chains over three adjacent S-byte blocks and join
// them with the GF(2) shift:
//   raw_l(A || B || C) = M_2S(raw_l(A)) ^ M_S(raw_0(B)) ^ raw_0(C)
// (raw_l: register from l; M_k: k zero bytes, applied as four byte tables).
struct Shift3 {
  uint32_t m1[4][256], m2[4][256];  // M_S, M_2S
  explicit Shift3(uint64_t S) {
    nova::gf2::byte_tables(nova::gf2::shift_bytes(S), m1);
    nova::gf2::byte_tables(nova::gf2::shift_bytes(2 * S), m2);
  }
  static uint32_t apply(const uint32_t (&t)[4][256], uint32_t x) {
    return t[0][x & 255] ^ t[1][(x >> 8) & 255] ^ t[2][(x >> 16) & 255] ^ t[3][x >> 24];
  }
};
constexpr size_t kS3Long = 2048, kS3Short = 256;  // block sizes of the 3-way passes
const Shift3& shift_long() {
  static const Shift3 s(kS3Long);
  return s;
}
const Shift3& shift_short() {
  static const Shift3 s(kS3Short);
  return s;
}

template <size_t S>
__attribute__((target("sse4.2"))) inline uint64_t pass3(uint64_t l, const uint8_t* p, const Shift3& sh) {
  uint64_t a = l, b = 0, c = 0;
  for (size_t i = 0; i < S; i += 8) {
    uint64_t wa, wb, wc;
    std::memcpy(&wa, p + i, 8);
    std::memcpy(&wb, p + S + i, 8);
    std::memcpy(&wc, p + 2 * S + i, 8);
    a = _mm_crc32_u64(a, wa);
    b = _mm_crc32_u64(b, wb);
    c = _mm_crc32_u64(c, wc);
  }
  return Shift3::apply(sh.m2, (uint32_t)a) ^ Shift3::apply(sh.m1, (uint32_t)b) ^ (uint32_t)c;
}

__attribute__((target("sse4.2"))) uint32_t raw_sse42(uint32_t l, const uint8_t* p, size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    l = _mm_crc32_u8(l, *p++);
    n--;
  }
  uint64_t l64 = l;
  if (n >= 3 * kS3Long) {
    const Shift3& sh = shift_long();
    do {
      l64 = pass3<kS3Long>(l64, p, sh);
      p += 3 * kS3Long;
      n -= 3 * kS3Long;
    } while (n >= 3 * kS3Long);
  }
  if (n >= 3 * kS3Short) {
    const Shift3& sh = shift_short();
    do {
      l64 = pass3<kS3Short>(l64, p, sh);
      p += 3 * kS3Short;
      n -= 3 * kS3Short;
    } while (n >= 3 * kS3Short);
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    l64 = _mm_crc32_u64(l64, w);
    p += 8;
    n -= 8;
  }
  l = static_cast<uint32_t>(l64);
  while (n--) l = _mm_crc32_u8(l, *p++);
  return l;
}
bool have_sse42() {
  static const bool ok = __builtin_cpu_supports("sse4.2");
  return ok;
}
#endif

// Raw register update (no pre/post complement).
uint32_t raw_update(uint32_t l, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (have_sse42()) return raw_sse42(l, p, n);
#endif
  return raw_portable(l, p, n);
}

}  // namespace

namespace leveldb {
namespace crc32c {

uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  // util/crc32c.cc:495 / :587: pre- and post-condition with all ones.
  return raw_update(init_crc ^ 0xffffffffu, reinterpret_cast<const uint8_t*>(data), n) ^
         0xffffffffu;
}

}  // namespace crc32c
}  // namespace leveldb

extern "C" {

uint32_t nova_crc32c_extend(uint32_t init_crc, const char* data, size_t n) {
  return leveldb::crc32c::Extend(init_crc, data, n);
}
uint32_t nova_crc32c_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }
uint32_t nova_crc32c_mask(uint32_t crc) { return leveldb::crc32c::Mask(crc); }
uint32_t nova_crc32c_unmask(uint32_t m) { return leveldb::crc32c::Unmask(m); }

// crc32_combine.  With raw() the zero-init register and M_n the n-zero-byte
// shift:  Extend(crc_a, B) = ~(M_n(~crc_a) ^ raw(B))  and  crc_b = ~(M_n(~0) ^ raw(B)),
// so Extend(crc_a, B) = crc_b ^ M_n(~crc_a) ^ M_n(~0) = crc_b ^ M_n(crc_a).
uint32_t nova_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  if (len_b == 0) return crc_a;
  const nova::gf2::Lin m = nova::gf2::shift_bytes(len_b);
  return crc_b ^ m(crc_a);
}

}  // extern "C"
