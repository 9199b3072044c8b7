// MI355X (gfx950) batched CRC-32C: the production kernels and their host
// launchers (shared by crc32c_device.hip and crc32c_diag.hip).  Drop-in for the per-SSTable-block checksum of NovaLSM
// (util/crc32c.cc:487-588 called from table/table_builder.cc:202-204,
// ltc/stoc_file_client_impl.cpp:713-719 and table/table.cc:434-440).
//
// ---------------------------------------------------------------------------
// Algorithm (all arithmetic is GF(2) on the 32-bit reflected register)
//
// A "unit" is a byte range [u0,u1) of one block (a whole block, or one
// segment of a long block).  G lanes ("a lane group", G in {1,2,4,8,16})
// process a unit; each lane owns 4 word streams, so the unit is 4G interleaved
// streams with a stride of S = 16G bytes -- the reference's 4-stream/16-byte
// stride loop (util/crc32c.cc:543-577) widened from one CPU thread to G lanes.
// Every wave-instruction of a group loads 16G contiguous bytes (dwordx4 per
// lane).  One stream step is  c = w ^ T0[c&255] ^ T1[c>>8&255] ^ T2[..] ^ T3[..]
// with T = "advance S bytes" split into four byte tables (the reference's
// kStrideExtensionTable is the S=16 case).
//
//   * Alignment: loads are always 16-B aligned.  The unit's region is
//     end-aligned at Eu = roundup16(u1); bytes before u0 read as zero (leading
//     zeros do not change a zero-initialised register), bytes after u1 are
//     zero (t = Eu-u1 trailing zeros, undone at the end by M_t^-1).
//   * Init: Extend(init, D) runs the register from ~init; that equals running
//     from 0 over D with ~init xor-ed into D's first four bytes.
//   * Fold: the 4G stream states are the words of a virtual 16G-byte message;
//     a tree (in-lane M4, M8, then cross-lane M16, M32, ... via shuffles)
//     reduces it to one pending word V; raw(unit) = (M_t^-1 o M4)(V).
//   * Long blocks are cut into segments so all lane groups of a wave carry
//     equal work; a segment j units from the end contributes M_{seg*j}(raw),
//     and contributions are xor-accumulated (order-free, so bit-exact).
//
// LDS (one 1024-thread workgroup per CU): the four main tables are stored as
// 32 bank replicas -- entry idx of copy c at byte (idx<<8)|(c<<2) (+128 for
// the odd table, +64 KiB for tables 2,3) -- so a ds_read_b32 wave-instruction
// is conflict-free whatever the data, and one v_perm_b32 builds each address
// from the register byte and the lane's replica offset.  128 KiB main tables
// + 4 KiB per tree level + 512 B per wave scratch <= 160 KiB.
// ---------------------------------------------------------------------------
#pragma once

#include "crc32c_internal.hpp"

namespace {

using namespace nova_dev;

// ---- log records: bounds and status (db/log_reader.cc:228-262) ------------
// A record at offset o (the image starts at a 32 KiB log-block boundary,
// db/log_format.h:27) must fit its log block and the image; otherwise it is
// not read and gets a status instead of a CRC check.  Inside the kernels such
// a record is carried as an EMPTY CRC range (n = 0; real records have n >= 1,
// the type byte) whose aux word holds the status.
constexpr uint32_t kLogBlock = 32768;
__device__ __forceinline__ uint64_t log_block_end(uint64_t o, uint64_t buf_len) {
  const uint64_t e = (o / kLogBlock + 1) * kLogBlock;
  return e < buf_len ? e : buf_len;
}
// Status of a record whose 7-byte header fits (o + 7 <= block end), from its
// length and type bytes; NOVA_LOG_OK means "check the CRC".
// A record that runs past its block: cut by the end of the file if that block
// is the file's last, partial one (the reader's eof_, :236-239), else "bad
// record length" (:230-235).
__device__ __forceinline__ uint32_t log_cut_status(uint64_t o, uint64_t buf_len) {
  const uint64_t be = log_block_end(o, buf_len);
  return (be == buf_len && (buf_len % kLogBlock) != 0) ? NOVA_LOG_TRUNCATED : NOVA_LOG_BAD_LENGTH;
}
__device__ __forceinline__ uint32_t log_status(uint64_t o, uint32_t length, uint32_t type,
                                               uint64_t buf_len) {
  if (o + 7 + length > log_block_end(o, buf_len)) return log_cut_status(o, buf_len);
  if (type == 0 && length == 0) return NOVA_LOG_ZERO_RECORD;  // :241-247 skipped
  return NOVA_LOG_OK;
}
__device__ __forceinline__ bool log_header_fits(uint64_t o, uint64_t buf_len) {
  return o + 7 <= log_block_end(o, buf_len);
}
// Status of a record whose header does not fit (fewer than 7 bytes left,
// :196-220): at or past the end of the file, or in its last partial block, the
// read ends (EOF, :204-211); in a full block the bytes are the block's
// trailer, skipped silently (:198-203).  Neither is reported.
__device__ __forceinline__ uint32_t log_nohdr_status(uint64_t o, uint64_t buf_len) {
  if (o >= buf_len) return NOVA_LOG_TRUNCATED;
  const uint64_t be = log_block_end(o, buf_len);
  return (be == buf_len && (buf_len % kLogBlock) != 0) ? NOVA_LOG_TRUNCATED : NOVA_LOG_BLOCK_TRAILER;
}

// ---- device helpers --------------------------------------------------------

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32 (gfx950)
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;



// 16-byte load through the global (not flat) address space.  Block bytes are
// read exactly once, so production loads carry the nt policy: on gfx950 it
// bypasses L1 and streams ~9% faster than the default policy at every block
// size measured (tools/ceiling.py).
template <int VAR = 0>
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  u32x4 v;
  if constexpr ((VAR & kVarCached) != 0) {
    v = *reinterpret_cast<gu32x4*>(addr);
  } else if constexpr ((VAR & kVarLdSys) != 0) {  // diagnostics A/B: sc0 sc1 (system scope)
    v = *reinterpret_cast<volatile gu32x4*>(addr);
  } else if constexpr ((VAR & kVarLdDev) != 0) {  // diagnostics A/B: sc1 (device scope), 2 x 8 B
    typedef __attribute__((address_space(1))) uint64_t gu64a;
    const uint64_t lo = __hip_atomic_load(reinterpret_cast<gu64a*>(addr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(reinterpret_cast<gu64a*>(addr + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v.x = (uint32_t)lo;
    v.y = (uint32_t)(lo >> 32);
    v.z = (uint32_t)hi;
    v.w = (uint32_t)(hi >> 32);
  } else {
    v = __builtin_nontemporal_load(reinterpret_cast<gu32x4*>(addr));
  }
  return make_uint4(v.x, v.y, v.z, v.w);
}

// A scalar-typed load of caller memory; NT: non-temporal (bypasses L1), as the
// persistent engine needs for buffers a caller may rewrite between requests.
template <bool NT, typename T>
__device__ __forceinline__ T ld_nt(const T* a) {
  if constexpr (NT)
    return __builtin_nontemporal_load((const __attribute__((address_space(1))) T*)a);
  else
    return *a;
}

// Read a dword at an absolute LDS byte address.  The kernel holds no static
// __shared__ objects, so the dynamic LDS region starts at address 0 and the
// v_perm-built table address is used as is (no base add per lookup).
__device__ __forceinline__ uint32_t lds_u32(const uint8_t* /*lds*/, uint32_t byte_addr) {
  return *reinterpret_cast<__attribute__((address_space(3))) const uint32_t*>(byte_addr);
}

// 4-lookup operator application from a [4][256] table in global memory.
__device__ __forceinline__ uint32_t gapply(const uint32_t* __restrict__ t, uint32_t x) {
  return t[x & 255] ^ t[256 + ((x >> 8) & 255)] ^ t[512 + ((x >> 16) & 255)] ^ t[768 + (x >> 24)];
}

// Same from a tree level held in LDS (non-replicated, used once per unit).
__device__ __forceinline__ uint32_t tapply(const uint8_t* lds, int level, uint32_t x) {
  const uint32_t* t = reinterpret_cast<const uint32_t*>(lds + kMainBytes + level * kTreeBytes);
  return t[x & 255] ^ t[256 + ((x >> 8) & 255)] ^ t[512 + ((x >> 16) & 255)] ^ t[768 + (x >> 24)];
}

// Byte-selector for v_perm_b32(x, lo, sel): out byte0 = lo.byte0 (replica
// offset, table parity bit 7), out byte1 = x.byte k (table row), out byte2 =
// lo.byte2 (64 KiB half), out byte3 = 0.
template <int K>
struct Sel {
  static constexpr uint32_t v = 0x0c020000u | ((4u + K) << 8);
};

// One stream step: c = w ^ M_S(c) via the replicated LDS tables.
template <int VAR = 0>
__device__ __forceinline__ uint32_t step(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lo0,
                                         uint32_t lo1, uint32_t lo2, uint32_t lo3) {
  if constexpr ((VAR & kVarNoLookup) != 0) return ((c << 1) | (c >> 31)) ^ w;  // keeps c live
  const uint32_t a0 = __builtin_amdgcn_perm(c, lo0, Sel<0>::v);
  const uint32_t a1 = __builtin_amdgcn_perm(c, lo1, Sel<1>::v);
  const uint32_t a2 = __builtin_amdgcn_perm(c, lo2, Sel<2>::v);
  const uint32_t a3 = __builtin_amdgcn_perm(c, lo3, Sel<3>::v);
  const uint32_t t0 = lds_u32(lds, a0), t1 = lds_u32(lds, a1);
  const uint32_t t2 = lds_u32(lds, a2), t3 = lds_u32(lds, a3);
  return xor3(xor3(t0, t1, t2), t3, w);
}

// Four swaths (16 B per lane each) into the lane's four stream registers.
template <int VAR = 0>
__device__ __forceinline__ void fold4(const uint8_t* lds, uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                      uint32_t& c3, const uint4& d0, const uint4& d1,
                                      const uint4& d2, const uint4& d3, uint32_t lo0, uint32_t lo1,
                                      uint32_t lo2, uint32_t lo3) {
  c0 = step<VAR>(lds, c0, d0.x, lo0, lo1, lo2, lo3);
  c1 = step<VAR>(lds, c1, d0.y, lo0, lo1, lo2, lo3);
  c2 = step<VAR>(lds, c2, d0.z, lo0, lo1, lo2, lo3);
  c3 = step<VAR>(lds, c3, d0.w, lo0, lo1, lo2, lo3);
  c0 = step<VAR>(lds, c0, d1.x, lo0, lo1, lo2, lo3);
  c1 = step<VAR>(lds, c1, d1.y, lo0, lo1, lo2, lo3);
  c2 = step<VAR>(lds, c2, d1.z, lo0, lo1, lo2, lo3);
  c3 = step<VAR>(lds, c3, d1.w, lo0, lo1, lo2, lo3);
  c0 = step<VAR>(lds, c0, d2.x, lo0, lo1, lo2, lo3);
  c1 = step<VAR>(lds, c1, d2.y, lo0, lo1, lo2, lo3);
  c2 = step<VAR>(lds, c2, d2.z, lo0, lo1, lo2, lo3);
  c3 = step<VAR>(lds, c3, d2.w, lo0, lo1, lo2, lo3);
  c0 = step<VAR>(lds, c0, d3.x, lo0, lo1, lo2, lo3);
  c1 = step<VAR>(lds, c1, d3.y, lo0, lo1, lo2, lo3);
  c2 = step<VAR>(lds, c2, d3.z, lo0, lo1, lo2, lo3);
  c3 = step<VAR>(lds, c3, d3.w, lo0, lo1, lo2, lo3);
}

// One swath into the lane's four stream registers with all 16 table lookups
// issued before any is consumed.  Written as four step() calls, the compiler
// serialises the four independent chains on the LDS latency (one word's four
// lookups in flight at a time: seen in the rounds kernel's ISA); the
// scheduling barrier keeps the reads ahead of the xors.
template <int VAR = 0>
__device__ __forceinline__ void swath4(const uint8_t* lds, uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                       uint32_t& c3, const uint4& d, uint32_t lo0, uint32_t lo1,
                                       uint32_t lo2, uint32_t lo3) {
  if constexpr ((VAR & kVarNoLookup) != 0) {
    c0 = step<VAR>(lds, c0, d.x, lo0, lo1, lo2, lo3);
    c1 = step<VAR>(lds, c1, d.y, lo0, lo1, lo2, lo3);
    c2 = step<VAR>(lds, c2, d.z, lo0, lo1, lo2, lo3);
    c3 = step<VAR>(lds, c3, d.w, lo0, lo1, lo2, lo3);
    return;
  }
#define NOVA_ADDR4(c, p)                                                   \
  const uint32_t p##0 = __builtin_amdgcn_perm(c, lo0, Sel<0>::v);          \
  const uint32_t p##1 = __builtin_amdgcn_perm(c, lo1, Sel<1>::v);          \
  const uint32_t p##2 = __builtin_amdgcn_perm(c, lo2, Sel<2>::v);          \
  const uint32_t p##3 = __builtin_amdgcn_perm(c, lo3, Sel<3>::v);
  NOVA_ADDR4(c0, a) NOVA_ADDR4(c1, b) NOVA_ADDR4(c2, e) NOVA_ADDR4(c3, f)
#undef NOVA_ADDR4
  const uint32_t ta0 = lds_u32(lds, a0), ta1 = lds_u32(lds, a1), ta2 = lds_u32(lds, a2),
                 ta3 = lds_u32(lds, a3);
  const uint32_t tb0 = lds_u32(lds, b0), tb1 = lds_u32(lds, b1), tb2 = lds_u32(lds, b2),
                 tb3 = lds_u32(lds, b3);
  const uint32_t te0 = lds_u32(lds, e0), te1 = lds_u32(lds, e1), te2 = lds_u32(lds, e2),
                 te3 = lds_u32(lds, e3);
  const uint32_t tf0 = lds_u32(lds, f0), tf1 = lds_u32(lds, f1), tf2 = lds_u32(lds, f2),
                 tf3 = lds_u32(lds, f3);
  __builtin_amdgcn_sched_barrier(0);
  c0 = xor3(xor3(ta0, ta1, ta2), ta3, d.x);
  c1 = xor3(xor3(tb0, tb1, tb2), tb3, d.y);
  c2 = xor3(xor3(te0, te1, te2), te3, d.z);
  c3 = xor3(xor3(tf0, tf1, tf2), tf3, d.w);
}

template <int VAR = 0>
__device__ __forceinline__ void fold4w(const uint8_t* lds, uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                       uint32_t& c3, const uint4& d0, const uint4& d1,
                                       const uint4& d2, const uint4& d3, uint32_t lo0, uint32_t lo1,
                                       uint32_t lo2, uint32_t lo3) {
  swath4<VAR>(lds, c0, c1, c2, c3, d0, lo0, lo1, lo2, lo3);
  swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
  swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
  swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
}

// The stream kernel's fold: fold4 (its compiled form keeps two chains' lookups
// in flight) or, with kVarWide, fold4w.
template <int VAR = 0>
__device__ __forceinline__ void fold4s(const uint8_t* lds, uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                       uint32_t& c3, const uint4& d0, const uint4& d1,
                                       const uint4& d2, const uint4& d3, uint32_t lo0, uint32_t lo1,
                                       uint32_t lo2, uint32_t lo3) {
  if constexpr ((VAR & kVarWide) != 0)
    fold4w<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
  else
    fold4<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
}

// Edge masking in 32-bit arithmetic.  For a 16-B piece at address a:
//   h = u0 - a: bytes [0, h) precede the unit and are dropped, and the bytes
//     of ~init that sit at [u0, u0+4) are xor-ed in (the piece holds a head
//     byte iff -4 < h < 16);
//   t = u1 - a: bytes [t, 16) follow the unit and are dropped (0 < t < 16).
// rel32 clamps u - a to [-4, hi]; values outside keep their meaning.
__device__ __forceinline__ int32_t rel32(uint64_t u, uint64_t a, int32_t hi) {
  const int64_t d = (int64_t)(u - a);
  return d < -4 ? -4 : (d > hi ? hi : (int32_t)d);
}
__device__ __forceinline__ bool is_head(int32_t h) { return (uint32_t)(h + 3) < 19u; }
__device__ __forceinline__ bool is_tail(int32_t t) { return (uint32_t)(t - 1) < 15u; }
// the word at offset 4j of a head piece: r = h - 4j
__device__ __forceinline__ uint32_t head_word(uint32_t w, int32_t r, uint32_t ninit) {
  const uint32_t keep = r <= 0 ? ~0u : (r >= 4 ? 0u : (~0u << (8 * r)));
  uint32_t iv = 0;
  if (r >= 0 && r < 4) iv = ninit << (8 * r);
  else if (r < 0 && r > -4) iv = ninit >> (-8 * r);
  return (w & keep) ^ iv;
}
__device__ __forceinline__ uint4 head_piece(uint4 d, int32_t h, uint32_t ninit) {
  d.x = head_word(d.x, h, ninit);
  d.y = head_word(d.y, h - 4, ninit);
  d.z = head_word(d.z, h - 8, ninit);
  d.w = head_word(d.w, h - 12, ninit);
  return d;
}
// keep bytes [0, r) of the word at offset 4j of a tail piece (r = t - 4j)
__device__ __forceinline__ uint32_t tail_word(uint32_t w, int32_t r) {
  return r >= 4 ? w : (r <= 0 ? 0u : (w & ((1u << (8 * r)) - 1u)));
}
__device__ __forceinline__ uint4 tail_piece(uint4 d, int32_t t) {
  d.x = tail_word(d.x, t);
  d.y = tail_word(d.y, t - 4);
  d.z = tail_word(d.z, t - 8);
  d.w = tail_word(d.w, t - 12);
  return d;
}
__device__ __forceinline__ uint4 edge_piece(uint4 d, int32_t h, int32_t t, uint32_t ninit) {
  if (is_head(h)) d = head_piece(d, h, ninit);
  if (is_tail(t)) d = tail_piece(d, t);
  return d;
}

// Bitwise byte step for the (rare) tiny-block and type-byte paths.
__device__ __forceinline__ uint32_t byte_step(uint32_t l, uint32_t b) {
  l ^= b;
#pragma unroll
  for (int i = 0; i < 8; i++) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
  return l;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) {
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;  // util/crc32c.h:28-31
}
__device__ __forceinline__ uint32_t unmask_crc(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;  // util/crc32c.h:34-37
  return (r >> 17) | (r << 15);
}
// Trailer [type][LE32 masked crc] (table/format.h:103, table/table_builder.cc:202-206):
// one byte store plus one unaligned dword store instead of five byte stores.
// gfx950 global memory runs in unaligned mode (the backend emits a plain
// global_store_dword for an align-1 u32); a store that straddles a 128-B line
// is split by the hardware.  With the TableBuilder quirk the dword's top byte is '!'.
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
__device__ __forceinline__ void store_u32_unaligned(uint8_t* d, uint32_t v) {
  *(__attribute__((address_space(1))) u32_unaligned*)d = v;
}
__device__ __forceinline__ void store_trailer(uint8_t* d, uint32_t type, uint32_t m, bool quirk) {
  *(__attribute__((address_space(1))) uint8_t*)d = (uint8_t)type;
  store_u32_unaligned(d + 1, quirk ? ((m & 0x00ffffffu) | ((uint32_t)'!' << 24)) : m);
}

// Write-through stores (agent scope: the line goes to memory, not just this
// XCD's L2) for the persistent engine's results: once its wave has drained
// them (s_waitcnt vmcnt(0)) they are where a copy or a kernel of any stream
// reads them, with no L2 write-back (a per-chunk release fence, buffer_wbl2,
// serialised the engine at ~15 us per request).
template <typename T>
__device__ __forceinline__ void st_through(T* a, T v) {
  __hip_atomic_store((__attribute__((address_space(1))) T*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_trailer_through(uint8_t* d, uint32_t type, uint32_t m, bool quirk) {
  const uint32_t w = quirk ? ((m & 0x00ffffffu) | ((uint32_t)'!' << 24)) : m;
  st_through(d, (uint8_t)type);
  st_through(d + 1, (uint8_t)w);
  st_through(d + 2, (uint8_t)(w >> 8));
  st_through(d + 3, (uint8_t)(w >> 16));
  st_through(d + 4, (uint8_t)(w >> 24));
}

// Patch the NB little-endian bytes of tv (a trailer: type | LE32 << 8, NB 5;
// a log header's CRC field, NB 4) at address u1 into the 16-B line at address
// pa (the line's other bytes keep d).
template <int NB = 5>
__device__ __forceinline__ uint4 patch_trailer(uint4 d, uint64_t pa, uint64_t u1, uint64_t tv) {
  const int32_t o = (int32_t)(int64_t)(u1 - pa);  // field start relative to the line
  auto dw = [&](uint32_t w, int32_t j) -> uint32_t {
    const int32_t r = 4 * j - o;  // byte of the field at the dword's first byte
    if (r >= NB || r <= -4) return w;
    const uint64_t m40 = (1ull << (8 * NB)) - 1;
    const uint64_t bits = r >= 0 ? tv >> (8 * r) : tv << (-8 * r);
    const uint64_t msk = r >= 0 ? m40 >> (8 * r) : m40 << (-8 * r);
    return (w & ~(uint32_t)msk) | ((uint32_t)bits & (uint32_t)msk);
  };
  return make_uint4(dw(d.x, 0), dw(d.y, 1), dw(d.z, 2), dw(d.w, 3));
}

// LDS helpers for tables at absolute LDS addresses (the dynamic region starts
// at 0): a 4-lookup operator application, 16-B loads/stores, and the 16-B
// prefix masks LM[n] (bytes [0, n) set) indexed by a clamped byte count.
[[maybe_unused]] __device__ __forceinline__ uint32_t lds_apply(uint32_t tab, uint32_t x) {
  const uint32_t t0 = lds_u32(nullptr, tab + ((x & 255u) << 2));
  const uint32_t t1 = lds_u32(nullptr, tab + 1024u + (((x >> 8) & 255u) << 2));
  const uint32_t t2 = lds_u32(nullptr, tab + 2048u + (((x >> 16) & 255u) << 2));
  const uint32_t t3 = lds_u32(nullptr, tab + 3072u + ((x >> 24) << 2));
  return xor3(t0, t1, t2) ^ t3;
}
__device__ __forceinline__ uint4 lds_u128(uint32_t a) {
  const u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const u32x4*>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}
[[maybe_unused]] __device__ __forceinline__ void lds_st128(uint32_t a, uint4 v) {
  u32x4 w;
  w.x = v.x;
  w.y = v.y;
  w.z = v.z;
  w.w = v.w;
  *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(a) = w;
}
// Inverse of one zero-byte step of the reflected register (M_1^-1): the forward
// bit step x' = (x >> 1) ^ (P if x & 1) leaves x & 1 in bit 31 of x' (P has it).
[[maybe_unused]] __device__ __forceinline__ uint32_t unstep_byte(uint32_t x) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t b = x >> 31;
    x = ((x ^ (0x82F63B78u & (0u - b))) << 1) | b;
  }
  return x;
}
__device__ __forceinline__ int32_t clamp16(int32_t x) { return x < 0 ? 0 : (x > 16 ? 16 : x); }

// v of lane (lane ^ K), K a power of two known at compile time, without an
// LDS round trip (__shfl_xor is a ds_bpermute, which also takes LDS bandwidth
// from the table lookups):
//   K <= 8: DPP within a 16-lane row (quad_perm; xor 4 = row_half_mirror after
//     quad_perm [3,2,1,0]; xor 8 = row_mirror after row_half_mirror);
//   K = 16: v_permlane16_swap(v, v) swaps the odd rows of its first operand
//     with the even rows of its second: the first result holds rows
//     (r0, r0, r2, r2) of v, the second (r1, r1, r3, r3), so lane l takes the
//     second in even rows and the first in odd rows;
//   K = 32: v_permlane32_swap(v, v) swaps the upper half of the first operand
//     with the lower half of the second: the first result is (lo, lo), the
//     second (hi, hi); the lower half takes the second.
// (Round 2 tried the swaps with one result for every lane -- a rotation, not
// a lane-xor, for half the lanes -- and dropped them after a wrong CRC;
// tests/test_gpu_parity.py::test_lane_xor pins every K against __shfl_xor.)
template <int K>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (K == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  } else if constexpr (K == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  } else if constexpr (K == 4) {
    return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false),
                                              0x141, 0xF, 0xF, false);
  } else if constexpr (K == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false),
                                              0x140, 0xF, 0xF, false);
  } else if constexpr (K == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((threadIdx.x >> 4) & 1u) ? r[0] : r[1];
  } else {
    static_assert(K == 32, "lane_xor: 1, 2, 4, 8, 16 or 32");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return ((threadIdx.x >> 5) & 1u) ? r[0] : r[1];
  }
}
// max over the wave's 64 lanes (every lane gets it).  The cross-row levels
// stay ds_bpermute (__shfl_xor): same-box A/Bs on the log-verify image
// (rounds kernel, one wave_max per round) measured the permlane-swap form
// (max of both swap results, no lane select) 0.5 points and a DPP + 4 x
// v_readlane + s_max form 0.3 points slower (profiles/r03_ab_wave_max.log).
__device__ __forceinline__ uint32_t wave_max(uint32_t m) {
  m = max(m, (uint32_t)__shfl_xor((int)m, 32));
  m = max(m, (uint32_t)__shfl_xor((int)m, 16));
  m = max(m, lane_xor<8>(m));
  m = max(m, lane_xor<4>(m));
  m = max(m, lane_xor<2>(m));
  return max(m, lane_xor<1>(m));
}

__device__ __forceinline__ uint32_t wave_min(uint32_t m) {
  m = min(m, (uint32_t)__shfl_xor((int)m, 32));
  m = min(m, (uint32_t)__shfl_xor((int)m, 16));
  m = min(m, lane_xor<8>(m));
  m = min(m, lane_xor<4>(m));
  m = min(m, lane_xor<2>(m));
  return min(m, lane_xor<1>(m));
}

// Fold the 4G pending stream words of a lane group (4 per lane, lane q holds
// the words at byte offsets 16q+0,4,8,12 of each 16G-byte swath) into the
// pending word V of the group's last word: in-lane M4, M8, then cross-lane
// M16, M32, ... with xor-shuffles.  Must be called from converged code.
template <int G>
__device__ __forceinline__ uint32_t group_fold(const uint8_t* lds, uint32_t c0, uint32_t c1,
                                               uint32_t c2, uint32_t c3, int q) {
  uint32_t v = tapply(lds, 1, tapply(lds, 0, c0) ^ c1) ^ (tapply(lds, 0, c2) ^ c3);
  auto level = [&](int k, uint32_t o) {  // o: v of lane q ^ 2^k
    const bool right = (q >> k) & 1;
    v = tapply(lds, 2 + k, right ? o : v) ^ (right ? v : o);
  };
  if constexpr (G > 1) level(0, lane_xor<1>(v));
  if constexpr (G > 2) level(1, lane_xor<2>(v));
  if constexpr (G > 4) level(2, lane_xor<4>(v));
  if constexpr (G > 8) level(3, lane_xor<8>(v));
  if constexpr (G > 16) level(4, lane_xor<16>(v));
  if constexpr (G > 32) level(5, lane_xor<32>(v));
  return v;
}

// Process unit [u0,u1) with G lanes; returns the pending word V of the
// virtual message that ends at Eu = roundup16(u1) (identical in all G lanes of
// the group).  Bytes outside [u0,u1) count as zero; t = Eu - u1 trailing pad
// bytes are undone by the caller (M_t^-1).
//   * Steps run on the group's 16G-byte line grid, so each swath is one
//     aligned line (as the rounds kernel: an unaligned grid splits every
//     group-swath over two cache lines).  The steps cover the lines from the
//     one holding u0 to the one holding byte Eu-1.
//   * Pieces before A0 = u0 & ~15 (first step only) read the zero line; the
//     piece(s) holding [u0, u0+4) drop the bytes before u0 and take ~init; the
//     piece holding u1 drops the bytes from u1 on; pieces at or after Eu (last
//     line only) read the zero line and leave their lane's registers unchanged.
//   * Every step's loads are issued while the previous step folds (two
//     register sets, no copies: a copy of a load destination would force a
//     vmcnt(0) drain); edge masking runs on the first two and the last step.
//   * On the line grid lane q holds position (q - e) mod G of the swaths that
//     end at Eu (e = (Eu mod 16G) / 16): the registers are rotated before the
//     group fold.
//   * Units stream back to back: a0..a3 arrive holding this unit's first step
//     (in flight) and leave holding the next unit's [nu0, nu1) first step, issued
//     with this unit's last prefetch.  pre() runs once this unit's loads are in
//     flight (the caller's deferred work for the previous unit overlaps them).
template <int G>
__device__ __forceinline__ void unit_first_addrs(uint64_t u0, uint64_t u1, int q, uint64_t zl,
                                                 uint64_t& x0, uint64_t& x1, uint64_t& x2,
                                                 uint64_t& x3) {
  constexpr uint64_t kStep = 64 * G, kLine = 16 * G;
  const bool ne = u1 > u0;
  const uint64_t Eu = (u1 + 15) & ~15ull;
  const uint64_t A0 = u0 & ~15ull;
  const uint64_t Le = (Eu + kLine - 1) & ~(kLine - 1);
  const uint64_t K4 = ne ? (Le - (A0 & ~(kLine - 1)) + kStep - 1) / kStep : 1;
  const uint64_t p0 = Le - K4 * kStep + 16 * q;
  x0 = (ne && p0 >= A0) ? p0 : zl;
  x1 = (ne && p0 + 16 * G >= A0) ? p0 + 16 * G : zl;
  x2 = (ne && p0 + 32 * G >= A0) ? p0 + 32 * G : zl;
  x3 = (ne && p0 + 48 * G >= A0 && p0 + 48 * G < Eu) ? p0 + 48 * G : zl;
}

template <int G, int VAR = 0, typename Pre>
__device__ __forceinline__ uint32_t unit_pending(const uint8_t* lds, uint64_t u0, uint64_t u1,
                                                 uint32_t ninit, int q, uint32_t lo0,
                                                 uint32_t lo1, uint32_t lo2, uint32_t lo3,
                                                 uint64_t zl, Pre&& pre, uint4& a0, uint4& a1,
                                                 uint4& a2, uint4& a3, uint64_t nu0, uint64_t nu1) {
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  uint32_t e = 0;
  uint64_t x0, x1, x2, x3;  // the next unit's first step
  unit_first_addrs<G>(nu0, nu1, q, zl, x0, x1, x2, x3);
  if (!(u1 > u0)) {
    pre();
    a0 = gload16<VAR>(x0);
    a1 = gload16<VAR>(x1);
    a2 = gload16<VAR>(x2);
    a3 = gload16<VAR>(x3);
  }
  if (u1 > u0) {
    constexpr uint64_t kStep = 64 * G, kLine = 16 * G;
    const uint64_t Eu = (u1 + 15) & ~15ull;
    const uint64_t A0 = u0 & ~15ull;
    const uint64_t Le = (Eu + kLine - 1) & ~(kLine - 1);
    const uint64_t K4 = (Le - (A0 & ~(kLine - 1)) + kStep - 1) / kStep;  // >= 1
    const uint64_t p0 = Le - K4 * kStep + 16 * q;  // the lane's first piece of step 0
    e = (uint32_t)(Eu >> 4) & (uint32_t)(G - 1);
    auto fold_at = [&](uint4 d0, uint4 d1, uint4 d2, uint4 d3, uint64_t s) {
      const uint64_t a = p0 + s * kStep;
      const bool last = s + 1 == K4;  // group-uniform
      if (s <= 1 || last) {           // the only steps holding edge pieces
        const int32_t h = rel32(u0, a, 48 * G + 16), t = rel32(u1, a, 48 * G + 16);
        d0 = edge_piece(d0, h, t, ninit);
        d1 = edge_piece(d1, h - 16 * G, t - 16 * G, ninit);
        d2 = edge_piece(d2, h - 32 * G, t - 32 * G, ninit);
        d3 = edge_piece(d3, h - 48 * G, t - 48 * G, ninit);
      }
      if (last) {
        swath4<VAR>(lds, c0, c1, c2, c3, d0, lo0, lo1, lo2, lo3);
        swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
        swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
        const uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = c3;
        swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
        if (a + 48 * G >= Eu) {  // past the unit's region: no step
          c0 = k0;
          c1 = k1;
          c2 = k2;
          c3 = k3;
        }
      } else if constexpr ((VAR & kVarNarrow) != 0) {
        fold4<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
      } else {
        fold4w<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
      }
    };
    // step 0 (already in a0..a3, unit_first_addrs): pieces before A0 read the
    // zero line; the last line: pieces at or after Eu read it too (they are not
    // in the unit and may be past the buffer)
    const uint64_t lim3 = Eu;
    pre();
    uint64_t s = 0;
    for (; s + 2 <= K4; s += 2) {
      const uint64_t pb = p0 + (s + 1) * kStep;
      const uint4 b0 = gload16<VAR>(pb), b1 = gload16<VAR>(pb + 16 * G);
      const uint4 b2 = gload16<VAR>(pb + 32 * G);
      const uint4 b3 = gload16<VAR>(pb + 48 * G < lim3 ? pb + 48 * G : zl);
      fold_at(a0, a1, a2, a3, s);
      // after this unit's last step the prefetch takes the next unit's first
      const bool more = s + 2 < K4;
      const uint64_t pn = pb + kStep;
      a0 = gload16<VAR>(more ? pn : x0);
      a1 = gload16<VAR>(more ? pn + 16 * G : x1);
      a2 = gload16<VAR>(more ? pn + 32 * G : x2);
      a3 = gload16<VAR>(more ? (pn + 48 * G < lim3 ? pn + 48 * G : zl) : x3);
      fold_at(b0, b1, b2, b3, s + 1);
    }
    if (s < K4) {
      fold_at(a0, a1, a2, a3, s);
      a0 = gload16<VAR>(x0);
      a1 = gload16<VAR>(x1);
      a2 = gload16<VAR>(x2);
      a3 = gload16<VAR>(x3);
    }
  }
  const int src = (threadIdx.x & 63) - q + (int)(((uint32_t)q + e) & (uint32_t)(G - 1));
  c0 = __shfl(c0, src);
  c1 = __shfl(c1, src);
  c2 = __shfl(c2, src);
  c3 = __shfl(c3, src);
  return group_fold<G>(lds, c0, c1, c2, c3, q);
}

// End of a scheduled launch: the last workgroup to finish zeroes the claim
// counters it used (words w*16 for w < gridDim.x) and the finish counter
// (word 1), so the stream's next launch starts from zero without a memset.
// Every claim of every workgroup has returned before that workgroup counts
// itself finished, so nothing touches the counters afterwards.
__device__ __forceinline__ void sched_release(uint32_t* sched) {
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t prev = 0;
    if (threadIdx.x == 0)
      prev = __hip_atomic_fetch_add(sched + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0);
    if (prev == gridDim.x - 1) {
      for (uint32_t w = threadIdx.x; w < gridDim.x; w += 64)
        __hip_atomic_store(sched + w * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x == 0)
        __hip_atomic_store(sched + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Launch prologue: the LDS table image (main tables, tree levels, optional
// byte table), contiguous in LDS, copied with 8 loads in flight per thread.
// A plain copy loop waits on every load before issuing the next: ~20 serial
// L2 round trips per workgroup, a fixed cost that dominated small batches.
__device__ __forceinline__ void lds_fill_tables(uint8_t* lds, const void* tab_main,
                                                const void* tab_tree, uint32_t tree16,
                                                const void* tab_byte, uint32_t byte16,
                                                uint32_t kMain16 = kMainBytes / 16) {
  const uint32_t n16 = kMain16 + tree16 + byte16;
  // per-source base addresses, rebased so that LDS index j reads base + 16 j
  const uint64_t am = (uint64_t)tab_main;
  const uint64_t at = (uint64_t)tab_tree - 16ull * kMain16;
  const uint64_t ab = (uint64_t)tab_byte - 16ull * (kMain16 + tree16);
  uint4* d = reinterpret_cast<uint4*>(lds);
  const uint32_t nt = blockDim.x;
  for (uint32_t i = threadIdx.x; i < n16; i += 8 * nt) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t j = i + k * nt;
      j = j < n16 ? j : n16 - 1;  // clamped: every load issued, stores predicated
      const uint64_t a = j < kMain16 ? am : (j < kMain16 + tree16 ? at : ab);
      v[k] = gload16<kVarCached>(a + 16ull * j);  // default policy: tables stay in L2
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i + k * nt < n16) d[i + k * nt] = v[k];
  }
}

// One claimed chunk of the units kernel (and of the persistent SSTable engine,
// crc32c_engine.hip): lane i < p.chunk owns block chunk * p.chunk + i; the
// chunk's units run in rounds of kGroups (one per lane group), largest first;
// lane i finishes its block.  wpre: the wave's kWaveScratch bytes of LDS.
// kVarEngine (the engine): every load of caller memory (descriptors, block
// bytes, stored CRCs) bypasses L1 -- the engine stays resident between
// requests, so no kernel start invalidates the CU's L1 lines of a buffer the
// caller has since rewritten.
template <int G, int MODE, int VAR = 0>
__device__ __forceinline__ void units_chunk(const uint8_t* lds, const CrcParams& p, uint64_t chunk,
                                            uint32_t* wpre) {
  const int lane = threadIdx.x & 63;
  const int q = lane & (G - 1);   // lane within its group
  const int grp = lane / G;       // group within the wave
  constexpr int kGroups = 64 / G;
  constexpr bool kEng = (VAR & kVarEngine) != 0;
  uint32_t* wacc = wpre + 64;
  uint32_t* wsort = wpre + 32;  // chunk lanes in descending unit-size order
  const uint64_t zl = (uint64_t)p.zline;  // 16 zero bytes
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t extra = (MODE == kVerify) ? 1u : 0u;  // verify covers block + type byte
  {
    // -- prologue: lane i < chunk owns block b = chunk*chunk_size + i
    const uint64_t b = chunk * p.chunk + lane;
    const bool valid = lane < (int)p.chunk && b < p.n_blocks;
    uint64_t a = 0;
    uint32_t n = 0, init = 0;
    uint32_t lstat = NOVA_LOG_OK;  // log modes: record status (log_status)
    uint32_t stored = 0;  // engine, verify: the block's stored CRC, loaded with its descriptor
    bool eng_bad = false;  // engine, verify: this lane's block failed
    if (valid) {
      a = (uint64_t)p.base + (p.offsets ? ld_nt<kEng>(p.offsets + b) : b * p.stride);
      if (MODE == kLogWrite || MODE == kLogVerify) {
        const uint64_t o = a - (uint64_t)p.base;
        if (log_header_fits(o, p.buf_len)) {
          const uint8_t* h = (const uint8_t*)a;  // record header
          const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
          lstat = log_status(o, length, MODE == kLogVerify ? h[6] : 1u, p.buf_len);
          n = lstat == NOVA_LOG_OK ? 1u + length : 0u;
        } else {
          lstat = log_nohdr_status(o, p.buf_len);
        }
        a += 6;  // CRC input starts at the type byte
      } else {
        n = (p.lengths ? ld_nt<kEng>(p.lengths + b) : p.len) + extra;
      }
      init = p.init ? ld_nt<kEng>(p.init + b) : 0u;
      if (kEng && MODE == kVerify) {
        const uint8_t* d = (const uint8_t*)a + n;
        stored = (uint32_t)ld_nt<true>(d) | ((uint32_t)ld_nt<true>(d + 1) << 8) |
                 ((uint32_t)ld_nt<true>(d + 2) << 16) | ((uint32_t)ld_nt<true>(d + 3) << 24);
      }
    }
    const uint32_t ninit = raw ? 0u : ~init;
    // Units: blocks >= seg bytes are cut into floor(n/seg) segments (seg..2seg-1
    // bytes each); shorter blocks are one unit.  A round lasts as long as its
    // longest unit, so the chunk's blocks are ranked by unit size, largest
    // first, and rounds take consecutive units in that order.
    uint32_t nq = 0;
    uint32_t small_crc = 0;
    if (valid) {
      if (n >= 4) {
        nq = (p.seg == 0 || n < p.seg) ? 1u : n / p.seg;
      } else {  // tiny block: bytewise on this lane
        uint32_t l = ninit;
        for (uint32_t i = 0; i < n; i++) l = byte_step(l, ld_nt<kEng>((const uint8_t*)a + i));
        small_crc = raw ? l : ~l;
      }
    }
    const uint32_t key = nq ? n / nq : 0u;  // bytes per unit (0: no units)
    uint32_t rank = 0;                       // position in descending key order
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t kk = __shfl(key, k);
      rank += (kk > key || (kk == key && k < (lane & 15))) ? 1u : 0u;
    }
    if (lane < 16) {
      wsort[rank] = lane;
      wacc[lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // inclusive prefix of unit counts in rank order
    uint32_t ib = __shfl(nq, (int)wsort[lane & 15]);
#pragma unroll
    for (int s = 1; s < 16; s <<= 1) {
      const uint32_t ob = __shfl_up(ib, s);
      if ((lane & 15) >= s) ib += ob;
    }
    const uint32_t total = __shfl(ib, 15);
    if (lane < 16) wpre[lane] = ib;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // -- rounds: each lane group takes one unit.  A unit's contribution
    // M_{seg*j}(M_t^-1 M4 (V)) needs table lookups in global memory; they are
    // deferred to the next unit's first loads (finalize), so the two latencies
    // overlap instead of adding up.
    bool d_on = false;
    uint32_t d_v = 0, d_t = 0;
    uint64_t d_m = 0;
    int d_i = 0;
    auto finalize = [&]() {
      if (d_on) {
        uint32_t c = d_t ? gapply(p.tab_ft + d_t * 1024, d_v) : tapply(lds, 0, d_v);  // M4 in LDS
        uint64_t m = d_m;  // shift in 16-byte units
        while (m) {
          const int bit = __builtin_ctzll(m);
          c = gapply(p.tab_sh16 + bit * 1024, c);
          m &= m - 1;
        }
        atomicXor(&wacc[d_i], c);
        d_on = false;
      }
    };
    // The group's unit of the round starting at r0: [u0,u1), its init, its
    // index j from the block's end and the lane i owning its block.
    struct Unit {
      uint64_t u0, u1;
      uint32_t init, j;
      int i;
      bool active;
    };
    auto unit_at = [&](uint32_t r0) -> Unit {
      Unit t{0, 0, 0, 0, 0, false};
      const uint32_t u = r0 + grp;
      t.active = u < total;
      int r = 0;
#pragma unroll
      for (int s = 8; s > 0; s >>= 1)
        if (wpre[r + s - 1] <= u) r += s;
      if (!t.active) r = 0;
      t.i = (int)wsort[r];  // lane owning the unit's block
      const uint32_t a_lo = __shfl((uint32_t)a, t.i);
      const uint32_t a_hi = __shfl((uint32_t)(a >> 32), t.i);
      const uint32_t bn = __shfl(n, t.i);
      const uint32_t bq = __shfl(nq, t.i);
      const uint32_t binit = __shfl(ninit, t.i);
      const uint32_t bincl = wpre[r];
      const uint64_t ba = ((uint64_t)a_hi << 32) | a_lo;
      t.j = bincl - 1 - u;  // 0 = last unit of the block
      if (t.active) {
        const uint64_t E = ba + bn;
        t.u1 = E - (uint64_t)p.seg * t.j;
        const bool first = (t.j == bq - 1);
        t.u0 = first ? ba : t.u1 - p.seg;
        t.init = first ? binit : 0u;
      }
      return t;
    };
    Unit cur = unit_at(0);
    uint4 a0, a1, a2, a3;  // the current unit's first step, in flight
    {
      uint64_t x0, x1, x2, x3;
      unit_first_addrs<G>(cur.u0, cur.u1, q, zl, x0, x1, x2, x3);
      a0 = gload16<VAR>(x0);
      a1 = gload16<VAR>(x1);
      a2 = gload16<VAR>(x2);
      a3 = gload16<VAR>(x3);
    }
    for (uint32_t r0 = 0; r0 < total; r0 += kGroups) {
      const Unit nxt = unit_at(r0 + kGroups);
      const uint32_t v = unit_pending<G, VAR>(lds, cur.u0, cur.u1, cur.init, q, lo0, lo1, lo2, lo3,
                                              zl, finalize, a0, a1, a2, a3, nxt.u0, nxt.u1);
      // this unit's contribution is folded in during the next unit's first loads
      d_on = cur.active && q == 0;
      d_v = v;
      d_t = (uint32_t)((16 - (cur.u1 & 15)) & 15);
      d_m = (uint64_t)(p.seg >> 4) * cur.j;
      d_i = cur.i;
      cur = nxt;
    }
    finalize();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // -- epilogue: lane i finalises block b
    if (valid) {
      uint32_t crc = (n >= 4) ? (raw ? wacc[lane] : ~wacc[lane]) : small_crc;
      if ((MODE == kLogWrite || MODE == kLogVerify) && lstat != NOVA_LOG_OK) {
        if (MODE == kLogVerify) {  // not read: the status (counted if the reader reports it)
          p.ok_out[b] = (uint8_t)lstat;
          if (lstat == NOVA_LOG_BAD_LENGTH && p.n_bad) atomicAdd(p.n_bad, 1u);
        }
      } else if (MODE == kLogWrite || MODE == kLogVerify) {
        uint8_t* h = (uint8_t*)a - 6;
        const uint32_t m = mask_crc(crc);  // db/log_writer.cc:113
        if (MODE == kLogWrite) {
          h[0] = (uint8_t)m;
          h[1] = (uint8_t)(m >> 8);
          h[2] = (uint8_t)(m >> 16);
          h[3] = (uint8_t)(m >> 24);
        } else {
          const uint32_t stored = (uint32_t)h[0] | ((uint32_t)h[1] << 8) |
                                  ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
          const bool ok = unmask_crc(stored) == crc;  // db/log_reader.cc:254-256
          p.ok_out[b] = ok ? 1 : 0;
          if (!ok && p.n_bad) atomicAdd(p.n_bad, 1u);
        }
      } else if (MODE == kVerify) {
        if (!kEng) {
          const uint8_t* d = (const uint8_t*)a;
          stored = (uint32_t)d[n] | ((uint32_t)d[n + 1] << 8) | ((uint32_t)d[n + 2] << 16) |
                   ((uint32_t)d[n + 3] << 24);
        }
        const bool ok = unmask_crc(stored) == crc;  // table/table.cc:435-437
        if constexpr (kEng) {
          st_through(p.ok_out + b, (uint8_t)(ok ? 1 : 0));
          eng_bad = !ok;
        } else {
          p.ok_out[b] = ok ? 1 : 0;
          if (!ok && p.n_bad) atomicAdd(p.n_bad, 1u);
        }
      } else {
        if (p.flags & NOVA_CRC32C_APPEND_TYPE) {  // table/table_builder.cc:203
          crc = ~byte_step(~crc, (p.flags >> 8) & 0xffu);
        }
        if (MODE == kTrailer) {
          const uint32_t m = mask_crc(crc);
          if constexpr (kEng)
            store_trailer_through((uint8_t*)a + n, (p.flags >> 8) & 0xffu, m,
                                  (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
          else
            store_trailer((uint8_t*)a + n, (p.flags >> 8) & 0xffu, m,
                          (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
        } else {
          if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
          if constexpr (kEng)
            st_through(p.out + b, crc);
          else
            p.out[b] = crc;
        }
      }
    }
    // engine, verify: one add per chunk (system scope: performed in memory,
    // where the caller's next copy reads the counter)
    if constexpr (kEng && MODE == kVerify) {
      const uint32_t nb = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(eng_bad));
      if (lane == 0 && nb && p.n_bad)
        __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t*)p.n_bad, nb, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Launch bound 12 waves (the launch size, kUnitsWaves): 168 VGPRs.  At the
// 16-wave bound the compiler had 128 and spilled 5-7 VGPRs to scratch in every
// instantiation (tools/kernel_meta.py).
constexpr int kUnitsMaxWaves = 12;
template <int G, int MODE, int VAR = 0>
__global__ void __launch_bounds__(kUnitsMaxWaves * 64) crc32c_units_kernel(CrcParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLevels * kTreeBytes / 16, nullptr, 0);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  uint32_t* wpre = reinterpret_cast<uint32_t*>(lds + kMainBytes + kLevels * kTreeBytes +
                                               wave * kWaveScratch);

  // Chunks of p.chunk (<= 16) blocks.  Workgroup w owns the interleaved chunks
  // w, w+nwg, ... and its waves claim them from a per-workgroup counter (one
  // relaxed device-scope atomic per chunk); a wave whose workgroup ran out
  // steals from up to p.steal_limit other workgroups.  Wave k's first chunk is
  // implicit.  (Static chunk assignment left the tail unbalanced, as measured
  // for the streaming kernel in DESIGN.md 3.3.)
  const uint32_t nwg = gridDim.x;
  const uint32_t nwaves = blockDim.x >> 6;
  uint32_t victim = blockIdx.x, tried = 0;
  uint64_t chunk = (uint64_t)wave * nwg + blockIdx.x;
  auto next_chunk = [&]() -> uint64_t {
    for (;;) {
      uint32_t idx = 0;
      if (lane == 0)
        idx = __hip_atomic_fetch_add(p.sched + victim * 16, 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      idx = __builtin_amdgcn_readfirstlane(idx);
      const uint64_t c = ((uint64_t)idx + nwaves) * nwg + victim;
      if (c < p.n_chunks) return c;
      if (++tried >= p.steal_limit + 1) return ~0ull;
      victim = (victim + 1) % nwg;
    }
  };
  if (chunk >= p.n_chunks) chunk = next_chunk();

  for (; chunk != ~0ull; chunk = next_chunk()) {
    units_chunk<G, MODE, VAR>(lds, p, chunk, wpre);
  }
  sched_release(p.sched);
}

// Aligned uniform batches (base, stride 16-B aligned, len a multiple of 64G).
//
// A "round" is kGroups*BPG consecutive blocks (BPG per lane group of a wave).
// Each wave walks its rounds as ONE flat sequence of 4-swath steps, so the
// two-register-set prefetch never stops at a block boundary; the per-block
// fold + store runs between steps while the next block's loads are in flight.
//
// Scheduling is dynamic: per-workgroup claim counters, claimed one round
// ahead, bounded stealing at the tail (see "work distribution" below).  Per-
// wave timestamps showed static partitioning leaves ~20% of wave time idle at
// the tail (XCDs and CUs stream at different speeds).  The counters are left
// zeroed by the previous launch on the stream (sched_release).
template <int G, int VAR = 0>
__global__ void __launch_bounds__(kThreads) crc32c_stream_kernel(CrcParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLevels * kTreeBytes / 16, nullptr, 0);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane & (G - 1);
  const int grp = lane / G;
  constexpr int kGroups = 64 / G;
  const uint32_t nwaves = blockDim.x >> 6;  // waves per workgroup (tunable)
  const uint64_t wid = (uint64_t)blockIdx.x * nwaves + wave;
  const uint64_t n = p.n_blocks;
  const uint64_t R = (n + (uint64_t)kGroups * p.bpg - 1) / ((uint64_t)kGroups * p.bpg);  // rounds
  const uint32_t KG = p.len / (64 * G);            // 4-swath steps per block (even, >= 2)
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint64_t base = (uint64_t)p.base + 16 * q;
  const uint64_t stride = p.stride;
  constexpr uint64_t kStep = 64 * G;  // bytes of one 4-swath step per lane group
  uint64_t t_begin = 0;
  if constexpr ((VAR & kVarStamps) != 0) t_begin = __builtin_amdgcn_s_memrealtime();

  // A round is kGroups*BPG consecutive blocks; lane group grp owns BPG
  // consecutive blocks of it (longer contiguous runs per group).  Blocks past
  // the end clamp to the last block: valid memory, results discarded.
  const uint32_t BPG = p.bpg;
  auto blk_of = [&](uint64_t r, uint32_t j) -> uint64_t {
    return (r * kGroups + grp) * BPG + j;
  };
  auto blk_addr = [&](uint64_t r, uint32_t j) -> uint64_t {
    uint64_t b = blk_of(r, j);
    if (b >= n) b = n - 1;
    return base + b * stride;
  };
  auto init_of = [&](uint64_t r, uint32_t j) -> uint32_t {
    uint64_t b = blk_of(r, j);
    if (b >= n) b = n - 1;
    return p.init[b * p.init_stride];
  };

  // ---- work distribution ----------------------------------------------------
  // Workgroup w owns the interleaved rounds w, w+nwg, w+2*nwg, ... (so the
  // whole grid sweeps memory together: contiguous per-workgroup ranges 16 MiB
  // apart measured ~30% slower, all streams hitting the same HBM channels).
  // Its waves claim those rounds one at a time from a per-workgroup counter in
  // global memory (relaxed device-scope atomic add by lane 0), one round AHEAD
  // of use, so the waves of a CU finish together instead of in age-priority
  // order; when its rounds run out a wave steals from other workgroups'
  // counters.  ~1 claim per round per wave keeps every counter far below its
  // atomic rate.  Wave k's first round is implicit (claim index k); counted
  // claims start after those.  The atomic is issued from inline asm with
  // EXEC = lane 0 so the compiler does not drain vmcnt(0) at a divergent join;
  // its result is read one round later after an explicit vmcnt(7): a round is
  // >= 2 steps, so >= 8 loads were issued after the claim and it is complete
  // once all but the 7 newest ops are; a smaller count would also wait on the
  // block's output store and the fresh prefetch (measured: ~14% slower).  The
  // asm "writes" the result register so the readfirstlane cannot be hoisted.
  const uint32_t nwg = gridDim.x;
  uint32_t victim = blockIdx.x;  // counter currently claimed from
  uint32_t tried = 0;            // victims found exhausted
  uint32_t req_old = 0;
  uint32_t static_idx = 0;
  auto claim = [&](uint32_t v) {
    if constexpr ((VAR & kVarStaticClaims) != 0) {
      req_old = wave + nwaves * (++static_idx) - nwaves;  // wave k takes k, k+nw, ...
      return;
    }
    uint64_t save;
    asm volatile(
        "s_mov_b64 %[save], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add %[old], %[zoff], %[one], %[ctr] sc0\n\t"
        "s_mov_b64 exec, %[save]"
        : [old] "=&v"(req_old), [save] "=&s"(save)
        : [zoff] "v"(v * 64u), [one] "v"(1u), [ctr] "s"(p.sched)  // byte offset: counter v is word 16v
        : "memory");
  };
  // round for claim index idx of workgroup v, or ~0 if v's rounds are exhausted
  auto round_of = [&](uint32_t v, uint32_t idx) -> uint64_t {
    const uint64_t r = ((uint64_t)idx + nwaves) * nwg + v;  // first nwaves claims are implicit
    return r < R ? r : ~0ull;
  };
  // Collect the pending claim; on an exhausted range move to the next victim
  // and claim synchronously (only happens at the tail).  Returns ~0 when all
  // ranges are exhausted.
  auto collect = [&](bool wait_all) -> uint64_t {
    if (wait_all) asm volatile("s_waitcnt vmcnt(0)" : "+v"(req_old) : : "memory");
    else asm volatile("s_waitcnt vmcnt(7)" : "+v"(req_old) : : "memory");
    uint64_t r = round_of(victim, __builtin_amdgcn_readfirstlane(req_old));
    while (r == ~0ull && ++tried < p.steal_limit) {
      victim = (victim + 1) % nwg;
      claim(victim);
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(req_old) : : "memory");
      r = round_of(victim, __builtin_amdgcn_readfirstlane(req_old));
    }
    return r;
  };

  // load cursor: round lr, block lj of the group's BPG blocks, step lk; the
  // wave streams its rounds as one flat sequence of steps (wave-uniform)
  uint64_t lr = (uint64_t)wave * nwg + blockIdx.x;
  bool live = lr < R;
  if (!live) {  // tiny batch: no implicit round; claim synchronously
    claim(victim);
    lr = collect(true);
    live = lr != ~0ull;
  }
  if (live) claim(victim);  // next round in flight
  uint32_t lk = 0, lj = 0;
  uint64_t na = live ? blk_addr(lr, 0) : base;
  auto advance = [&]() {
    if (!live) return;  // exhausted: keep re-reading the current step (discarded)
    if (++lk == KG) {
      lk = 0;
      if (++lj == BPG) {
        lj = 0;
        const uint64_t nr = collect(false);
        if (nr != ~0ull) {
          lr = nr;
          claim(victim);
          na = blk_addr(lr, 0);
        } else {
          live = false;  // keep re-reading the last round (results discarded)
        }
      } else {
        na = blk_addr(lr, lj);
      }
    } else {
      na += kStep;
    }
  };
  // fold cursor: round fr, block fj (lags the load cursor by one step)
  uint64_t fr = lr;
  uint32_t fk = 0, fj = 0;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  uint32_t init_cur = p.init_stride ? init_of(fr, 0) : 0u;
  uint32_t init_next = 0;
  uint64_t fr_next = fr;
  bool fold_live = live;
  auto finish_step = [&]() {
    if (++fk == KG) {  // wave-uniform: every group ends a block on the same step
      const uint32_t v = group_fold<G>(lds, c0, c1, c2, c3, q);
      const uint32_t reg = tapply(lds, 0, v);  // M4: pending -> register at block end
      uint32_t crc = raw ? reg : ~reg;
      if (p.flags & NOVA_CRC32C_APPEND_TYPE) crc = ~byte_step(~crc, (p.flags >> 8) & 0xffu);
      if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
      const uint64_t blk = blk_of(fr, fj);
      if (q == 0 && blk < n) p.out[blk] = crc;
      c0 = c1 = c2 = c3 = 0;
      fk = 0;
      init_cur = init_next;
      if (++fj == BPG) {
        fj = 0;
        fold_live = fr != fr_next;  // the load cursor moved on to another round
        fr = fr_next;
      }
    }
  };
  const bool has_init = p.init_stride != 0;  // uniform; NULL init needs no loads
  auto note_block = [&]() {  // called right after loading step 0 of block (lr, lj)
    if (lj == 0) fr_next = lr;
    if (has_init) init_next = init_of(lr, lj);
  };

  if (live) {
    uint4 a0 = gload16<VAR>(na), a1 = gload16<VAR>(na + 16 * G);
    uint4 a2 = gload16<VAR>(na + 32 * G), a3 = gload16<VAR>(na + 48 * G);
    advance();
    for (;;) {
      if (lk == 0 && live) note_block();
      uint4 b0 = gload16<VAR>(na), b1 = gload16<VAR>(na + 16 * G);
      uint4 b2 = gload16<VAR>(na + 32 * G), b3 = gload16<VAR>(na + 48 * G);
      const bool b_live = live;
      advance();
      if (fk == 0 && q == 0 && !raw) a0.x ^= ~init_cur;  // Extend init -> word 0
      fold4s<VAR>(lds, c0, c1, c2, c3, a0, a1, a2, a3, lo0, lo1, lo2, lo3);
      finish_step();
      if (!fold_live) break;
      if (!b_live && fk == 0 && fj == 0) break;
      if (lk == 0 && live) note_block();
      a0 = gload16<VAR>(na);
      a1 = gload16<VAR>(na + 16 * G);
      a2 = gload16<VAR>(na + 32 * G);
      a3 = gload16<VAR>(na + 48 * G);
      const bool a_live = live;
      advance();
      if (fk == 0 && q == 0 && !raw) b0.x ^= ~init_cur;
      fold4s<VAR>(lds, c0, c1, c2, c3, b0, b1, b2, b3, lo0, lo1, lo2, lo3);
      finish_step();
      if (!fold_live) break;
      if (!a_live && fk == 0 && fj == 0) break;
    }
  }
  if constexpr ((VAR & kVarStamps) != 0) {
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && p.stamps) {
      p.stamps[3 * wid] = t_begin;
      p.stamps[3 * wid + 1] = t_end;
      p.stamps[3 * wid + 2] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    }
  }
  sched_release(p.sched);
}


// One step of a lane group in the rounds / burst kernels (and the
// diagnostics flat kernel): its loaded pieces and the block it belongs to.
struct FlatSet {
  uint4 d0, d1, d2, d3;  // the step's four swaths (16 B per lane each)
  uint4 t, t2;           // tail line(s) at E (valid on the block's last step)
  uint64_t pa;           // group base address of the step
  uint64_t u0, u1, rec;  // the block's CRC input range and its index
  uint32_t ninit, st;    // ~init (0 in RAW mode); stored CRC (log verify)
  bool valid, last;
  bool head;             // rounds kernel: the step holds a byte of [u0, u0+4) (group-uniform)
  bool l3;               // rounds kernel: the lane's last-swath piece is in the region
  bool wsec;             // rounds kernel, trailer writer: t2 holds this lane's sector piece
  uint32_t slot;         // rounds kernel (chunk epilogue): the block's sorted slot in its chunk
  bool cend;             // rounds kernel (chunk epilogue): the chunk's last round ends here
  uint32_t skip;         // rounds kernel: leading swaths of a round's first step no lane needs (0-3)
};

constexpr uint64_t kNoChunk = ~0ull;
constexpr int kFlatMaxWaves = 12;  // 3 waves per SIMD: up to 168 VGPRs, no spills
constexpr int kFlatThreads = kFlatMaxWaves * 64;

__device__ __forceinline__ uint32_t sel5(uint32_t k, uint32_t a, uint32_t b, uint32_t c,
                                         uint32_t d, uint32_t e) {
  return k == 0 ? a : k == 1 ? b : k == 2 ? c : k == 3 ? d : e;
}


// A block's result from the group's pending word v (its region ended at
// E = u1 & ~15): finish the register with the tail bytes [E,u1), add M_n(~init)
// for blocks shorter than 4 bytes, apply the mode's epilogue.  The memory
// write is returned (wb_*) and issued later (write_result).
// kTree: LDS byte offset of the tree's level 0 (M4).
__device__ __forceinline__ uint32_t lapply(const uint8_t* t, uint32_t x) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(t);
  return w[x & 255] ^ w[256 + ((x >> 8) & 255)] ^ w[512 + ((x >> 16) & 255)] ^ w[768 + (x >> 24)];
}

template <int MODE, uint32_t kTree = kMainBytes>
__device__ __forceinline__ void finish_block(const uint8_t* lds, uint32_t byte_tab, const CrcParams& p,
                                             bool raw, uint32_t v, const FlatSet& Y, uint64_t& wb_a,
                                             uint32_t& wb_v) {
  constexpr bool kLog = MODE == kLogWrite || MODE == kLogVerify;
  const uint64_t E = Y.u1 & ~15ull;
  const uint32_t nb = (uint32_t)(Y.u1 - E);
  const uint8_t* m4 = lds + kTree;
  uint32_t R = lapply(m4, v);  // register at E
  {
    // The tail line's bytes from u1 on are never consumed below (whole words
    // only below nb, then nb & 3 single bytes), so only the head edge (a block
    // inside this line) and ~init need masking.
    const int32_t ht = rel32(Y.u0, E, 16);
    const uint32_t w0 = head_word(Y.t.x, ht, Y.ninit);
    const uint32_t w1 = head_word(Y.t.y, ht - 4, Y.ninit);
    const uint32_t w2 = head_word(Y.t.z, ht - 8, Y.ninit);
    const uint32_t w3 = head_word(Y.t.w, ht - 12, Y.ninit);
    uint32_t r;
    r = lapply(m4, R ^ w0);
    R = nb >= 4 ? r : R;
    r = lapply(m4, R ^ w1);
    R = nb >= 8 ? r : R;
    r = lapply(m4, R ^ w2);
    R = nb >= 12 ? r : R;
    const uint32_t wl = sel5(nb >> 2, w0, w1, w2, w3, 0u);
    const uint32_t nr = nb & 3u;
    r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ wl) & 255u) * 4u);
    R = nr >= 1 ? r : R;
    r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ (wl >> 8)) & 255u) * 4u);
    R = nr >= 2 ? r : R;
    r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ (wl >> 16)) & 255u) * 4u);
    R = nr >= 3 ? r : R;
  }
  // n < 4: the data ran from a zero register; add the init's part M_n(~init)
  // (no loads here: a load in this branch would make the compiler drain
  // the prefetch at the loop head).
  const uint32_t nn = (uint32_t)(Y.u1 - Y.u0);
  if (nn < 4 && !raw) {
    uint32_t l = ~((kLog || MODE == kTrailer) ? 0u : Y.st);  // (trailer mode: Y.st is the piece eligibility)
    for (uint32_t i = 0; i < 3; i++) {
      const uint32_t r = (l >> 8) ^ lds_u32(lds, byte_tab + (l & 255u) * 4u);
      l = i < nn ? r : l;
    }
    R ^= l;
  }
  uint32_t crc = raw ? R : ~R;
  if constexpr (kLog) {
    const bool status_only = Y.u1 == Y.u0;  // a record not read: Y.st holds its status
    wb_a = status_only ? 0ull : Y.u0 - 6;  // log write: nothing is written for it
    wb_v = mask_crc(crc);  // db/log_writer.cc:113
    if constexpr (MODE == kLogVerify) {
      wb_a = (uint64_t)(p.ok_out + Y.rec);
      wb_v = status_only ? Y.st : (unmask_crc(Y.st) == crc ? 1u : 0u);  // db/log_reader.cc:254-256
    }
  } else if constexpr (MODE == kVerify) {
    const uint32_t k = nb >> 2;
    const uint32_t wlo = sel5(k, Y.t.x, Y.t.y, Y.t.z, Y.t.w, Y.t2.x);
    const uint32_t whi = sel5(k, Y.t.y, Y.t.z, Y.t.w, Y.t2.x, Y.t2.y);
    const uint32_t stored = __builtin_amdgcn_alignbyte(whi, wlo, nb & 3u);
    wb_a = (uint64_t)(p.ok_out + Y.rec);
    wb_v = unmask_crc(stored) == crc ? 1u : 0u;  // table/table.cc:435-437
  } else {
    if (p.flags & NOVA_CRC32C_APPEND_TYPE) crc = ~byte_step(~crc, (p.flags >> 8) & 0xffu);
    if constexpr (MODE == kTrailer) {
      wb_a = Y.u1;
      wb_v = mask_crc(crc);
    } else {
      if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
      wb_a = (uint64_t)(p.out + Y.rec);
      wb_v = crc;
    }
  }
}

// Issue a finished block's memory write.  Global (not flat) stores: a flat
// store would also count as an LDS access the table lookups must wait for.
template <int MODE>
__device__ __forceinline__ void write_result(const CrcParams& p, uint64_t wb_a, uint32_t wb_v) {
  typedef __attribute__((address_space(1))) uint8_t gu8;
  typedef __attribute__((address_space(1))) uint32_t gu32;
  if constexpr (MODE == kLogWrite) {
    if (wb_a) store_u32_unaligned((uint8_t*)wb_a, wb_v);
  } else if constexpr (MODE == kLogVerify) {
    *(gu8*)wb_a = (uint8_t)wb_v;
    if ((wb_v == NOVA_LOG_CHECKSUM_MISMATCH || wb_v == NOVA_LOG_BAD_LENGTH) && p.n_bad)
      atomicAdd(p.n_bad, 1u);
  } else if constexpr (MODE == kVerify) {
    *(gu8*)wb_a = (uint8_t)wb_v;
    if (!wb_v && p.n_bad) atomicAdd(p.n_bad, 1u);
  } else if constexpr (MODE == kTrailer) {
    store_trailer((uint8_t*)wb_a, (p.flags >> 8) & 0xffu, wb_v, (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
  } else {
    *(gu32*)wb_a = wb_v;
  }
}



// The chunk epilogue's two halves (rounds kernel, lane-parallel per block).
// R(u1) = M_nb(R(E)) ^ tail_raw for the block's last nb = u1 - E < 16 bytes
// (E = u1 & ~15): tail_raw is those bytes run from a zero register, with the
// head edge of a block that starts inside the tail line (bytes before u0
// dropped, ~init at [u0, u0+4)) -- the same steps as finish_block, split by
// linearity so the data part runs when the block's descriptor is decoded.
template <uint32_t kTree>
__device__ __forceinline__ uint32_t tail_raw(const uint8_t* lds, uint32_t byte_tab, uint4 t, uint32_t nb,
                                             int32_t ht, uint32_t ninit) {
  const uint8_t* m4 = lds + kTree;
  const uint32_t w0 = head_word(t.x, ht, ninit), w1 = head_word(t.y, ht - 4, ninit);
  const uint32_t w2 = head_word(t.z, ht - 8, ninit), w3 = head_word(t.w, ht - 12, ninit);
  uint32_t R = 0, r;
  r = lapply(m4, w0);
  R = nb >= 4 ? r : R;
  r = lapply(m4, R ^ w1);
  R = nb >= 8 ? r : R;
  r = lapply(m4, R ^ w2);
  R = nb >= 12 ? r : R;
  const uint32_t wl = sel5(nb >> 2, w0, w1, w2, w3, 0u);
  const uint32_t nr = nb & 3u;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ wl) & 255u) * 4u);
  R = nr >= 1 ? r : R;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ (wl >> 8)) & 255u) * 4u);
  R = nr >= 2 ? r : R;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + ((R ^ (wl >> 16)) & 255u) * 4u);
  R = nr >= 3 ? r : R;
  return R;
}
// M_nb(R) for nb < 16 zero bytes (M4 word steps, then byte steps).
template <uint32_t kTree>
__device__ __forceinline__ uint32_t shift_nb(const uint8_t* lds, uint32_t byte_tab, uint32_t R, uint32_t nb) {
  const uint8_t* m4 = lds + kTree;
  uint32_t r;
  r = lapply(m4, R);
  R = nb >= 4 ? r : R;
  r = lapply(m4, R);
  R = nb >= 8 ? r : R;
  r = lapply(m4, R);
  R = nb >= 12 ? r : R;
  const uint32_t nr = nb & 3u;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + (R & 255u) * 4u);
  R = nr >= 1 ? r : R;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + (R & 255u) * 4u);
  R = nr >= 2 ? r : R;
  r = (R >> 8) ^ lds_u32(lds, byte_tab + (R & 255u) * 4u);
  R = nr >= 3 ? r : R;
  return R;
}

// ---- crc32c_rounds_kernel<G, MODE> ---------------------------------------------
// Variable-length batches in ROUNDS: the wave's lane groups take kGroups blocks
// at a time, all padded to the round's line count (its largest block, end-
// aligned, so shorter blocks start later on zero pieces that leave a zero
// register unchanged).  Every group starts and ends the round together, so the
// per-block work (group fold, tail, epilogue) runs once per round for all
// groups, not divergently per block as in the flat kernel; the loads stream
// across rounds and chunks as in the stream kernel.  For the rounds to be
// even, each claimed chunk is sorted by line count, largest first.
//
// Chunk epilogue (default; kVarRoundEpi keeps the per-round form): when a
// chunk's descriptors are decoded, each lane (one block per lane) loads its
// block's tail line and folds the 0..15 tail bytes into one word (tail_raw);
// a round's end stores only each group's pending word in LDS; after the
// chunk's last round, lane l finishes slot l's block -- register at E, tail,
// init of a block under 4 bytes, mask, store or compare -- for all 64 blocks
// at once.  The per-block work no longer runs once per round in 8 lanes per
// group, and the steps load no tail lines.



// The per-block-init variant (kVarInit) carries the general head masking: at
// the 12-wave bound (168 VGPRs) it spilled 6 VGPRs, so it launches 8 waves.
constexpr int kInitMaxWaves = 8;
template <int G, int MODE, int VAR = 0>
__global__ void __launch_bounds__((VAR & kVarInit) ? kInitMaxWaves * 64 : (VAR & kVarW16) ? 1024 : kFlatThreads)
    crc32c_rounds_kernel(CrcParams p0) {
  CrcParams p = p0;  // the log-stream follow-up narrows the batch below
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  constexpr uint32_t kByteTab = kMainBytes + kLevels * kTreeBytes;
  constexpr bool kLog = MODE == kLogWrite || MODE == kLogVerify;
  constexpr bool kTail2 = MODE == kVerify;
  constexpr uint64_t kStep = 64 * G;
  constexpr uint32_t kGroups = 64 / G;
  static_assert(kByteTab == kMainBytes + kLevels * kTreeBytes, "byte table follows the tree");
  constexpr bool kDiag = (VAR & kVarDiag) != 0;  // diagnostics instantiation (crc32c_diag.hip)
  constexpr bool kBatch = (VAR & (kVarRoundEpi | kVarNoTail)) == 0;  // chunk epilogue
  if (kDiag && p.gate) {  // follow-up of the log-stream kernel
    // gate[0]: precondition flag -> the whole batch; else gate[2] leftover
    // records listed at p.perm (and the log-stream mismatches fold into n_bad)
    if (*(volatile const uint32_t*)p.gate == 0) {
      if (kLog && blockIdx.x == 0 && threadIdx.x == 0 && p.n_bad && p.ls_bad)
        atomicAdd(p.n_bad, *(volatile const uint32_t*)p.ls_bad);
      const uint32_t nl = *(volatile const uint32_t*)(p.gate + 2);
      if (nl == 0) return;
      p.n_blocks = nl;
      p.n_chunks = (nl + p.chunk - 1) / p.chunk;
    } else {
      p.perm = nullptr;
    }
  }
  // byte table (1 KiB) + 17 x 16-B prefix masks (LM[n] = bytes [0, n)), one image
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLevels * kTreeBytes / 16, p.tab_byte, 64 + 17);
  __syncthreads();
  constexpr uint32_t kLM = kByteTab + 1024u;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane & (G - 1);
  const int grp = lane / G;
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t extra = (MODE == kVerify) ? 1u : 0u;  // verify covers block + type byte
  const uint64_t zl = (uint64_t)p.zline;
  const uint64_t base = (uint64_t)p.base;
  const uint32_t C = p.chunk;  // sorted positions per chunk: R rounds of kGroups, <= 64
  // per-block init values (store mode with an init array): the general head
  // masking, in its own instantiation (the common path keeps fewer registers)
  constexpr bool any_init = MODE == kStore && (VAR & kVarInit) != 0;
  const uint32_t R = C / kGroups;
  const uint32_t nwg = gridDim.x;
  const uint32_t nwaves = blockDim.x >> 6;
  // trailer writer: whole-piece trailer stores allowed (trailer_layout_kernel;
  // a block's eligibility comes in as its init word)
  // log write: the same for the 64-B piece holding each record's CRC field
  // (log_window_kernel)
  // (diagnostics instantiation only: the product never passes tr_flag)
  const bool sect = kDiag && (MODE == kTrailer || MODE == kLogWrite) && G >= 8 && p.tr_flag &&
                    *p.tr_flag == 0;

  // ---- chunk claims (as the flat kernel) ---------------------------------------
  uint32_t victim = blockIdx.x, tried = 0, req = 0;
  auto claim = [&](uint32_t v) {
    uint32_t r = 0;
    if (lane == 0)
      r = __hip_atomic_fetch_add(p.sched + v * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    req = r;
  };
  // XCD-aware chunk order for batches in file order: workgroup v runs on XCD
  // v % 8 (round-robin dispatch), so the 8 XCDs take contiguous runs of
  // nwg / 8 chunks of each grid-wide step instead of every 8th chunk, and the
  // lines two neighbouring chunks share are found in one XCD's L2 (a
  // permutation of workgroups: every chunk is still taken exactly once).
  // Same-box A/B (profiles/r04_ab_xcd_chunk_order*.log): SSTable verify +0.5
  // points, trailers +0.4; log verify's sorted windows (p.perm) lost 5 points
  // with it and keep the interleaved order.
  // (diagnostics A/B, wvar 7: the XCD-contiguous order for sorted windows too)
  const uint32_t xper = (nwg % 8 == 0 && (!p.perm || (kDiag && p.wvar == 7))) ? nwg / 8 : 0;
  auto xslot = [&](uint32_t v) -> uint32_t { return xper ? (v % 8) * xper + v / 8 : v; };
  auto chunk_of = [&](uint32_t v, uint32_t idx) -> uint64_t {
    const uint64_t c = ((uint64_t)idx + nwaves) * nwg + xslot(v);
    return c < p.n_chunks ? c : kNoChunk;
  };
  auto collect = [&]() -> uint64_t {
    uint64_t c = chunk_of(victim, __builtin_amdgcn_readfirstlane(req));
    while (c == kNoChunk && ++tried < p.steal_limit + 1) {
      victim = (victim + 1) % nwg;
      claim(victim);
      c = chunk_of(victim, __builtin_amdgcn_readfirstlane(req));
    }
    return c;
  };

  // ---- descriptor pipeline: lane l holds chunk slot l -----------------------------
  // The next chunk is loaded in stages at fixed points of the two-step loop body
  // (stage 1 in a first take, 2 in the second, 3 in the next first, 4 in the next
  // second), each from values loaded a step or more before, into "nxt"
  // registers holding computed values, which a bank switch copies to "cur"
  // without waiting on any load.  A switch that finds nxt not yet ready stalls
  // the load side (empty steps) until it is: no stage ever runs out of order.
  constexpr uint32_t kNone = 0xffffffffu;  // no chunk (chunk ids fit 32 bits: n < 2^38)
  uint32_t t_rec = 0, t_olo = 0, t_ohi = 0, t_len = 0, t_aux = 0;
  // log records: the header's bytes 3-6 (length LE16 at bits 8-23, type at
  // 24-31) and, for verify, bytes 0-3 (the stored masked CRC), as two
  // unaligned dword loads (gfx950 takes them whole: two registers and two
  // loads per record instead of seven byte loads)
  uint32_t hw0 = 0, hw1 = 0;
  uint64_t n_u0 = 0, c_u0 = 0;
  uint32_t n_n = 0, n_rec = 0, n_aux = 0, c_n = 0, c_rec = 0, c_aux = 0;
  uint32_t t_ok = 0, n_ok = 0, c_ok = 0;  // slot holds a block of the batch
  // sorted chunks: each slot's line count, and whether the sort was exact (no
  // bucket clamped), so a round's longest block is its first slot
  uint32_t n_S = 0, c_S = 0;
  bool n_exact = false, c_exact = false;
  uint32_t n_chunk = kNone, c_chunk = kNone, t_chunk = kNone;
  // wave-uniform state packed in one word (fewer scalar registers)
  constexpr uint32_t fReady = 1, fRefill = 2, fDry = 4, fDone = 8, fRoundDone = 16, fClaim = 32;
  constexpr uint32_t fChunkEnd = 64;  // chunk epilogue: the chunk's last step was issued
  uint32_t fl = 0;
  uint32_t stage = 0;  // next pipeline stage due (0: none)
  const uint32_t my = (uint32_t)lane < C ? (uint32_t)lane : C - 1;
  // Sort the loaded chunk's slots by line count, largest first (rank by
  // shuffles, inverse permutation through the wave's LDS scratch), so each
  // round's blocks have similar lengths while the chunk keeps its locality.
  uint32_t* const sortbuf = reinterpret_cast<uint32_t*>(lds + kByteTab + 1024u + 272u) + wave * 64;
  // chunk epilogue: the groups' pending words by sorted slot (after all sort scratch)
  uint32_t* const vbuf = reinterpret_cast<uint32_t*>(lds + kByteTab + 1024u + 272u) + (nwaves + wave) * 64;
  // chunk epilogue: the tail line (and verify's stored-CRC overflow word) of
  // the block being decoded, its tail bytes' contribution per bank, and the
  // chunk being finished ("e" bank: the "c" bank of the previous chunk)
  uint4 t_tl = make_uint4(0, 0, 0, 0);
  uint32_t t_t2 = 0, n_tr = 0, c_tr = 0;
  uint64_t e_u0 = 0;
  uint32_t e_n = 0, e_rec = 0, e_aux = 0, e_ok = 0, e_tr = 0;
  typedef __attribute__((address_space(1))) const uint32_t gcu32;
  auto tail_issue = [&](uint64_t u0, uint32_t n, bool ok) {
    // (diagnostics timing ablation, wvar 4 / 6: the decode stage reads no
    // tail line -- the tail bytes read as zeros, WRONG CRCs)
    if (kDiag && (p.wvar == 4 || p.wvar == 6)) ok = false;
    const uint64_t u1 = u0 + n, E = u1 & ~15ull;
    // verify: the stored CRC starts at u1 (the line is needed even when nb = 0)
    t_tl = gload16<VAR | kVarCached>((ok && (kTail2 || (u1 & 15))) ? E : zl);
    if constexpr (kTail2) t_t2 = *(gcu32*)((ok && u1 + 4 > E + 16) ? E + 16 : zl);
  };
  auto tail_finish = [&]() {  // n_tr; verify: the stored CRC into n_aux
    const uint64_t u1 = n_u0 + n_n, E = u1 & ~15ull;
    const uint32_t nb = (uint32_t)(u1 - E);
    const uint32_t ninit = (raw || n_n < 4) ? 0u : ~(any_init ? n_aux : 0u);
    n_tr = tail_raw<kMainBytes>(lds, kByteTab, t_tl, nb, rel32(n_u0, E, 16), ninit);
    if constexpr (kTail2) {
      const uint32_t k = nb >> 2;
      const uint32_t wlo = sel5(k, t_tl.x, t_tl.y, t_tl.z, t_tl.w, t_t2);
      const uint32_t whi = sel5(k, t_tl.y, t_tl.z, t_tl.w, t_t2, 0u);
      n_aux = __builtin_amdgcn_alignbyte(whi, wlo, nb & 3u);  // table/table.cc:434-436
    }
  };
  auto sort_nxt = [&]() {
    n_ok = t_ok;
    n_exact = false;
    if (!p.sort_local) return;
    uint32_t S = 0;
    if (t_ok) {  // key: lines on the group's line grid (a round costs its longest block's lines)
      const uint64_t E = (n_u0 + n_n) & ~15ull;
      constexpr uint64_t kL = 16 * G;
      const uint64_t Le = (E + (kL - 1)) & ~(kL - 1);
      const uint64_t s64 = (Le - (n_u0 & ~(kL - 1))) / kL;
      S = s64 == 0 ? 1u : (s64 > 0xffffffffull ? 0xffffffffu : (uint32_t)s64);
    }
    // Rank by bucket, largest first: key = lines above the chunk's shortest
    // slot, clamped to kBk - 1 (exact for the spreads that matter: SSTable
    // blocks differ by 1-2 lines, short log records span < 16 lines at G = 4).
    // One ballot + mbcnt per bucket instead of a 64-iteration readlane
    // compare loop (~300 VALU per chunk; 4-5 per log record).
    constexpr uint32_t kBk = G >= 8 ? 32u : 16u;
    const uint32_t mn = wave_min(t_ok ? S : 0xffffffffu);
    const uint32_t bk = t_ok ? min(kBk - 1u, S - mn) : 0u;  // invalid slots: bucket 0, sorted last
    // exact: no key clamped (invalid slots have S = 0, below every valid one)
    n_exact = __builtin_amdgcn_ballot_w64(t_ok && S - mn > kBk - 1u) == 0;
    uint32_t rank = 0, base = 0;
    for (int k = (int)kBk - 1; k >= 0; k--) {
      // (invalid slots -- the chunk's highest lanes -- rank after bucket 0's valid ones)
      const uint64_t m = __builtin_amdgcn_ballot_w64(bk == (uint32_t)k);
      if (m == 0) continue;  // (scalar branch)
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (bk == (uint32_t)k) rank = base + below;
      base += (uint32_t)__builtin_popcountll(m);
    }
    sortbuf[rank] = (uint32_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int src = (int)sortbuf[lane];
    const uint32_t ulo = __shfl((uint32_t)n_u0, src), uhi = __shfl((uint32_t)(n_u0 >> 32), src);
    n_u0 = ((uint64_t)uhi << 32) | ulo;
    n_n = __shfl(n_n, src);
    n_rec = __shfl(n_rec, src);
    n_aux = __shfl(n_aux, src);
    if constexpr (kBatch) n_tr = __shfl(n_tr, src);
    n_ok = __shfl(t_ok, src);
    n_S = __shfl(S, src);
  };
  auto pipe = [&](uint32_t st) {  // run stage st (its inputs are complete or waited for)
    if (st == 1) {
      uint64_t pos = (uint64_t)(t_chunk == kNone ? 0u : t_chunk) * C + my;
      t_ok = (t_chunk != kNone && (uint32_t)lane < C && pos < p.n_blocks) ? 1u : 0u;
      if (pos >= p.n_blocks) pos = p.n_blocks - 1;
      t_rec = p.perm ? p.perm[pos] : (uint32_t)pos;
      stage = 2;
    } else if (st == 2) {
      const uint64_t o = p.offsets[t_rec & p.omask];
      t_olo = (uint32_t)o;
      t_ohi = (uint32_t)(o >> 32);
      if constexpr (!kLog) {
        t_len = p.lengths[t_rec & p.lmask];
        t_aux = p.init[t_rec & p.imask];
      } else if constexpr (MODE == kLogWrite) {
        t_aux = p.init[t_rec & p.imask];  // whole-piece eligibility (log_window_kernel)
      }
      if constexpr (kLog && kDiag) {  // (timing ablation wvar 5 / 6: gap to the next record)
        if (p.wvar == 5 || p.wvar == 6) {
          const uint64_t nx = (uint64_t)t_rec + 1 < p.n_blocks ? (uint64_t)t_rec + 1 : (uint64_t)t_rec;
          const uint64_t gap = p.offsets[nx & p.omask] - o;
          t_len = gap >= 8 && gap < 65536 + 7 ? (uint32_t)(gap - 7) : 1u;
        }
      }
      stage = 3;
    } else if (st == 3) {
      const uint64_t a = base + (((uint64_t)t_ohi << 32) | t_olo) + (uint64_t)t_rec * p.stride;
      if constexpr (kLog) {
        // a header past its log block / the image is not read (bounds, status)
        const uint64_t o = ((uint64_t)t_ohi << 32) | t_olo;
        // (diagnostics timing ablation, wvar 5 / 6: no header loads; the
        // length comes from the next record's offset, stage 2 -- WRONG statuses
        // at block ends and for verify's stored CRCs)
        const bool nohdr = kDiag && (p.wvar == 5 || p.wvar == 6);
        const uint8_t* h = (log_header_fits(o, p.buf_len) && !nohdr) ? (const uint8_t*)a : p.zline;
        typedef __attribute__((address_space(1))) const uint32_t __attribute__((aligned(1))) gu32u;
        hw1 = *(gu32u*)(h + 3);
        if constexpr (MODE == kLogVerify) hw0 = *(gu32u*)h;
        stage = 4;
      } else {
        n_u0 = a;
        n_n = t_len + p.len + extra;
        n_rec = t_rec;
        n_aux = t_aux;
        n_chunk = t_chunk;
        if constexpr (kBatch) {
          tail_issue(n_u0, n_n, t_ok != 0);
          stage = 4;
        } else {
          sort_nxt();
          fl |= fReady;
          stage = 0;
        }
      }
    } else if (st == 4 && !kLog) {  // (chunk epilogue) the tail bytes, then sort
      tail_finish();
      sort_nxt();
      fl |= fReady;
      stage = 0;
    } else if (st == 5) {  // (chunk epilogue, log records) the tail bytes, then sort
      tail_finish();
      sort_nxt();
      fl |= fReady;
      stage = 0;
    } else if (st == 4) {
      const uint64_t o = ((uint64_t)t_ohi << 32) | t_olo;
      n_u0 = base + o + 6;  // CRC input: type byte + payload
      uint32_t length = (hw1 >> 8) & 0xffffu;  // db/log_format.h:27-30
      if (kDiag && (p.wvar == 5 || p.wvar == 6)) {  // (timing ablation: no header loads)
        length = t_len;
        hw1 = (length << 8) | (1u << 24);  // a FULL record
      }
      const uint32_t ls = log_header_fits(o, p.buf_len)
                              ? log_status(o, length, MODE == kLogVerify ? hw1 >> 24 : 1u, p.buf_len)
                              : log_nohdr_status(o, p.buf_len);
      n_n = ls == NOVA_LOG_OK ? 1u + length : 0u;  // 0: not read, n_aux = status
      // kVarOutPos: results go to the record's position in p.perm's order
      // (dense per chunk); log_unperm_kernel moves them to the records
      n_rec = (VAR & kVarOutPos) ? t_chunk * C + my : t_rec;
      n_aux = ls == NOVA_LOG_OK ? (MODE == kLogWrite ? t_aux : hw0)
                                : ls;
      n_chunk = t_chunk;
      if constexpr (kBatch) {
        tail_issue(n_u0, n_n, t_ok != 0 && n_n != 0);
        stage = 5;
      } else {
        sort_nxt();
        fl |= fReady;
        stage = 0;
      }
    }
  };
  auto start_refill = [&](uint32_t chunk) {  // stage 1 of chunk (or none)
    t_chunk = chunk;
    if (chunk == kNone) {
      n_chunk = kNone;
      fl |= fReady;
      stage = 0;
    } else {
      pipe(1);
    }
  };

  // ---- rounds (load side; group-uniform / wave-uniform state) ---------------------
  uint64_t g_u0 = 0, g_u1 = 0, g_lp = 0, g_end = 0, g_rec = 0;
  uint32_t g_ninit = 0, g_st = 0, g_slot = 0;
  bool g_valid = false, r_clast = false;
  uint32_t r_idx = R, r_step = 0, r_S = 0, r_sk = 0, r_fast = 0;
  constexpr uint64_t kLine = 16 * G;  // one swath of a lane group
  uint64_t g_le = 0;                  // the group's region end on the line grid
  uint32_t g_w0 = 0, g_hs = 0, g_hs2 = 0;  // first region swath of this lane; head steps
  bool g_l3 = false, g_nz = false, g_hneed = false;
  // Take the next non-empty round (switching chunks as needed).  Returns with
  // r_S == 0 if the switch must wait for nxt (stall) or the work is done.
  auto next_round = [&]() {
    r_S = 0;
    g_valid = false;
    for (;;) {
      if (r_idx == R) {  // chunk exhausted: switch to nxt, start loading the one after
        if (!(fl & fReady)) return;  // stall: nxt still in the pipeline
        if constexpr (kBatch) c_tr = n_tr;
        c_u0 = n_u0;
        c_n = n_n;
        c_rec = n_rec;
        c_aux = n_aux;
        c_ok = n_ok;
        c_S = n_S;
        c_exact = n_exact;
        c_chunk = n_chunk;
        fl &= ~fReady;
        r_idx = 0;
        if (c_chunk == kNone) {
          fl |= fDone;
          return;
        }
        fl |= fRefill;
      }
      const uint32_t slot = r_idx * kGroups + (uint32_t)grp;
      g_slot = slot;
      r_idx++;
      const bool ok = __shfl(c_ok, (int)slot) != 0;
      const uint32_t a_lo = __shfl((uint32_t)c_u0, (int)slot);
      const uint32_t a_hi = __shfl((uint32_t)(c_u0 >> 32), (int)slot);
      const uint32_t n = __shfl(c_n, (int)slot);
      const uint32_t rec = __shfl(c_rec, (int)slot);
      const uint32_t aux = __shfl(c_aux, (int)slot);
      const uint64_t a = ((uint64_t)a_hi << 32) | a_lo;
      g_valid = ok;
      g_u0 = a;
      g_u1 = a + n;
      g_rec = rec;
      // ~init goes into the data's first 4 bytes; a block shorter than 4 bytes
      // gets it at the end instead (finish_block)
      g_ninit = (raw || n < 4) ? 0u : ~((kLog || MODE == kTrailer || MODE == kVerify) ? 0u : aux);
      g_st = aux;
      g_end = g_u1 & ~15ull;
      // steps on the group's 16G-byte line grid: lines from the one holding
      // the first byte to the one holding byte E-1 (load_step, kLines)
      g_le = (g_end + (kLine - 1)) & ~(kLine - 1);
      // the round runs the wave's largest line count m, in steps of 4 swaths:
      // r_S = ceil(m / 4) steps, the first of which skips its 4 r_S - m leading
      // swaths (no lane of the wave holds a region piece there)
      uint64_t NL = (g_le - (a & ~(kLine - 1))) / kLine;
      if (NL == 0) NL = 1;
      const uint32_t nl = NL > 0xfffffff0ull ? 0xfffffff0u : (uint32_t)NL;
      uint32_t m = ok ? nl : 0u;
      // the shortest non-empty region: its first line is the latest one, so
      // from step r_fast on every lane's four pieces are region pieces
      uint32_t mn = (ok && n > 0) ? nl : 0xffffffffu;
      if (c_exact) {
        // an exactly sorted chunk (largest first, invalid slots last): the
        // round's first slot holds its longest block (m is then exact, as it
        // must be), its last slot a lower bound of the shortest (a smaller mn
        // only takes fewer fast steps)
        const int s0 = __builtin_amdgcn_readfirstlane((int)(slot - (uint32_t)grp));
        m = (uint32_t)__builtin_amdgcn_readlane((int)c_S, s0);
        mn = (uint32_t)__builtin_amdgcn_readlane((int)c_S, s0 + (int)kGroups - 1);  // 0: an invalid slot
      } else {
        m = wave_max(m);
        mn = wave_min(mn);
      }
      r_S = (uint32_t)__builtin_amdgcn_readfirstlane((int)((m + 3) >> 2));  // wave-uniform: scalar control flow
      r_sk = (uint32_t)__builtin_amdgcn_readfirstlane((int)(4 * r_S - m));
      {
        // a lane's first region swath is at most line 4 r_S - nl + 1 of the
        // round (lanes whose piece of the first line lies before u0 & ~15)
        const uint32_t mnl = (uint32_t)__builtin_amdgcn_readfirstlane((int)mn);
        const uint32_t gmax = mnl == 0xffffffffu ? 0u : (mnl >= 4 * r_S ? 1u : 4 * r_S - mnl + 1);
        r_fast = (gmax + 3) >> 2;
      }
      if (r_S != 0) break;  // an empty round (past the batch's end): next one
    }
    // the chunk's last round: no rounds left, or only empty ones (invalid
    // slots are the chunk's last: positions past the batch, sorted last)
    r_clast = r_idx == R ||
              __builtin_amdgcn_readlane((int)c_ok, (int)__builtin_amdgcn_readfirstlane(r_idx * kGroups)) == 0;
    g_lp = g_le - (uint64_t)r_S * kStep;
    r_step = 0;
    // Per-lane 32-bit thresholds for the round's steps (issue/fold run no 64-bit
    // compares): lane q's piece of swath w (w = 4 * step + k) is at
    // g_lp + 16q + 16G*w; it is a region piece iff w >= g_w0 (at or after the
    // line holding A0 = u0 & ~15) and, for the last swath, below E.  The
    // head steps hold the bytes [u0, u0+4) that need masking / ~init.
    {
      const int64_t a0d = (int64_t)((g_u0 & ~15ull) - g_lp) - 16 * q;
      g_w0 = a0d <= 0 ? 0u : (uint32_t)((uint64_t)(a0d + (int64_t)kLine - 1) / kLine);
      g_l3 = g_lp + 16 * q + kLine * (4ull * r_S - 1) < g_end;
      const uint64_t u0rel = g_u0 - g_lp;
      g_hs = (uint32_t)(u0rel / kStep);
      g_hs2 = (uint32_t)((u0rel + 3) / kStep);
      g_nz = g_valid && g_u1 > g_u0;
      g_hneed = g_nz && ((g_u0 & 15) != 0 || g_ninit != 0);
    }
  };

  // Values loaded in one take and used only later are consumed at fixed points
  // (an empty asm reading them): the compiler then resolves their loads with
  // exact counts instead of waiting for all loads where its paths merge.
  auto take = [&](bool first) {
    // fl and stage are wave-uniform; saying so keeps the control flow below
    // scalar (the compiler's divergence analysis could not prove it)
    fl = (uint32_t)__builtin_amdgcn_readfirstlane((int)fl);
    stage = (uint32_t)__builtin_amdgcn_readfirstlane((int)stage);
    if (kBatch && (fl & fChunkEnd)) {
      // The chunk whose last step the previous take issued, for its epilogue
      // (which runs when that step folds, after this take): copied before a
      // switch can replace "c", and after the previous chunk's epilogue ran.
      fl &= ~fChunkEnd;
      e_u0 = c_u0;
      e_n = c_n;
      e_rec = c_rec;
      e_aux = c_aux;
      e_ok = c_ok;
      e_tr = c_tr;
    }
    if (first) {
      asm volatile("" ::"v"(req), "v"(t_olo), "v"(t_ohi), "v"(t_len), "v"(t_aux));
      if constexpr (kBatch && kLog)  // stage 4's tail loads, for stage 5
        asm volatile("" ::"v"(t_tl.x), "v"(t_tl.y), "v"(t_tl.z), "v"(t_tl.w));
      if (stage == 3) pipe(3);
      else if (kBatch && kLog && stage == 5) pipe(5);
      if ((fl & fRefill) && stage == 0 && !(fl & fReady)) {
        fl &= ~fRefill;
        uint32_t nc = kNone;
        if (!(fl & fDry)) {
          const uint64_t c = collect();
          if (c == kNoChunk) fl |= fDry;
          else {
            nc = (uint32_t)c;
            fl |= fClaim;
          }
        }
        start_refill(nc);
      }
    } else {
      asm volatile("" ::"v"(t_rec));
      if constexpr (kLog)
        asm volatile("" ::"v"(hw0), "v"(hw1));
      if constexpr (kBatch && !kLog) {  // stage 3's tail loads, for stage 4
        asm volatile("" ::"v"(t_tl.x), "v"(t_tl.y), "v"(t_tl.z), "v"(t_tl.w));
        if constexpr (kTail2) asm volatile("" ::"v"(t_t2));
      }
      if (stage == 2) pipe(2);
      else if (stage == 4) pipe(4);
      if (fl & fClaim) {
        claim(victim);
        fl &= ~fClaim;
      }
    }
    if ((fl & fRoundDone) && !(fl & fDone)) {
      next_round();
      if (r_S != 0) fl &= ~fRoundDone;  // else: stalled (retry next take) or done
    }
  };

  auto issue = [&](FlatSet& X) -> bool {
    fl = (uint32_t)__builtin_amdgcn_readfirstlane((int)fl);  // (wave-uniform: a scalar loop exit)
    r_step = (uint32_t)__builtin_amdgcn_readfirstlane((int)r_step);
    r_S = (uint32_t)__builtin_amdgcn_readfirstlane((int)r_S);
    r_fast = (uint32_t)__builtin_amdgcn_readfirstlane((int)r_fast);  // (a divergent branch
    // between the two load forms made the compiler drain every load: vmcnt(0))
    const bool live = !(fl & fDone);
    const bool run = r_S != 0;             // a round is active (else: stalled, empty step)
    const bool v = g_valid && run;
    const bool last = run && r_step + 1 == r_S;  // wave-uniform
    {
      const bool vz = g_nz && run;
      const uint32_t w = 4 * r_step;
      const uint64_t pa = g_lp + 16 * q;
      // The addresses are chosen in a wave-uniform branch and the four loads
      // issued after it: loads inside the branch made the compiler drain
      // every load (vmcnt(0)) where its register reuse met the other path.
      uint64_t a0, a1, a2, a3;
      if (run && !last && r_step >= r_fast) {
        // all four pieces of every lane are region pieces (or its group has
        // no data: the zero block, 1 KiB) -- one select
        const uint64_t b = vz ? pa : zl;
        a0 = b;
        a1 = b + 16 * G;
        a2 = b + 32 * G;
        a3 = b + 48 * G;
      } else {
        a0 = (vz && w >= g_w0) ? pa : zl;
        a1 = (vz && w + 1 >= g_w0) ? pa + 16 * G : zl;
        a2 = (vz && w + 2 >= g_w0) ? pa + 32 * G : zl;
        a3 = (vz && w + 3 >= g_w0 && (!last || g_l3)) ? pa + 48 * G : zl;
      }
      X.d0 = gload16<VAR>(a0);
      X.d1 = gload16<VAR>(a1);
      X.d2 = gload16<VAR>(a2);
      X.d3 = gload16<VAR>(a3);
      const bool vl = v && last;
      if constexpr (kBatch) {
        // (the chunk epilogue loaded the tail lines with the descriptors)
      } else if constexpr ((VAR & kVarNoTail) != 0) {  // timing ablation (diagnostics)
        X.t = make_uint4(0, 0, 0, 0);
        if constexpr (kTail2) X.t2 = make_uint4(0, 0, 0, 0);
      } else if constexpr (kTail2) {
        // tail lines: default (cached) policy -- on every step but a block's
        // last they all read the zero line, an L1 hit instead of an L2 request
        // (read-verify +0.4 points, log write +0.4; the trailer writer, which
        // stores into that line, -3: it keeps nt loads; profiles/r02_ab_tail_cached.log)
        const uint64_t ta = vl ? g_end : zl;  // holds the stored CRC's first byte
        X.t = gload16<VAR | kVarCached>(ta);
        X.t2 = gload16<VAR | kVarCached>((vl && g_u1 + 4 > g_end + 16) ? g_end + 16 : ta);
      } else {
        uint64_t ta = (vl && vz && (g_u1 & 15)) ? g_end : zl;
        if constexpr (MODE == kTrailer) {
          // whole-piece trailer stores: the 64-B piece(s) holding the trailer
          // [u1, u1+5) are 16-B lines s0 + 16k, k < 4 (8 when the trailer crosses
          // a piece); lane q < np loads line q instead of the tail line, which
          // is line (E - s0) / 16 -- fold shuffles it to the group
          const uint64_t s0 = g_u1 & ~63ull;
          const uint32_t np = ((g_u1 + 4) & ~63ull) != s0 ? 8u : 4u;
          const bool w = vl && sect && g_st != 0 && (uint32_t)q < np;
          if (w) ta = s0 + 16 * q;
          X.wsec = w;
        }
        if constexpr (MODE == kLogWrite) {
          // whole-piece CRC-field stores: lanes q < 4 load the 64-B piece holding
          // the header's CRC field [u0-6, u0-2); lanes 4.. load the tail line,
          // which fold shuffles to the group (G >= 8)
          const bool w = vl && vz && sect && g_st != 0 && (uint32_t)q < 4;
          if (w) ta = ((g_u0 - 6) & ~63ull) + 16 * q;
          X.wsec = w;
        }
        constexpr int kTailVar = (MODE == kTrailer || MODE == kStore) ? VAR : (VAR | kVarCached);
        X.t = gload16<kTailVar>(ta);  // (policy: see the verify branch above)
      }
      X.head = vz && g_hneed && (r_step == g_hs || r_step == g_hs2);
      X.l3 = g_l3;  // (fold runs after the next round may have started)
    }
    X.pa = g_lp;
    X.u0 = g_u0;
    X.u1 = g_u1;
    if constexpr (!kBatch) {
      X.rec = g_rec;
      X.st = g_st;
    } else {
      X.slot = g_slot;
      X.cend = last && r_clast;
    }
    // An invalid group's step (or a stalled one) reads zeros; with no init
    // xor-ed in it leaves the group's zero registers zero for its next block.
    X.ninit = v ? g_ninit : 0u;
    X.valid = v;
    X.last = last;
    // wave-uniform; 4 (never a round's skip: r_sk <= 3) marks an empty step,
    // which fold skips (kVarFoldEmpty: folds its zeros, the round-4 form)
    X.skip = !run ? ((VAR & kVarFoldEmpty) ? 0u : 4u) : (r_step == 0 ? r_sk : 0u);
    if (run) {
      g_lp += kStep;
      if (++r_step == r_S) fl |= kBatch && r_clast ? (fRoundDone | fChunkEnd) : fRoundDone;
    }
    return live;
  };

  // Lane l finishes sorted slot l of the chunk whose last round just folded
  // (its descriptors are in the e bank).  Stores go out after the next step's
  // loads were issued (fold runs after issue).
  auto chunk_epilogue = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kDiag && p.wvar == 3) return;  // timing ablation: no per-block epilogue, no result (WRONG)
    typedef __attribute__((address_space(1))) uint8_t gu8;
    typedef __attribute__((address_space(1))) uint32_t gu32;
    const bool ok = e_ok != 0;
    const bool wr = ok && (!kDiag || p.wvar < 2 || p.wvar >= 4);
    const uint64_t u1 = e_u0 + e_n;
    const uint32_t nb = (uint32_t)(u1 & 15u);
    uint32_t R = shift_nb<kMainBytes>(lds, kByteTab, lapply(lds + kMainBytes, vbuf[lane]), nb) ^ e_tr;
    if (e_n < 4 && !raw) {  // the data ran from a zero register: add M_n(~init)
      uint32_t l = ~(any_init ? e_aux : 0u);
      for (uint32_t i = 0; i < 3; i++) {
        const uint32_t r = (l >> 8) ^ lds_u32(lds, kByteTab + (l & 255u) * 4u);
        l = i < e_n ? r : l;
      }
      R ^= l;
    }
    uint32_t crc = raw ? R : ~R;
    bool bad = false;
    if constexpr (MODE == kLogWrite) {
      const bool status_only = e_n == 0;  // a record not read: e_aux holds its status
      const uint32_t m = mask_crc(crc);  // db/log_writer.cc:113
      if constexpr ((VAR & kVarOutPos) != 0) {
        if (wr) {
          *(gu32*)(p.out + e_rec) = m;
          *(gu8*)(p.ok_out + e_rec) = (uint8_t)(status_only ? e_aux : (uint32_t)NOVA_LOG_OK);
        }
      } else if (wr && !status_only) {
        store_u32_unaligned((uint8_t*)(e_u0 - 6), m);
      }
    } else if constexpr (MODE == kLogVerify) {
      const uint32_t st = e_n == 0 ? e_aux : (unmask_crc(e_aux) == crc ? 1u : 0u);  // db/log_reader.cc:254-256
      if (wr) *(gu8*)(p.ok_out + e_rec) = (uint8_t)st;
      bad = wr && (st == NOVA_LOG_CHECKSUM_MISMATCH || st == NOVA_LOG_BAD_LENGTH);
    } else if constexpr (MODE == kVerify) {
      const uint32_t st = unmask_crc(e_aux) == crc ? 1u : 0u;  // table/table.cc:435-437
      if (wr) *(gu8*)(p.ok_out + e_rec) = (uint8_t)st;
      bad = wr && !st;
    } else {
      if (p.flags & NOVA_CRC32C_APPEND_TYPE) crc = ~byte_step(~crc, (p.flags >> 8) & 0xffu);
      if constexpr (MODE == kTrailer) {
        if (wr)
          store_trailer((uint8_t*)u1, (p.flags >> 8) & 0xffu, mask_crc(crc),
                        (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
      } else {
        if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
        if (wr) *(gu32*)(p.out + e_rec) = crc;
      }
    }
    if constexpr (MODE == kVerify || MODE == kLogVerify) {
      const uint64_t b = __builtin_amdgcn_ballot_w64(bad);  // one atomic per chunk
      // (the timing ablations that compute WRONG CRCs count nothing: every
      // chunk's atomic on one word would time the counter, not the kernel)
      const bool wrong = kDiag && p.wvar >= 4 && p.wvar != 7;
      if (b && lane == 0 && p.n_bad && !wrong) atomicAdd(p.n_bad, (uint32_t)__builtin_popcountll(b));
    }
  };

  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  bool wb_on = false, wb_sec = false;
  uint64_t wb_a = 0;
  uint32_t wb_v = 0;
  uint4 wb_w = make_uint4(0, 0, 0, 0);  // trailer writer: the patched sector piece
  uint32_t wb_pos = 0, wb_st = 0;       // kVarOutPos log write: position, status
  auto fold = [&](FlatSet& Y) {
    uint4 d0 = Y.d0, d1 = Y.d1, d2 = Y.d2, d3 = Y.d3;
    // (diagnostics timing ablation, wvar 8: no head masking -- WRONG CRCs)
    if (!(kDiag && p.wvar == 8) && __builtin_amdgcn_ballot_w64(Y.head)) {  // wave-uniform: some group's head step
      // h = u0 - (lane's piece of swath 0 of the step); pieces wholly before u0
      // came from the zero line, so only [u0, u0+4) and the bytes before u0 in
      // u0's piece need work.  Non-head groups keep their data (h <= -16).
      const int32_t h = Y.head ? (int32_t)(Y.u0 - Y.pa) - 16 * q : -64;
      if constexpr (any_init) {  // per-block init values: byte-exact head_piece
        d0 = head_piece(d0, h, Y.ninit);
        d1 = head_piece(d1, h - 16 * G, Y.ninit);
        d2 = head_piece(d2, h - 32 * G, Y.ninit);
        d3 = head_piece(d3, h - 48 * G, Y.ninit);
      } else {  // ~init is ~0 (Value) or 0 (RAW, n < 4): ((d ^ LM[lo4]) & ~LM[lo])
        // At most one of the lane's four pieces (16G bytes apart) holds a byte
        // of [u0, u0+4): swath kk with -4 < h - 16G kk < 16.  Its pieces before
        // u0's came from the zero line, so only that piece is masked -- two
        // 16-B mask reads per lane instead of eight.
        const int32_t hh = h + 3;
        const int32_t kk = hh < 0 ? 4 : (hh >> (4 + __builtin_ctz(G)));  // hh / 16G
        const int32_t hk0 = h - 16 * G * kk;
        const int32_t hk = (kk < 4 && hk0 < 16) ? hk0 : -4;  // -4: masks of nothing
        const int32_t i4 = Y.ninit ? 4 : 0;
        const uint4 B = lds_u128(kLM + 16u * (uint32_t)clamp16(hk));
        const uint4 I = lds_u128(kLM + 16u * (uint32_t)clamp16(hk + i4));
        // word by word, in registers (a select of whole uint4 values went
        // through a private-memory array: 2.4x slower launches)
        const bool s0 = kk == 0, s1 = kk == 1, s2 = kk == 2, s3 = kk == 3;
        auto word = [&](uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t b, uint32_t i) {
          const uint32_t x = s0 ? a0 : (s1 ? a1 : (s2 ? a2 : a3));
          const uint32_t y = (x ^ i) & ~b;
          a0 = s0 ? y : a0;
          a1 = s1 ? y : a1;
          a2 = s2 ? y : a2;
          a3 = s3 ? y : a3;
        };
        word(d0.x, d1.x, d2.x, d3.x, B.x, I.x);
        word(d0.y, d1.y, d2.y, d3.y, B.y, I.y);
        word(d0.z, d1.z, d2.z, d3.z, B.z, I.z);
        word(d0.w, d1.w, d2.w, d3.w, B.w, I.w);
      }
    }
    // A round's first step skips the leading swaths in which no lane of the
    // wave holds a region piece (they read the zero line into zero registers),
    // so a round costs its longest block's lines, not whole 4-swath steps.
    const uint32_t sk = (uint32_t)__builtin_amdgcn_readfirstlane((int)Y.skip);
    if (sk >= 4) {
      // an empty step (the load side waited for the next chunk's descriptors):
      // no region piece, nothing to fold -- give the SIMD's issue slots to the
      // other waves instead of folding zeros (64 table lookups per lane)
      __builtin_amdgcn_s_sleep(1);
      return;
    }
    if (Y.last) {  // wave-uniform: the region's last line may end past E
      if (sk < 1) swath4<VAR>(lds, c0, c1, c2, c3, d0, lo0, lo1, lo2, lo3);
      if (sk < 2) swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
      if (sk < 3) swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
      const uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = c3;
      swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
      if (!Y.l3) {  // piece at or after E: not in the region
        c0 = k0;
        c1 = k1;
        c2 = k2;
        c3 = k3;
      }
    } else if (sk != 0) {
      if (sk < 2) swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
      if (sk < 3) swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
      swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
    } else if constexpr ((VAR & kVarNarrow) != 0) {
      fold4<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
    } else {
      fold4w<VAR>(lds, c0, c1, c2, c3, d0, d1, d2, d3, lo0, lo1, lo2, lo3);
    }
    // the tail line(s) are used only on a block's last step: consume anyway, so
    // the compiler resolves their loads here with an exact count
    if constexpr (!kBatch) {
      asm volatile("" ::"v"(Y.t.x), "v"(Y.t.y), "v"(Y.t.z), "v"(Y.t.w));
      if constexpr (kTail2) asm volatile("" ::"v"(Y.t2.x), "v"(Y.t2.y), "v"(Y.t2.z), "v"(Y.t2.w));
    }
    if (Y.last) {  // wave-uniform: every group ends its block on this step
      // On the line grid lane q's pieces sit at position (q - e) mod G of the
      // 16G-byte swaths that end at E (e = (E mod 16G) / 16); group_fold wants
      // position p in lane p, which reads lane (p + e) mod G.
      const uint32_t e = (uint32_t)(Y.u1 >> 4) & (uint32_t)(G - 1);
      const int src = (grp * G) + (int)(((uint32_t)q + e) & (uint32_t)(G - 1));
      uint32_t v;
      if (kDiag && p.wvar == 9) {  // (timing ablation: no group fold -- WRONG CRCs)
        v = c0 ^ c1 ^ c2 ^ c3;
      } else {
        c0 = __shfl(c0, src);
        c1 = __shfl(c1, src);
        c2 = __shfl(c2, src);
        c3 = __shfl(c3, src);
        v = group_fold<G>(lds, c0, c1, c2, c3, q);
      }
      c0 = c1 = c2 = c3 = 0;
      if constexpr (kBatch) {
        if (q == 0 && Y.valid) vbuf[Y.slot] = v;
        if (Y.cend) chunk_epilogue();  // wave-uniform
        return;
      }
      bool elig = false;
      uint4 piece = Y.t;
      if constexpr (MODE == kLogWrite) {
        elig = sect && Y.valid && Y.st != 0 && Y.u1 != Y.u0;  // (status-only records: Y.st = status)
        const int src = elig ? grp * G + 4 : lane;
        Y.t.x = __shfl(piece.x, src);
        Y.t.y = __shfl(piece.y, src);
        Y.t.z = __shfl(piece.z, src);
        Y.t.w = __shfl(piece.w, src);
      }
      if constexpr (MODE == kTrailer) {
        // whole-piece form (group-uniform eligibility): the tail line is the
        // group's window line (E - s0) / 16; every lane takes it from there
        elig = sect && Y.valid && Y.st != 0;
        const uint32_t k = (uint32_t)((Y.u1 >> 4) & 3u);  // (E - s0) / 16
        const int src = elig ? grp * G + (int)k : lane;
        Y.t.x = __shfl(piece.x, src);
        Y.t.y = __shfl(piece.y, src);
        Y.t.z = __shfl(piece.z, src);
        Y.t.w = __shfl(piece.w, src);
      }
      if (kDiag && p.wvar == 3) {  // timing ablation: no per-block epilogue, no result (WRONG)
        wb_a = 0;
        wb_v = v;
      } else {
        finish_block<MODE>(lds, kByteTab, p, raw, v, Y, wb_a, wb_v);
      }
      wb_on = q == 0 && Y.valid;  // written after the next step's loads are issued
      if constexpr ((VAR & kVarOutPos) != 0 && MODE == kLogWrite) {
        wb_pos = (uint32_t)Y.rec;
        wb_st = Y.u1 == Y.u0 ? Y.st : (uint32_t)NOVA_LOG_OK;  // (status-only records: Y.st = status)
      }
      if constexpr (MODE == kTrailer) {
        // lanes holding a sector piece store it patched with the trailer;
        // lane 0's byte stores are not used
        wb_sec = elig;
        if (elig) {
          wb_on = Y.wsec;
          const bool quirk = (p.flags & NOVA_TRAILER_TB_QUIRK) != 0;
          const uint32_t m = quirk ? ((wb_v & 0x00ffffffu) | ((uint32_t)'!' << 24)) : wb_v;
          const uint64_t tv = (uint64_t)((p.flags >> 8) & 0xffu) | ((uint64_t)m << 8);
          wb_a = (Y.u1 & ~63ull) + 16u * (uint32_t)q;
          wb_w = patch_trailer(piece, wb_a, Y.u1, tv);
        }
      }
      if constexpr (MODE == kLogWrite) {
        wb_sec = elig;
        if (elig) {
          wb_on = Y.wsec;
          wb_a = ((Y.u0 - 6) & ~63ull) + 16u * (uint32_t)q;
          wb_w = patch_trailer<4>(piece, wb_a, Y.u0 - 6, wb_v);
        }
      }
    }
  };
  auto writeback = [&]() {
    if (wb_on) {
      if constexpr ((VAR & kVarOutPos) != 0 && MODE == kLogWrite) {
        // position-indexed: Mask(crc) and the record's status (log_unperm_kernel
        // writes the CRC field of the records whose status is OK)
        typedef __attribute__((address_space(1))) uint32_t gu32;
        typedef __attribute__((address_space(1))) uint8_t gu8;
        if (!kDiag || p.wvar < 2 || p.wvar >= 4) {
          *(gu32*)(p.out + wb_pos) = wb_v;
          *(gu8*)(p.ok_out + wb_pos) = (uint8_t)wb_st;
        }
        wb_on = false;
        return;
      }
      if ((MODE == kTrailer || MODE == kLogWrite) && wb_sec) {
        u32x4 w;
        w.x = wb_w.x;
        w.y = wb_w.y;
        w.z = wb_w.z;
        w.w = wb_w.w;
        if (kDiag && p.wvar == 1)
          __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)wb_a);
        else if (!kDiag || p.wvar != 2)
          *(__attribute__((address_space(1))) u32x4*)wb_a = w;
      } else {
        if (!kDiag || p.wvar < 2 || p.wvar >= 4) write_result<MODE>(p, wb_a, wb_v);
      }
      wb_on = false;
    }
  };

  // ---- prologue: the first chunk is implicit, the second is claimed; both are
  // loaded synchronously (stages back to back) ----------------------------------
  {
    uint64_t k0 = (uint64_t)wave * nwg + xslot(blockIdx.x);
    if (k0 >= p.n_chunks) {
      claim(victim);
      k0 = collect();
    }
    if (k0 == kNoChunk) fl |= fDry;
    start_refill(k0 == kNoChunk ? kNone : (uint32_t)k0);
    while (stage != 0) pipe(stage);
    next_round();  // switches to k0 and takes its first round
    uint64_t k1 = kNoChunk;
    if (!(fl & fDry)) {
      claim(victim);
      k1 = collect();
      if (k1 == kNoChunk) fl |= fDry;
      else fl |= fClaim;
    }
    start_refill(k1 == kNoChunk ? kNone : (uint32_t)k1);
    while (stage != 0) pipe(stage);
    fl &= ~fRefill;
    if (r_S == 0 && !(fl & fDone)) fl |= fRoundDone;  // k0 empty: next take moves on
  }
  FlatSet A, B;
  A.d0 = A.d1 = A.d2 = A.d3 = A.t = A.t2 = make_uint4(0, 0, 0, 0);
  A.pa = A.u0 = A.u1 = A.rec = 0;
  A.ninit = A.st = 0;
  A.valid = A.last = A.head = A.l3 = A.wsec = A.cend = false;
  A.slot = 0;
  for (;;) {
    take(true);
    issue(B);
    writeback();
    fold(A);
    take(false);
    const bool a_live = issue(A);
    writeback();
    fold(B);
    if (!a_live) break;
  }
  writeback();
  __builtin_amdgcn_s_waitcnt(0);  // the last claim has returned (see the flat kernel)
  sched_release(p.sched);
}


// ---- crc32c_burst_kernel<G, MODE>: one SSTable per call (latency path) -------
// NovaLSM checksums one SSTable (~4K blocks of ~4 KiB) per call and waits for
// it.  The throughput kernels keep ONE step of loads in
// flight per wave, so a small batch pays a full HBM round trip per step.
// Here a lane group takes one block and issues ALL of its loads at once:
//   * the block's region [E - K*S, E) (E = u1 & ~15, S = 16G) is K swaths;
//     lane q holds the 16-B piece q of every swath, so its four registers are
//     word streams with an S-byte stride (c = w ^ M_S(c)); pieces before the
//     block read the zero line (leading zeros leave a zero register alone), the
//     piece(s) holding [u0, u0+4) take ~init.  The wave's groups run the
//     wave's largest K, each group's region end-aligned (shorter blocks start
//     on zero pieces);
//   * up to kK swaths per pass are loaded together; a longer block loads its
//     next pass before folding the current one;
//   * the stream words fold in-lane (M4, M8) and across the group, then the
//     0..15 tail bytes [E, u1) and the mode's epilogue run as in the rounds
//     kernel (finish_block);
//   * the first block's descriptor and data loads are issued before the LDS
//     tables are filled, and the fill is LDS-DMA (global_load_lds_dwordx4: no
//     VGPRs, the whole image in flight at once), so the three round trips
//     (descriptors, data, tables) overlap instead of adding up.
// Two table sets:
//   G = 64 (one block per wave): the M_1024 operator NOT bank-replicated plus
//     8 tree levels and the byte table, 37 KiB -- for a few blocks per call,
//     where the fill and the dependency chain are the cost;
//   G = 16 (four blocks per wave): the rounds kernel's bank-replicated M_256
//     image (128 KiB) + 6 tree levels + byte table -- conflict-free lookups for
//     thousands of blocks, where LDS lookups are the cost (random 8-bit
//     indices into one 1 KiB table collide ~4-way per wave-instruction).
// V: the table set.  64: one wave per block, compact M_1024; 65: the same with
// the M_1024 operator 16-way bank-replicated (64 KiB; lane l reads replica
// l & 15); 16: four blocks per wave on the replicated M_256 image.
template <int V>
struct BurstCfg;
template <>
struct BurstCfg<64> {
  static constexpr int kG = 64;
  static constexpr int kWaves = 16;                           // launch bound
  static constexpr int kDefWaves = 8;                         // per workgroup by default
  static constexpr int kK = 8;                                // swaths per pass
  static constexpr uint32_t kTree = 4096;                     // after the M_1024 op
  static constexpr int kLevels = 8;                           // M4 .. M512
};
// The diagnostics build's table sets (measured slower).
template <>
struct BurstCfg<65> {
  static constexpr int kG = 64;
  static constexpr int kWaves = 16;
  static constexpr int kDefWaves = 16;
  static constexpr int kK = 8;
  static constexpr uint32_t kTree = 65536;                    // after the replicated M_1024 op
  static constexpr int kLevels = 8;
};
template <>
struct BurstCfg<16> {
  static constexpr int kG = 16;
  static constexpr int kWaves = 16;
  static constexpr int kDefWaves = 16;
  static constexpr int kK = 16;
  static constexpr uint32_t kTree = kMainBytes;               // after the replicated image
  static constexpr int kLevels = 6;                           // M4 .. M128
};
template <int V>
constexpr uint32_t burst_byte_tab() { return BurstCfg<V>::kTree + BurstCfg<V>::kLevels * kTreeBytes; }
template <int V>
constexpr uint32_t burst_lds() { return burst_byte_tab<V>() + 1024; }
constexpr uint64_t kBurstSw = 1024;  // G = 64 swath (the M_1024 operator)

// LDS-DMA copy of `bytes` (a multiple of 1 KiB) from `src` to LDS byte `dst`:
// each wave-instruction moves 1 KiB (lane l: 16 B at +16 l).  Not waited for.
__device__ __forceinline__ void glds_copy(uint32_t dst, const void* src, uint32_t bytes) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = blockDim.x >> 6, wave = threadIdx.x >> 6;
  for (uint32_t c = wave; c < bytes / 1024; c += nw)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)((const uint8_t*)src + 1024u * c + 16u * lane),
        (__attribute__((address_space(3))) void*)(uintptr_t)(dst + 1024u * c), 16, 0, 0);
}

// The 16-way replicated M_1024 operator: table k, entry idx, replica c at LDS
// byte k*16384 + idx*64 + c*4 (c4 = 4c).
[[maybe_unused]] __device__ __forceinline__ uint32_t rapply(uint32_t c4, uint32_t x) {
  const uint32_t a0 = ((x & 255u) << 6) | c4;
  const uint32_t a1 = (((x >> 8) & 255u) << 6) | c4 | 16384u;
  const uint32_t a2 = (((x >> 16) & 255u) << 6) | c4 | 32768u;
  const uint32_t a3 = ((x >> 24) << 6) | c4 | 49152u;
  return xor3(lds_u32(nullptr, a0), lds_u32(nullptr, a1), lds_u32(nullptr, a2)) ^ lds_u32(nullptr, a3);
}

// Stream step of one swath piece for the group's four registers.
template <int V>
__device__ __forceinline__ void burst_step(const uint8_t* lds, uint32_t& c0, uint32_t& c1,
                                           uint32_t& c2, uint32_t& c3, const uint4& w,
                                           uint32_t lo0, uint32_t lo1, uint32_t lo2, uint32_t lo3) {
  if constexpr (V == 64) {
    c0 = lapply(lds, c0) ^ w.x;
    c1 = lapply(lds, c1) ^ w.y;
    c2 = lapply(lds, c2) ^ w.z;
    c3 = lapply(lds, c3) ^ w.w;
  } else if constexpr (V == 65) {
    const uint32_t c4 = (threadIdx.x & 15u) << 2;
    c0 = rapply(c4, c0) ^ w.x;
    c1 = rapply(c4, c1) ^ w.y;
    c2 = rapply(c4, c2) ^ w.z;
    c3 = rapply(c4, c3) ^ w.w;
  } else {
    swath4<0>(lds, c0, c1, c2, c3, w, lo0, lo1, lo2, lo3);
  }
}

template <int V, int MODE, int VAR = 0>
__global__ void __launch_bounds__(BurstCfg<V>::kWaves * 64) crc32c_burst_kernel(CrcParams p) {
  using Cfg = BurstCfg<V>;
  constexpr int G = Cfg::kG;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr bool kTail2 = MODE == kVerify;  // the stored CRC follows the CRC input
  constexpr int kK = Cfg::kK;
  constexpr uint64_t kS = 16ull * G;
  constexpr uint32_t kGroups = 64 / G;
  const int lane = threadIdx.x & 63;
  const int q = lane & (G - 1);
  const int grp = lane / G;
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const uint8_t* tree = lds + Cfg::kTree;  // level l: M_{4 * 2^l}
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t extra = (MODE == kVerify) ? 1u : 0u;  // verify covers block + type byte
  const uint64_t zl = (uint64_t)p.zline;
  const uint64_t base = (uint64_t)p.base;
  const uint64_t n_all = p.n_blocks;
  const uint64_t step_blocks = (uint64_t)gridDim.x * (blockDim.x >> 6) * kGroups;

  // per-group block state (the group's lanes hold identical values)
  uint64_t bw = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kGroups;
  FlatSet Y;
  uint64_t A0 = 0, first = 0, Kw = 0;
  bool valid = false;
  uint4 d[kK], e[kK];
  auto load_pass = [&](uint4 (&x)[kK], uint64_t k0) {
#pragma unroll
    for (int i = 0; i < kK; i++) {
      const uint64_t a = first + (k0 + i) * kS;
      x[i] = gload16((valid && k0 + i < Kw && a >= A0) ? a : zl);
    }
  };
  // descriptors of the wave's next blocks, tail lines and the first pass
  auto start_blocks = [&]() {
    const uint64_t b = bw + grp;
    valid = b < n_all;
    const uint64_t bb = valid ? b : n_all - 1;  // clamped: valid memory, result unused
    const uint64_t u0 = base + p.offsets[bb & p.omask] + bb * p.stride;
    const uint32_t n = p.lengths[bb & p.lmask] + p.len + extra;
    const uint32_t init = p.init[bb & p.imask];
    const uint64_t u1 = u0 + n;
    const uint64_t E = u1 & ~15ull;
    A0 = u0 & ~15ull;
    const uint64_t K = E > A0 ? (E - A0 + kS - 1) / kS : 0;
    uint64_t km = valid ? K : 0;  // the wave's largest block (groups end-aligned)
    if constexpr (G < 64) {  // per-block step counts fit 32 bits (a block is < 4 GiB)
      km = wave_max((uint32_t)km);
    }
    Kw = km;
    first = E - Kw * kS + 16ull * q;
    Y.u0 = u0;
    Y.u1 = u1;
    Y.rec = b;
    Y.ninit = (raw || n < 4) ? 0u : ~init;
    Y.st = init;
    Y.valid = valid;
    // tail line(s): [E, E+16) holds the tail bytes (verify: the start of the
    // stored CRC), [E+16, E+32) the rest of a stored CRC
    const bool need_t = valid && (kTail2 || (u1 & 15) != 0);
    Y.t = gload16(need_t ? E : zl);
    if constexpr (kTail2) Y.t2 = gload16(valid && u1 + 4 > E + 16 ? E + 16 : zl);
    if (Kw) load_pass(d, 0);
  };
  // kVarStamps (diagnostics): per-wave phase stamps (s_memrealtime, 100 MHz):
  // entry, descriptors used, tables + first data landed, first block folded,
  // first result written
  constexpr bool kStamps = (VAR & kVarStamps) != 0;
  uint64_t st[5] = {0, 0, 0, 0, 0};
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (kStamps && p.stamps) st[0] = __builtin_amdgcn_s_memrealtime();
  const bool live0 = bw < n_all;
  if (live0) start_blocks();
  if (kStamps && p.stamps) {
    asm volatile("" ::"v"((uint32_t)Kw));
    st[1] = __builtin_amdgcn_s_memrealtime();
  }
  // tables by LDS-DMA while the first block's loads are in flight
  glds_copy(0, p.tab_main, Cfg::kTree);
  glds_copy(Cfg::kTree, p.tab_tree, Cfg::kLevels * kTreeBytes);
  glds_copy(burst_byte_tab<V>(), p.tab_byte, 1024);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (kStamps && p.stamps) st[2] = __builtin_amdgcn_s_memrealtime();
  if (!live0) return;

  for (;;) {
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    auto fold_pass = [&](const uint4 (&x)[kK], uint64_t k0) {
#pragma unroll
      for (int i = 0; i < kK; i++) {
        if (k0 + i < Kw) {  // wave-uniform
          const uint64_t a = first + (k0 + i) * kS;
          const int32_t h = rel32(Y.u0, a, 32);
          const uint4 w = is_head(h) ? head_piece(x[i], h, Y.ninit) : x[i];
          burst_step<V>(lds, c0, c1, c2, c3, w, lo0, lo1, lo2, lo3);
        }
      }
    };
    for (uint64_t k0 = 0; k0 < Kw; k0 += 2 * kK) {
      if (k0 + kK < Kw) load_pass(e, k0 + kK);
      fold_pass(d, k0);
      if (k0 + kK < Kw) {
        if (k0 + 2 * kK < Kw) load_pass(d, k0 + 2 * kK);
        fold_pass(e, k0 + kK);
      }
    }
    // fold the group's stream words: in-lane M4/M8, then M16 .. across the group
    uint32_t v = lapply(tree + kTreeBytes, lapply(tree, c0) ^ c1) ^ (lapply(tree, c2) ^ c3);
    auto level = [&](int k, uint32_t o) {  // o: v of lane q ^ 2^k
      const bool right = (q >> k) & 1;
      v = lapply(tree + (2 + k) * kTreeBytes, right ? o : v) ^ (right ? v : o);
    };
    if constexpr (G > 1) level(0, lane_xor<1>(v));
    if constexpr (G > 2) level(1, lane_xor<2>(v));
    if constexpr (G > 4) level(2, lane_xor<4>(v));
    if constexpr (G > 8) level(3, lane_xor<8>(v));
    if constexpr (G > 16) level(4, lane_xor<16>(v));
    if constexpr (G > 32) level(5, lane_xor<32>(v));
    uint64_t wb_a = 0;
    uint32_t wb_v = 0;
    if (kStamps && p.stamps && !st[3]) {
      asm volatile("" ::"v"(v));
      st[3] = __builtin_amdgcn_s_memrealtime();
    }
    finish_block<MODE, Cfg::kTree>(lds, burst_byte_tab<V>(), p, raw, v, Y, wb_a, wb_v);
    if (q == 0 && Y.valid) write_result<MODE>(p, wb_a, wb_v);
    if (kStamps && p.stamps && !st[4]) {
      __builtin_amdgcn_s_waitcnt(0);
      st[4] = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) {
        for (int k = 0; k < 5; k++) p.stamps[8 * wid + k] = st[k];
        p.stamps[8 * wid + 5] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // XCC id
        p.stamps[8 * wid + 6] = Kw;
      }
    }
    bw += step_blocks;
    if (bw >= n_all) break;
    start_blocks();
  }
}


// ---- host: kernel attributes and launchers ------------------------------------
// Templates over the kernel variant VAR: each translation unit instantiates
// the variants it launches -- the product VAR 0 (and kVarInit), the
// diagnostics TU its ablations.

// Waves per workgroup.  The tables fill the CU's LDS, so a CU runs exactly one
// workgroup; fewer waves keep fewer HBM reads in flight per CU, which the
// streaming kernel prefers (tools/ceiling.py: 8 waves 2-3% faster than 16).
constexpr int kStreamWaves = 8;
constexpr int kUnitsWaves = 12;  // config 3 sweep: 12 > 16 > 8

template <int G, int MODE, int VAR = 0>
int set_lds_attr() {
  const int lds = (int)(kMainBytes + (2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16)) * kTreeBytes +
                        kWaves * kWaveScratch);
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_units_kernel<G, MODE, VAR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <int G, int VAR = 0>
int set_lds_attr_stream() {
  const int lds = (int)(kMainBytes + (2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16)) * kTreeBytes);
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_stream_kernel<G, VAR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

// Rounds (and flat) kernel LDS: tables + byte table; the rounds kernel adds
// the prefix masks and per-wave sort scratch (launch_rounds_v).
template <int G>
constexpr size_t flat_lds() {
  return kMainBytes + (2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16)) * kTreeBytes + 1024;
}
inline size_t flat_lds_g(int G) {
  switch (G) {
    case 1: return flat_lds<1>();
    case 2: return flat_lds<2>();
    case 4: return flat_lds<4>();
    case 8: return flat_lds<8>();
    default: return flat_lds<16>();
  }
}

template <int G, int MODE, int VAR = 0>
int set_lds_attr_rounds() {
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_rounds_kernel<G, MODE, VAR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax);
}

template <int MODE, int VAR = 0>
int set_lds_attrs_rounds() {
  int e = 0;
  if ((e = set_lds_attr_rounds<2, MODE, VAR>())) return e;
  if ((e = set_lds_attr_rounds<4, MODE, VAR>())) return e;
  if ((e = set_lds_attr_rounds<8, MODE, VAR>())) return e;
  return set_lds_attr_rounds<16, MODE, VAR>();
}

template <int V, int MODE, int VAR = 0>
int set_lds_attr_burst() {
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_burst_kernel<V, MODE, VAR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)burst_lds<V>());
}

template <int VAR = 0>
int set_lds_attrs_stream() {
  int e = 0;
  if ((e = set_lds_attr_stream<1, VAR>())) return e;
  if ((e = set_lds_attr_stream<2, VAR>())) return e;
  if ((e = set_lds_attr_stream<4, VAR>())) return e;
  if ((e = set_lds_attr_stream<8, VAR>())) return e;
  return set_lds_attr_stream<16, VAR>();
}

template <int MODE, int VAR = 0>
int set_lds_attrs_mode() {
  int e = 0;
  if ((e = set_lds_attr<1, MODE, VAR>())) return e;
  if ((e = set_lds_attr<2, MODE, VAR>())) return e;
  if ((e = set_lds_attr<4, MODE, VAR>())) return e;
  if ((e = set_lds_attr<8, MODE, VAR>())) return e;
  return set_lds_attr<16, MODE, VAR>();
}

// The first nwaves x wgs chunks (rounds) are implicit (one per wave): when
// they cover the batch, a claim or a steal can only come back empty, and each
// of the 8 probes is a serial device-scope atomic (~1.5 us) on the launch's
// tail.
inline uint32_t steal_limit(uint64_t work, uint64_t wgs, uint64_t nwaves) {
  const int sl = g_tune_static_pct.load();
  if (sl >= 0) return (uint32_t)sl;
  return work <= wgs * nwaves ? 0u : 8u;  // 8 probes = one victim per XCD
}

// ---- units kernel (segmented rounds; mostly >= 16 KiB blocks) ----------------
template <int MODE, int VAR>
int launch_units_g(int G, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const CrcParams& p) {
  switch (G) {
    case 1: hipLaunchKernelGGL((crc32c_units_kernel<1, MODE, VAR>), grid, block, lds, stream, p); break;
    case 2: hipLaunchKernelGGL((crc32c_units_kernel<2, MODE, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_units_kernel<4, MODE, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_units_kernel<8, MODE, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_units_kernel<16, MODE, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
}

template <int MODE, int VAR>
int launch_units_v(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
  p.tab_main = t->main[gindex(G)];
  p.tab_tree = t->tree;
  p.tab_ft = t->ft;
  p.tab_sh16 = t->sh16;
  p.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
  {
    const int ch = g_tune_chunk.load();
    p.chunk = (ch > 0 && ch <= 16) ? (uint32_t)ch : 8u;
  }
  p.n_chunks = (p.n_blocks + p.chunk - 1) / p.chunk;
  uint64_t nwaves = waves_per_wg(kUnitsWaves);
  if (nwaves > (uint64_t)kUnitsMaxWaves) nwaves = kUnitsMaxWaves;  // the kernel's launch bound
  uint64_t wgs = (p.n_chunks + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  if (wgs == 0) return 0;
  p.steal_limit = steal_limit(p.n_chunks, wgs, nwaves);
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const int levels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  const size_t lds = kMainBytes + levels * kTreeBytes + kWaves * kWaveScratch;
  return launch_units_g<MODE, VAR>(G, dim3(wgs), dim3(64 * nwaves), lds, stream, p);
}

// ---- stream kernel (aligned uniform batches) ------------------------------------
// Blocks per lane group per round: a wave-round of ~64 KiB measured best on
// MI355X at every block size tried (4 KiB: G=8 x 2 blocks, 76% of 8 TB/s vs
// 71% with 1; 16 KiB: G=16 x 1 block, 82%).
inline uint32_t stream_bpg(int G, uint32_t len) {
  const int tb = g_tune_bpg.load();
  if (tb > 0) return (uint32_t)tb;
  const uint64_t per_round = (uint64_t)(64 / G) * len;
  uint64_t b = 65536 / (per_round ? per_round : 1);
  return b < 1 ? 1u : (b > 64 ? 64u : (uint32_t)b);
}

template <int VAR>
int launch_stream_g(int G, dim3 grid, size_t lds, hipStream_t stream, const CrcParams& p) {
  const dim3 block(64 * waves_per_wg(kStreamWaves));
  switch (G) {
    case 1: hipLaunchKernelGGL((crc32c_stream_kernel<1, VAR>), grid, block, lds, stream, p); break;
    case 2: hipLaunchKernelGGL((crc32c_stream_kernel<2, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_stream_kernel<4, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_stream_kernel<8, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_stream_kernel<16, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
}

template <int VAR>
int launch_stream_v(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
  p.init_stride = p.init ? 1u : 0u;
  if (!p.init) p.init = t->zero_word;
  p.tab_main = t->main[gindex(G)];
  p.tab_tree = t->tree;
  p.bpg = stream_bpg(G, p.len);
  const uint64_t groups = 64 / G;
  const uint64_t rounds = (p.n_blocks + groups * p.bpg - 1) / (groups * p.bpg);
  const uint64_t nwaves = waves_per_wg(kStreamWaves);
  uint64_t wgs = (rounds + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  p.steal_limit = steal_limit(rounds, wgs, nwaves);
  // claim counters of this stream (left zeroed by the previous launch)
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const int levels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  const size_t lds = kMainBytes + levels * kTreeBytes;
  return launch_stream_g<VAR>(G, dim3(wgs), lds, stream, p);
}

// ---- rounds kernel (whole variable-length blocks in lockstep rounds) ----------
template <int MODE, int VAR>
int launch_rounds_g(int G, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const CrcParams& p) {
  if constexpr ((VAR & kVarOutPos) != 0) {  // large logs only: G = 8 (diagnostics A/B: 2, 4)
    if constexpr ((VAR & kVarDiag) != 0 && (VAR & kVarCached) != 0) {
      if (G == 2 || G == 4) {  // short records in sorted windows, default-policy loads
        if (G == 2) hipLaunchKernelGGL((crc32c_rounds_kernel<2, MODE, VAR>), grid, block, lds, stream, p);
        else hipLaunchKernelGGL((crc32c_rounds_kernel<4, MODE, VAR>), grid, block, lds, stream, p);
        return (int)hipGetLastError();
      }
    }
    if (G != 8) return NOVA_E_INVAL;
    hipLaunchKernelGGL((crc32c_rounds_kernel<8, MODE, VAR>), grid, block, lds, stream, p);
    return (int)hipGetLastError();
  } else if constexpr ((VAR & kVarCached) != 0 && (MODE == kLogWrite || MODE == kLogVerify)) {
    // default-policy log records run at 2 or 4 lanes only (launch_rounds)
    if (G == 2) hipLaunchKernelGGL((crc32c_rounds_kernel<2, MODE, VAR>), grid, block, lds, stream, p);
    else if (G == 4) hipLaunchKernelGGL((crc32c_rounds_kernel<4, MODE, VAR>), grid, block, lds, stream, p);
    else return NOVA_E_INVAL;
    return (int)hipGetLastError();
  } else {
  switch (G) {
    case 2: hipLaunchKernelGGL((crc32c_rounds_kernel<2, MODE, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_rounds_kernel<4, MODE, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_rounds_kernel<8, MODE, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_rounds_kernel<16, MODE, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
  }
}

// Descriptor arrays the rounds kernel always loads: absent ones read word 0
// of the zero line through a zero index mask (offset = offsets[i & omask] +
// i * stride, length = lengths[i & lmask] + len, init = init[i & imask]).
inline void rounds_params(int G, CrcParams& p, DevTables* t) {
  p.tab_main = t->main[gindex(G)];
  p.tab_tree = t->tree;
  p.tab_byte = t->byte8lm;
  p.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
  p.omask = p.lmask = p.imask = ~0ull;
  if (p.offsets) {
    p.stride = 0;
  } else {
    p.offsets = reinterpret_cast<const uint64_t*>(t->zero_word);
    p.omask = 0;
  }
  if (p.lengths) {
    p.len = 0;
  } else {
    p.lengths = t->zero_word;
    p.lmask = 0;
  }
  if (!p.init) {
    p.init = t->zero_word;
    p.imask = 0;
  }
}

// p.perm: the caller's order of blocks (null in the product).
template <int MODE, int VAR>
int launch_rounds_v(int G, CrcParams& p, DevTables* t, hipStream_t stream, uint32_t chunk = 0) {
  if (G < 2) G = 2;
  rounds_params(G, p, t);
  {
    const int so = g_tune_sort.load();
    p.sort_local = (so == 2 || so == 4) ? 1u : 0u;  // sort each chunk by step count
  }
  {
    // chunk = R rounds of 64/G blocks.  Default (plan() passes 0 only when
    // tuning forces G): log records 64, SSTable blocks 4 rounds, since a chunk
    // is also the unit of the tail balance and big blocks make big chunks.
    // plan() sizes both to the batch (latency-bound small batches).
    const uint32_t groups = 64u / (uint32_t)G;
    const bool log = MODE == kLogWrite || MODE == kLogVerify;
    uint32_t c = chunk ? chunk : (log ? 64u : 4u * groups);
    const int tc = g_tune_chunk.load();
    if (tc > 0) c = (uint32_t)tc;
    c = (c / groups) * groups;
    if (c < groups) c = groups;
    if (c > 64) c = 64;
    p.chunk = c;
  }
  p.n_chunks = (p.n_blocks + p.chunk - 1) / p.chunk;
  uint64_t nwaves = flat_waves();
  if ((VAR & kVarInit) && nwaves > (uint64_t)kInitMaxWaves) nwaves = kInitMaxWaves;  // launch bound
  if (VAR & kVarW16) nwaves = 16;
  uint64_t wgs = (p.n_chunks + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  if (wgs == 0) return 0;
  p.steal_limit = steal_limit(p.n_chunks, wgs, nwaves);
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const dim3 block(64 * nwaves);
  // + prefix masks, per-wave sort scratch (and the chunk epilogue's slot words)
  const size_t lds = flat_lds_g(G) + 272 + nwaves * 64 * 4 * ((VAR & (kVarRoundEpi | kVarNoTail)) ? 1 : 2);
  return launch_rounds_g<MODE, VAR>(G, dim3(wgs), block, lds, stream, p);
}

// ---- burst kernel (one SSTable per call) -----------------------------------------
template <int V, int MODE, int VAR = 0>
int launch_burst_v(CrcParams& p, DevTables* t, hipStream_t stream) {
  constexpr int G = BurstCfg<V>::kG;
  p.tab_main = V == 64 ? t->op1024 : V == 65 ? t->op1024r : t->main[gindex(16)];
  p.tab_tree = t->tree;
  p.tab_byte = t->byte8;
  p.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
  p.omask = p.lmask = p.imask = ~0ull;
  if (p.offsets) {
    p.stride = 0;
  } else {
    p.offsets = reinterpret_cast<const uint64_t*>(t->zero_word);
    p.omask = 0;
  }
  if (p.lengths) {
    p.len = 0;
  } else {
    p.lengths = t->zero_word;
    p.lmask = 0;
  }
  if (!p.init) {
    p.init = t->zero_word;
    p.imask = 0;
  }
  // one block per lane group; G = 16: at most one workgroup per CU (LDS), so
  // the waves per workgroup follow the batch to spread it over the CUs
  constexpr uint64_t per_wave = 64 / G;
  const uint64_t waves_needed = (p.n_blocks + per_wave - 1) / per_wave;
  // 4 waves per workgroup up to 2K blocks, 8 above (tools/latency_burst.py)
  uint64_t nw = (uint64_t)waves_per_wg(V == 64 && p.n_blocks <= 2048 ? 4 : BurstCfg<V>::kDefWaves);
  if (nw > (uint64_t)BurstCfg<V>::kWaves) nw = BurstCfg<V>::kWaves;
  uint64_t wgs = (waves_needed + nw - 1) / nw;
  if (V != 64) {
    const uint64_t cus = (uint64_t)t->cus;
    if (wgs < cus) {  // fewer waves per workgroup, more workgroups
      nw = (waves_needed + cus - 1) / cus;
      if (nw < 4) nw = 4;
      wgs = (waves_needed + nw - 1) / nw;
    }
    if (wgs > cus) wgs = cus;  // the rest by the grid-stride loop
  }
  hipLaunchKernelGGL((crc32c_burst_kernel<V, MODE, VAR>), dim3(wgs), dim3(64 * nw), burst_lds<V>(),
                     stream, p);
  return (int)hipGetLastError();
}

// XOR parity block over k data fragments (ltc/stoc_file_client_impl.cpp:334-349):
// parity[i] = XOR_f mem[frag_off[f] + i] for i < parity_len.  Like the
// reference, every fragment contributes parity_len bytes from its start (the
// reference loop reads past a shorter fragment's end).  Each thread makes kU
// 16-byte output chunks (grid-strided), so every fragment step issues kU
// independent loads.  A fragment's misalignment s is wave-uniform: unaligned
// fragments cost one more aligned load per chunk + v_alignbyte funnel shifts.
// Loads are clamped to the aligned 16 B holding the fragment's last byte, so
// nothing past the parity region's last 16-B line is touched; lanes past the
// end re-read the last chunk and discard it.
//
// FU fragments are loaded together (U * FU loads in flight per thread) when
// they are all 16-B aligned; a group with an unaligned fragment takes them one
// at a time through the funnel-shift path.
template <int U, int FU>
__global__ void __launch_bounds__(256) xor_parity_kernel(const uint8_t* base, const uint64_t* frag_off,
                                                         uint32_t n_frags, uint64_t parity_len,
                                                         uint8_t* out) {
  const uint64_t nchunks = (parity_len + 15) / 16;
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c0 < nchunks;
       c0 += U * nth) {
    uint32_t x[U][4] = {};
    uint64_t cc[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint64_t c = c0 + k * nth;
      cc[k] = c < nchunks ? c : nchunks - 1;
    }
    uint32_t f = 0;
    for (; f + FU <= n_frags; f += FU) {
      uint64_t fa[FU];
      uint32_t any_s = 0;
#pragma unroll
      for (int i = 0; i < FU; i++) {
        fa[i] = (uint64_t)base + frag_off[f + i];
        any_s |= (uint32_t)(fa[i] & 15);
      }
      if (any_s != 0) break;  // unaligned: the per-fragment path below
      uint4 v[FU][U];
#pragma unroll
      for (int i = 0; i < FU; i++)
#pragma unroll
        for (int k = 0; k < U; k++) v[i][k] = gload16(fa[i] + 16 * cc[k]);
#pragma unroll
      for (int i = 0; i < FU; i++)
#pragma unroll
        for (int k = 0; k < U; k++) {
          x[k][0] ^= v[i][k].x; x[k][1] ^= v[i][k].y; x[k][2] ^= v[i][k].z; x[k][3] ^= v[i][k].w;
        }
    }
    for (; f < n_frags; f++) {
      const uint64_t fa = (uint64_t)base + frag_off[f];
      const uint32_t s = (uint32_t)(fa & 15);
      const uint64_t fb = fa - s;                              // aligned line of byte 0
      const uint64_t lastline = (fa + parity_len - 1) & ~15ull;  // line of the last byte
      if (s == 0) {
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) v[k] = gload16(fb + 16 * cc[k]);
#pragma unroll
        for (int k = 0; k < U; k++) {
          x[k][0] ^= v[k].x; x[k][1] ^= v[k].y; x[k][2] ^= v[k].z; x[k][3] ^= v[k].w;
        }
      } else {
        uint4 lo[U], hi[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
          const uint64_t l = fb + 16 * cc[k];
          lo[k] = gload16(l);
          hi[k] = gload16(l + 16 <= lastline ? l + 16 : lastline);
        }
        const uint32_t ws = s >> 2, bs = s & 3;
#pragma unroll
        for (int k = 0; k < U; k++) {
          const uint32_t w[8] = {lo[k].x, lo[k].y, lo[k].z, lo[k].w,
                                 hi[k].x, hi[k].y, hi[k].z, hi[k].w};
#pragma unroll
          for (int e = 0; e < 4; e++) {
            // W[e+ws], W[e+ws+1] without dynamic register indexing
            uint32_t a = w[e], b = w[e + 1];
            if (ws == 1) { a = w[e + 1]; b = w[e + 2]; }
            else if (ws == 2) { a = w[e + 2]; b = w[e + 3]; }
            else if (ws == 3) { a = w[e + 3]; b = w[e + 4]; }
            x[k][e] ^= __builtin_amdgcn_alignbyte(b, a, bs);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
      const uint64_t c = c0 + k * nth;
      if (c >= nchunks) break;
      const uint64_t o = 16 * c;
      if (o + 16 <= parity_len) {
        u32x4 val = {x[k][0], x[k][1], x[k][2], x[k][3]};
        __builtin_nontemporal_store(val, (__attribute__((address_space(1))) u32x4*)(uint64_t)(out + o));
      } else {
        for (uint64_t i = o; i < parity_len; i++)
          out[i] = (uint8_t)(x[k][(i - o) >> 2] >> (8 * ((i - o) & 3)));
      }
    }
  }
}

}  // namespace
