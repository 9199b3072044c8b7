// MI355X (gfx950) batched CRC-32C: kernels, per-device tables, C-ABI batch
// entry points.  Drop-in for the per-SSTable-block checksum of NovaLSM
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
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/nova_crc32c.h"
#include "gf2_crc32c.hpp"

namespace {

constexpr int kWaves = 16;                 // waves per workgroup
constexpr int kThreads = kWaves * 64;
constexpr uint32_t kMainBytes = 131072;    // 4 tables x 256 x 32 replicas x 4 B
constexpr int kTreeLevels = 8;             // M4, M8, M16, ..., M512 (M256/M512: burst kernel)
constexpr uint32_t kTreeBytes = 4096;      // per level
constexpr uint32_t kWaveScratch = 512;     // per wave: 2x16 prefixes (+pad) + accumulators
constexpr int kNumG = 5;                   // G = 1, 2, 4, 8, 16

// kLogWrite / kLogVerify: offsets[i] points at a log record header
// [LE32 masked crc][LE16 length][type] (db/log_format.h:27-30); the CRC covers
// type byte + payload (db/log_writer.cc:112-114, db/log_reader.cc:251-262).
enum Mode { kStore = 0, kTrailer = 1, kVerify = 2, kLogWrite = 3, kLogVerify = 4 };

struct CrcParams {
  const uint8_t* base;
  const uint64_t* offsets;   // null: strided
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t len;
  uint32_t flags;
  const uint32_t* init;      // may be null (units kernel); stream kernel: never null
  uint32_t init_stride;      // 1, or 0 with init -> a zero word (stream kernel)
  uint32_t* out;             // kStore
  uint8_t* ok_out;           // kVerify
  uint32_t* n_bad;           // kVerify, may be null
  uint64_t n_blocks;
  uint32_t seg;              // segment bytes (multiple of 16); 0 = one unit per block
  uint32_t chunk;            // blocks per wave chunk (<= 16)
  uint64_t n_chunks;
  const uint32_t* tab_main;  // replicated LDS image, 32768 u32
  const uint32_t* tab_tree;  // kTreeLevels x 1024 u32
  const uint32_t* tab_ft;    // 16 x 1024 u32
  const uint32_t* tab_sh16;  // 32 x 1024 u32
  uint64_t* stamps;          // diagnostics: per-wave {tables loaded, done} (or null)
  uint32_t* sched;           // stream kernel: per-workgroup claim counters, 64 B apart
  uint32_t steal_limit;      // stream kernel: max other workgroups probed when out of work
  uint32_t bpg;              // stream kernel: consecutive blocks per lane group per round
  const uint32_t* tab_byte;  // flat kernel: one-byte step table M_1 (256 u32)
  const uint8_t* zline;      // flat kernel: 16 zero bytes (target of masked-off loads)
  // flat kernel: descriptor arrays are always loaded (no branch), absent ones
  // read word 0 of zline through a zero mask; offset = offsets[i & omask] +
  // i * stride, length = lengths[i & lmask] + len, init = init[i & imask].
  uint64_t omask, lmask, imask;
  const uint32_t* perm;      // rounds kernel: block index per sorted position (or null)
  uint32_t sort_local;       // rounds kernel: sort each chunk's blocks by step count
  uint64_t buf_len;          // log modes: bytes of the log image at base (bounds of every record)
  // log-stream kernel (crc32c_logstream_kernel) and its gated fallback
  const uint32_t* first;     // first record of each 32 KiB log block (n_lblocks + 1 entries)
  uint64_t n_lblocks;        // log blocks in the image
  uint32_t* ls_flag;         // bit 0: offsets unsorted (pre-pass), bit 1: records overlap
  uint32_t* ls_bad;          // log-stream mismatch count (added to n_bad unless it falls back)
  uint32_t* ls_left;         // records the log-stream kernel leaves to the rounds follow-up
  const uint32_t* gate;      // rounds kernel: run only if *gate != 0 (else fold ls_bad in)
  // trailer writer (rounds kernel): *tr_flag == 0 (trailer_layout_kernel found
  // the blocks ascending and disjoint) lets each block with init[i] != 0 (the
  // pre-pass's eligibility array) rewrite the whole 64-B pieces holding its
  // trailer; null or nonzero: byte stores
  const uint32_t* tr_flag;
  uint32_t wvar;  // diagnostics (timing): 1 = whole-piece stores non-temporal, 2 = no result writes
};

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

// Kernel variants (diagnostics / tuning; 0 = production).
constexpr int kVarNoLookup = 1;  // ablation: stream step without table lookups
constexpr int kVarCached = 2;    // default-policy data loads (production uses nt)
constexpr int kVarStamps = 4;    // record per-wave s_memrealtime stamps (diagnostics)
constexpr int kVarStaticClaims = 8;  // stream kernel: claims without atomics (diagnostics)
constexpr int kVarNarrow = 16;  // flat/rounds/units: one word's lookups in flight (fold4, A/B)
constexpr int kVarWide = 32;    // stream kernel: a swath's 16 lookups in flight (fold4w, A/B)
[[maybe_unused]] constexpr int kVarLsFast = 64;  // log-stream kernel: every swath on the fast path (ablation: WRONG CRCs)
constexpr int kVarInit = 128;   // rounds kernel, store mode: per-block init values (general head masking)
[[maybe_unused]] constexpr int kVarNoTail = 256;  // rounds kernel ablation: no tail-line loads (WRONG CRCs)

// 16-byte load through the global (not flat) address space.  Block bytes are
// read exactly once, so production loads carry the nt policy: on gfx950 it
// bypasses L1 and streams ~9% faster than the default policy at every block
// size measured (tools/ceiling.py).
template <int VAR = 0>
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  u32x4 v;
  if constexpr ((VAR & kVarCached) != 0)
    v = *reinterpret_cast<gu32x4*>(addr);
  else
    v = __builtin_nontemporal_load(reinterpret_cast<gu32x4*>(addr));
  return make_uint4(v.x, v.y, v.z, v.w);
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

// v of lane (lane ^ K), K a power of two known at compile time.  Within a
// 16-lane row without an LDS round trip (__shfl_xor is a ds_bpermute): DPP for
// k <= 8 (quad_perm; xor 4 = row_half_mirror after quad_perm [3,2,1,0]; xor 8 =
// row_mirror after row_half_mirror); 16 and 32 cross rows (ds_bpermute).
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
  } else {
    // 16, 32: ds_bpermute.  With the gfx950 permlane swaps here the burst
    // kernel's trailer launch took 2.4 us longer at 16 blocks and one
    // log-stream experiment case (diagnostics build) failed, so they are not used.
    static_assert(K == 16 || K == 32, "lane_xor: 1, 2, 4, 8, 16 or 32");
    return (uint32_t)__shfl_xor((int)v, K);
  }
}
// max over the wave's 64 lanes (every lane gets it)
__device__ __forceinline__ uint32_t wave_max(uint32_t m) {
  m = max(m, lane_xor<32>(m));
  m = max(m, lane_xor<16>(m));
  m = max(m, lane_xor<8>(m));
  m = max(m, lane_xor<4>(m));
  m = max(m, lane_xor<2>(m));
  return max(m, lane_xor<1>(m));
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

template <int G, int MODE, int VAR = 0>
__global__ void __launch_bounds__(kThreads) crc32c_units_kernel(CrcParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLevels * kTreeBytes / 16, nullptr, 0);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane & (G - 1);   // lane within its group
  const int grp = lane / G;       // group within the wave
  constexpr int kGroups = 64 / G;
  uint32_t* wpre = reinterpret_cast<uint32_t*>(lds + kMainBytes + kLevels * kTreeBytes +
                                               wave * kWaveScratch);
  uint32_t* wacc = wpre + 64;
  uint32_t* wsort = wpre + 32;  // chunk lanes in descending unit-size order
  const uint64_t zl = (uint64_t)p.zline;  // 16 zero bytes
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t extra = (MODE == kVerify) ? 1u : 0u;  // verify covers block + type byte

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
    // -- prologue: lane i < chunk owns block b = chunk*chunk_size + i
    const uint64_t b = chunk * p.chunk + lane;
    const bool valid = lane < (int)p.chunk && b < p.n_blocks;
    uint64_t a = 0;
    uint32_t n = 0, init = 0;
    uint32_t lstat = NOVA_LOG_OK;  // log modes: record status (log_status)
    if (valid) {
      a = (uint64_t)p.base + (p.offsets ? p.offsets[b] : b * p.stride);
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
        n = (p.lengths ? p.lengths[b] : p.len) + extra;
      }
      init = p.init ? p.init[b] : 0u;
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
        for (uint32_t i = 0; i < n; i++) l = byte_step(l, ((const uint8_t*)a)[i]);
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
        const uint8_t* d = (const uint8_t*)a;
        const uint32_t stored = (uint32_t)d[n] | ((uint32_t)d[n + 1] << 8) |
                                ((uint32_t)d[n + 2] << 16) | ((uint32_t)d[n + 3] << 24);
        const bool ok = unmask_crc(stored) == crc;  // table/table.cc:435-437
        p.ok_out[b] = ok ? 1 : 0;
        if (!ok && p.n_bad) atomicAdd(p.n_bad, 1u);
      } else {
        if (p.flags & NOVA_CRC32C_APPEND_TYPE) {  // table/table_builder.cc:203
          crc = ~byte_step(~crc, (p.flags >> 8) & 0xffu);
        }
        if (MODE == kTrailer) {
          const uint32_t m = mask_crc(crc);
          store_trailer((uint8_t*)a + n, (p.flags >> 8) & 0xffu, m,
                        (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
        } else {
          if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
          p.out[b] = crc;
        }
      }
    }
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

// ---- crc32c_flat_kernel<G, MODE> -------------------------------------------
// Variable-length batches (any alignment and length; per-block init; all
// modes).  Every lane group walks its own sequence of WHOLE blocks, one
// 4-swath step (64G bytes) at a time, and the wave streams all its groups'
// steps as one flat sequence with the next step's loads in flight while the
// current one folds -- across block boundaries, like the stream kernel.  The
// groups of a wave change blocks independently, so a wave never waits for its
// longest block (the units kernel's rounds did) and no block is split.
//
//   * Region of a block [u0,u1): its steps end at E = u1 & ~15 (16-B aligned)
//     and start at E - S*64G <= u0 & ~15.  Pieces before u0 read as zero (a
//     zero register ignores leading zeros; they are not loaded), ~init is
//     xor-ed into the bytes [u0,u0+4).  After the group fold the register at E
//     is M4(V); the 0..15 tail bytes [E,u1) (loaded with the last step) finish
//     it with <= 3 word steps (M4 in LDS) and <= 3 byte steps (M1 in LDS).
//   * Blocks reach the groups through per-wave chunks of C consecutive block
//     descriptors held one per lane, in two banks (current and next).  The
//     groups whose block ended take the next positions of the chunk sequence
//     (ballot + popcount), reading the descriptor from its lane (bpermute).
//     A bank is refilled as soon as it is used up, so its loads are at least
//     one step old when first read and never drain the data prefetch.
//   * Chunks are claimed like the units kernel's (per-workgroup counters,
//     bounded stealing), one claim ahead, the claim issued from inline asm
//     with EXEC = lane 0 and collected after >= one step of loads.
//   * Log modes: descriptors are record headers; the refill loads the offsets,
//     the next step loads the header bytes, the one after packs them.
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
};

constexpr uint64_t kNoChunk = ~0ull;
constexpr int kFlatMaxWaves = 12;  // 3 waves per SIMD: up to 168 VGPRs, no spills
constexpr int kFlatThreads = kFlatMaxWaves * 64;

__device__ __forceinline__ uint32_t sel5(uint32_t k, uint32_t a, uint32_t b, uint32_t c,
                                         uint32_t d, uint32_t e) {
  return k == 0 ? a : k == 1 ? b : k == 2 ? c : k == 3 ? d : e;
}

// ---- shared by the flat and rounds kernels ---------------------------------
// Issue one 4-swath step of a block region for this lane (pieces before the
// block's first line, or of an invalid group, read the zero line) plus, on the
// block's last step, its tail line(s).
//
// kLines (rounds kernel): the step grid is aligned to 16G-byte lines, so each
// swath of a group is one aligned 16G-byte line (an unaligned grid splits
// every group-swath over two cache lines: measured 61.5% vs 71.5% of HBM peak
// on 4 KiB blocks).  The region then ends at Le = roundup(E, 16G) >= E; the
// last step's last swath holds the pieces at or after E, which read the zero
// line here and leave their lane's registers unchanged in fold_step.
template <int G, int VAR, bool kTail2, bool kLines = false>
__device__ __forceinline__ void load_step(FlatSet& X, uint64_t lp, uint64_t u0, uint64_t u1,
                                          uint64_t end, bool v, bool last, uint64_t zl, int q) {
  const uint64_t A0 = u0 & ~15ull;
  const bool nz = v && u1 > u0;
  const uint64_t pa = lp + 16 * q;
  const uint64_t a0 = pa, a1 = pa + 16 * G, a2 = pa + 32 * G, a3 = pa + 48 * G;
  const bool in3 = !kLines || !last || a3 < end;
  X.d0 = gload16<VAR>((nz && a0 >= A0) ? a0 : zl);
  X.d1 = gload16<VAR>((nz && a1 >= A0) ? a1 : zl);
  X.d2 = gload16<VAR>((nz && a2 >= A0) ? a2 : zl);
  X.d3 = gload16<VAR>((nz && a3 >= A0 && in3) ? a3 : zl);
  if constexpr (kTail2) {
    const uint64_t ta = last ? end : zl;  // holds the stored CRC's first byte
    X.t = gload16<VAR>(ta);
    X.t2 = gload16<VAR>((last && u1 + 4 > end + 16) ? end + 16 : ta);
  } else {
    X.t = gload16<VAR>((last && nz && (u1 & 15)) ? end : zl);
  }
}

// Mask the head piece(s) of a step (bytes before u0, ~init at u0) and run it
// through the lane's four stream registers.  A piece needs it only if it holds
// a byte of [u0, u0+4): pieces wholly before u0 were loaded from the zero line
// (load_step) and are zero already.  No region piece holds a byte at or after
// u1 (regions end at E = u1 & ~15; the tail bytes come from the tail line).
template <int G, int VAR, bool kTail2, bool kLines = false>
__device__ __forceinline__ void fold_step(const uint8_t* lds, const FlatSet& Y, int q, uint32_t& c0,
                                          uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t lo0,
                                          uint32_t lo1, uint32_t lo2, uint32_t lo3) {
  const int32_t h = rel32(Y.u0, Y.pa + 16 * q, 48 * G + 16);
  uint4 d0 = Y.d0, d1 = Y.d1, d2 = Y.d2, d3 = Y.d3;
  if (is_head(h)) d0 = head_piece(d0, h, Y.ninit);
  if (is_head(h - 16 * G)) d1 = head_piece(d1, h - 16 * G, Y.ninit);
  if (is_head(h - 32 * G)) d2 = head_piece(d2, h - 32 * G, Y.ninit);
  if (is_head(h - 48 * G)) d3 = head_piece(d3, h - 48 * G, Y.ninit);
  if (kLines && Y.last) {  // wave-uniform: the region's last line may end past E
    swath4<VAR>(lds, c0, c1, c2, c3, d0, lo0, lo1, lo2, lo3);
    swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
    swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
    const uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = c3;
    swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
    if (Y.pa + 16 * q + 48 * G >= (Y.u1 & ~15ull)) {  // piece at or after E: not in the region
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
  // the tail line(s) are used only on a block's last step: consume anyway, so
  // the compiler resolves their loads here with an exact count
  asm volatile("" ::"v"(Y.t.x), "v"(Y.t.y), "v"(Y.t.z), "v"(Y.t.w));
  if constexpr (kTail2) asm volatile("" ::"v"(Y.t2.x), "v"(Y.t2.y), "v"(Y.t2.z), "v"(Y.t2.w));
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

#ifdef NOVA_DIAG
// The flat kernel is measured slower than the rounds kernel on every workload
// (DESIGN.md 3.5): diagnostics build only.
template <int G, int MODE, int VAR = 0>
__global__ void __launch_bounds__(kFlatThreads) crc32c_flat_kernel(CrcParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  constexpr uint32_t kByteTab = kMainBytes + kLevels * kTreeBytes;
  constexpr bool kLog = MODE == kLogWrite || MODE == kLogVerify;
  constexpr bool kTail2 = MODE == kVerify;  // stored CRC follows the CRC input
  constexpr uint64_t kStep = 64 * G;
  static_assert(kByteTab == kMainBytes + kLevels * kTreeBytes, "byte table follows the tree");
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLevels * kTreeBytes / 16, p.tab_byte, 64);
  __syncthreads();

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
  const uint32_t C = p.chunk;  // kGroups <= C <= 64
  const uint32_t nwg = gridDim.x;
  const uint32_t nwaves = blockDim.x >> 6;

  // ---- chunk claims (wave-uniform) ------------------------------------------
  // A compiler-visible atomic by lane 0.  (Issued from inline asm, as the
  // stream kernel does, the compiler copied the result register before the
  // atomic had returned.)  The claim for the next switch is issued in the
  // loop body's second take and read at the next switch, a step or more later.
  uint32_t victim = blockIdx.x, tried = 0, req = 0;
  bool claim_due = false;  // the next switch's claim is still to be issued
  auto claim = [&](uint32_t v) {
    uint32_t r = 0;
    if (lane == 0)
      r = __hip_atomic_fetch_add(p.sched + v * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    req = r;
  };
  auto chunk_of = [&](uint32_t v, uint32_t idx) -> uint64_t {
    const uint64_t c = ((uint64_t)idx + nwaves) * nwg + v;  // first nwaves chunks implicit
    return c < p.n_chunks ? c : kNoChunk;
  };
  // The chunk of the claim in req (issued in the second take since the last
  // switch, or just before in the prologue); steal if exhausted.
  auto collect = [&]() -> uint64_t {
    uint64_t c = chunk_of(victim, __builtin_amdgcn_readfirstlane(req));
    while (c == kNoChunk && ++tried < p.steal_limit + 1) {
      victim = (victim + 1) % nwg;
      claim(victim);
      c = chunk_of(victim, __builtin_amdgcn_readfirstlane(req));
    }
    return c;
  };

  // ---- descriptor banks (LDS): bank k, slot i = block chunk_k*C + i -------------
  // A refill loads the chunk's descriptors into registers (t_*); the next take,
  // at least one step later, writes them to the wave's LDS bank, so neither
  // the write nor any read waits on fresh loads.  (Registers as banks made
  // the compiler copy fresh load results between registers at once, which
  // drained the data prefetch at every refill.)  Log modes: the next take
  // loads the header bytes, the one after packs and writes them.
  const uint32_t desc_base = kByteTab + 1024u + (uint32_t)wave * 2u * C * 16u;
  auto desc_at = [&](uint32_t bank, uint32_t i) -> uint4* {
    return reinterpret_cast<uint4*>(lds + desc_base + (bank * C + i) * 16u);
  };
  uint32_t t_olo = 0, t_ohi = 0, t_len = 0, t_aux = 0;      // descriptor words in flight
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0, h5 = 0, h6 = 0;  // log: header bytes in flight
  int pend = 0;            // 1: LDS write due (log: header loads due), 2: log pack + write due
  uint32_t pend_bank = 0;
  uint64_t ch0 = kNoChunk, ch1 = kNoChunk;  // chunk held by bank 0 / 1
  const uint32_t my = (uint32_t)lane < C ? (uint32_t)lane : C - 1;
  auto refill = [&](uint64_t chunk, uint32_t bank) {
    uint64_t rec = (chunk == kNoChunk ? 0 : chunk * C) + my;
    if (rec >= p.n_blocks) rec = p.n_blocks - 1;
    const uint64_t o = p.offsets[rec & p.omask];
    t_olo = (uint32_t)o;
    t_ohi = (uint32_t)(o >> 32);
    if constexpr (!kLog) {
      t_len = p.lengths[rec & p.lmask];
      t_aux = p.init[rec & p.imask];
    }
    if (bank) ch1 = chunk;
    else ch0 = chunk;
    pend = 1;
    pend_bank = bank;
  };
  // The descriptor pipeline runs at fixed points of the two-step loop body, so
  // every value in it has one producer and one consumer (no register copies,
  // which would wait on the loads): refill in the first take, LDS write in
  // the second (log: header loads in the second, pack + write in the next
  // first).
  auto step_pending = [&](bool first) {
    if constexpr (kLog) {
      const uint64_t o = ((uint64_t)t_ohi << 32) | t_olo;
      if (pend == 1 && !first) {
        const uint8_t* h = log_header_fits(o, p.buf_len) ? (const uint8_t*)(base + o) : p.zline;
        h4 = h[4];
        h5 = h[5];
        if constexpr (MODE == kLogVerify) {
          h0 = h[0];
          h1 = h[1];
          h2 = h[2];
          h3 = h[3];
          h6 = h[6];
        }
        pend = 2;
        return;
      }
      if (pend != 2 || !first) return;
      const uint32_t length = h4 | (h5 << 8);  // type byte + payload (db/log_format.h:27-30)
      const uint32_t ls = log_header_fits(o, p.buf_len)
                              ? log_status(o, length, MODE == kLogVerify ? h6 : 1u, p.buf_len)
                              : log_nohdr_status(o, p.buf_len);
      t_len = ls == NOVA_LOG_OK ? 1u + length : 0u;  // 0: not read, t_aux = status
      t_aux = ls == NOVA_LOG_OK ? (h0 | (h1 << 8) | (h2 << 16) | (h3 << 24)) : ls;
    } else {
      if (pend != 1 || first) return;
    }
    if ((uint32_t)lane < C) *desc_at(pend_bank, lane) = make_uint4(t_olo, t_ohi, t_len, t_aux);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    pend = 0;
  };
  auto complete_pending = [&]() {  // out of order (drains); only when C is small
    step_pending(false);
    step_pending(true);
  };

  // ---- per-group block state (load side; group-uniform values) ---------------
  uint64_t g_u0 = 0, g_u1 = 0, g_lp = 0, g_end = 0, g_rec = 0;
  uint32_t g_ninit = 0, g_st = 0;
  bool g_valid = false, g_need = true;
  uint32_t pos = 0;     // next position in the current bank
  uint32_t cb = 0;      // current bank
  bool dry = false;     // no more chunks for this wave

  // first: the loop body's first take (the only one that switches banks and
  // refills; positions may run past the current bank into the other one
  // meanwhile: C >= 2 groups keeps them below 2C).
  // Values loaded in one take and used only conditionally later are consumed
  // here unconditionally (an empty asm reading them), so the compiler
  // resolves their loads at a fixed point with an exact count instead of
  // waiting for all loads wherever its paths merge.
  auto take = [&](bool first) {
    if (first) {
      asm volatile("" ::"v"(req));
      if constexpr (kLog)
        asm volatile("" ::"v"(h0), "v"(h1), "v"(h2), "v"(h3), "v"(h4), "v"(h5), "v"(h6));
    } else {
      asm volatile("" ::"v"(t_olo), "v"(t_ohi), "v"(t_len), "v"(t_aux));
    }
    step_pending(first);
    if (!first && claim_due) {
      claim(victim);
      claim_due = false;
    }
    const uint64_t needm = __ballot(g_need && q == 0);
    const uint32_t cnt = (uint32_t)__popcll(needm);
    if (pend && pos + cnt > C) complete_pending();  // reads the refilled bank (small C only)
    const uint32_t rank = (uint32_t)__popcll(needm & ((1ull << (grp * G)) - 1));
    const uint32_t s = pos + rank;
    const bool oth = s >= C;  // past the current bank: the other one
    const uint32_t idx = oth ? s - C : s;
    const uint32_t bank = oth ? cb ^ 1u : cb;
    if (g_need) {  // (no group needing a block: only the switch check below)
      const uint4 d = *desc_at(bank, idx);
      const uint64_t cid = bank ? ch1 : ch0;
      const uint64_t rec = cid * C + idx;
      const bool ok = cid != kNoChunk && rec < p.n_blocks;
      uint64_t a = base + (((uint64_t)d.y << 32) | d.x) + rec * p.stride;
      if (kLog) a += 6;  // CRC input starts at the type byte (db/log_writer.cc:112)
      const uint32_t n = d.z + p.len + extra;
      const uint32_t aux = d.w;
      g_valid = ok;
      g_need = false;
      g_u0 = a;
      g_u1 = a + n;
      g_rec = rec;
      // ~init goes into the data's first 4 bytes; a block shorter than 4 bytes
      // gets it at the end instead (R ^= M_n(~init), see fold).
      g_ninit = (raw || n < 4) ? 0u : ~((kLog || MODE == kTrailer) ? 0u : aux);  // log records: Value(), init 0
      g_st = aux;
      const uint64_t E = g_u1 & ~15ull;
      const uint64_t A0 = a & ~15ull;
      uint64_t S = (E - A0 + kStep - 1) / kStep;
      if (S == 0) S = 1;
      g_end = E;
      g_lp = E - S * kStep;
    }
    pos += cnt;
    // Checked in every first take, even with no block taken: the second take
    // may then run past the current bank by < 1 group count, never past the
    // other one (positions < C + 2 * groups <= 2C).
    if (first && pos >= C) {  // the current bank is used up: switch, refill it
      pos -= C;
      cb ^= 1u;
      uint64_t nc = kNoChunk;
      if (!dry) {
        nc = collect();
        if (nc == kNoChunk) dry = true;
        else claim_due = true;
      }
      refill(nc, cb ^ 1u);
    }
  };

  auto issue = [&](FlatSet& X) -> bool {
    const bool v = g_valid;
    const bool last = v && (g_lp + kStep == g_end);
    load_step<G, VAR, kTail2>(X, g_lp, g_u0, g_u1, g_end, v, last, zl, q);
    X.pa = g_lp;
    X.u0 = g_u0;
    X.u1 = g_u1;
    X.rec = g_rec;
    X.ninit = v ? g_ninit : 0u;
    X.st = g_st;
    X.valid = v;
    X.last = last;
    if (v) g_lp += kStep;
    if (last) g_need = true;
    return __ballot(v) != 0;
  };

  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  bool wb_on = false;  // a finished block's write is pending (lane q == 0)
  uint64_t wb_a = 0;
  uint32_t wb_v = 0;
  auto fold = [&](FlatSet& Y) {
    fold_step<G, VAR, kTail2>(lds, Y, q, c0, c1, c2, c3, lo0, lo1, lo2, lo3);
    if (Y.last) {  // group-uniform
      const uint32_t v = group_fold<G>(lds, c0, c1, c2, c3, q);
      c0 = c1 = c2 = c3 = 0;
      // The memory write waits until after the next step's loads are issued
      // (writeback): a store here would make the compiler drain the prefetch
      // before the store's address registers are reused.
      finish_block<MODE>(lds, kByteTab, p, raw, v, Y, wb_a, wb_v);
      wb_on = q == 0;
    }
  };
  auto writeback = [&]() {
    if (wb_on) {
      write_result<MODE>(p, wb_a, wb_v);
      wb_on = false;
    }
  };

  // ---- prologue: wave k's first chunk is implicit, the second is claimed ------
  {
    uint64_t c0 = (uint64_t)wave * nwg + blockIdx.x;
    if (c0 >= p.n_chunks) {
      claim(victim);
      c0 = collect();
    }
    if (c0 == kNoChunk) dry = true;
    refill(c0, 0);
    complete_pending();
    uint64_t c1 = kNoChunk;
    if (!dry) {
      claim(victim);
      c1 = collect();
      if (c1 == kNoChunk) dry = true;
      else claim_due = true;
    }
    refill(c1, 1);
    complete_pending();
  }
  // The loop starts by folding an empty set A (zeros, not valid): no data
  // load is in flight when the loop is entered, so the compiler's wait
  // counts at the loop head follow the steady state (an A issued before the
  // loop made it wait for everything there, every iteration).
  FlatSet A, B;
  A.d0 = A.d1 = A.d2 = A.d3 = A.t = A.t2 = make_uint4(0, 0, 0, 0);
  A.pa = A.u0 = A.u1 = A.rec = 0;
  A.ninit = A.st = 0;
  A.valid = A.last = A.head = A.l3 = A.wsec = false;
  for (;;) {
    take(true);
    issue(B);
    writeback();
    fold(A);
    // No exit here: a mid-body exit makes the CFG structurizer add a path
    // that enters the loop head with B's loads outstanding, and the head then
    // waits for all loads every iteration.  A B without valid groups costs
    // one more (empty) half.
    take(false);
    const bool a_live = issue(A);
    writeback();
    fold(B);
    if (!a_live) break;
  }
  writeback();
  // The last claim (if any) must have returned before this workgroup counts
  // itself finished: the last workgroup then zeroes the counters.
  __builtin_amdgcn_s_waitcnt(0);
  sched_release(p.sched);
}
#endif  // NOVA_DIAG

// ---- binning pre-pass + crc32c_rounds_kernel<G, MODE> ------------------------
// Variable-length batches in ROUNDS: the wave's lane groups take kGroups blocks
// at a time, all padded to the round's step count (its largest block, end-
// aligned, so shorter blocks start later on zero pieces that leave a zero
// register unchanged).  Every group starts and ends the round together, so the
// per-block work (group fold, tail, epilogue) runs once per round for all
// groups, not divergently per block as in the flat kernel; the loads stream
// across rounds and chunks as in the stream kernel.  For the rounds to be
// even, a pre-pass sorts the batch by step count, largest first (a counting
// sort into 256 classes: exact below 128 steps, 16 per octave above), which
// also hands the last, smallest work to the tail of the launch.

#ifdef NOVA_DIAG
// The whole-batch sort was measured slower than sorting each claimed chunk
// (DESIGN.md 3.5a): diagnostics build only.
constexpr int kBins = 256;

__device__ __forceinline__ uint32_t steps_class(uint64_t S) {
  if (S < 128) return (uint32_t)S;
  const uint32_t lg = 63u - (uint32_t)__builtin_clzll(S);  // >= 7
  const uint32_t c = 128u + (lg - 7u) * 16u + (uint32_t)((S >> (lg - 4)) & 15u);
  return c > 255u ? 255u : c;
}

// Step count of block b (region [A0, E) in kStep-byte steps), as the rounds
// kernel computes it; rank = 255 - class orders the largest first.
template <int MODE>
__device__ __forceinline__ uint32_t block_rank(const CrcParams& p, uint64_t b, uint64_t kStep) {
  constexpr bool kLog = MODE == kLogWrite || MODE == kLogVerify;
  uint64_t a = (uint64_t)p.base + p.offsets[b & p.omask] + b * p.stride;
  uint32_t n;
  if constexpr (kLog) {
    const uint8_t* h = (const uint8_t*)a;
    n = 1u + ((uint32_t)h[4] | ((uint32_t)h[5] << 8));
    a += 6;
  } else {
    n = p.lengths[b & p.lmask] + p.len + (MODE == kVerify ? 1u : 0u);
  }
  const uint64_t E = (a + n) & ~15ull, A0 = a & ~15ull;
  uint64_t S = (E - A0 + kStep - 1) / kStep;
  if (S == 0) S = 1;
  return 255u - steps_class(S);
}

template <int MODE>
__global__ void __launch_bounds__(256) bin_count_kernel(CrcParams p, uint64_t kStep, uint32_t* hist) {
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < p.n_blocks; b += nth)
    atomicAdd(&h[block_rank<MODE>(p, b, kStep)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// hist -> cursor: exclusive prefix over the ranks (one workgroup of kBins threads).
__global__ void __launch_bounds__(kBins) bin_scan_kernel(const uint32_t* hist, uint32_t* cursor) {
  __shared__ uint32_t t[kBins];
  const int i = threadIdx.x;
  t[i] = hist[i];
  __syncthreads();
  for (int d = 1; d < kBins; d <<= 1) {
    const uint32_t v = i >= d ? t[i - d] : 0u;
    __syncthreads();
    t[i] += v;
    __syncthreads();
  }
  cursor[i] = t[i] - hist[i];
}

// Same grid-stride assignment as bin_count_kernel: each workgroup reserves its
// ranges per class with one atomic, then places its blocks.
template <int MODE>
__global__ void __launch_bounds__(256) bin_scatter_kernel(CrcParams p, uint64_t kStep, uint32_t* cursor,
                                                          uint32_t* perm) {
  __shared__ uint32_t h[kBins];
  __shared__ uint32_t base[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < p.n_blocks; b += nth)
    atomicAdd(&h[block_rank<MODE>(p, b, kStep)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) {
    base[i] = h[i] ? atomicAdd(&cursor[i], h[i]) : 0u;
    h[i] = 0;
  }
  __syncthreads();
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < p.n_blocks; b += nth) {
    const uint32_t r = block_rank<MODE>(p, b, kStep);
    perm[base[r] + atomicAdd(&h[r], 1u)] = (uint32_t)b;
  }
}
#endif  // NOVA_DIAG

template <int G, int MODE, int VAR = 0>
__global__ void __launch_bounds__(kFlatThreads) crc32c_rounds_kernel(CrcParams p0) {
  CrcParams p = p0;  // the log-stream follow-up narrows the batch below
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int kLevels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  constexpr uint32_t kByteTab = kMainBytes + kLevels * kTreeBytes;
  constexpr bool kLog = MODE == kLogWrite || MODE == kLogVerify;
  constexpr bool kTail2 = MODE == kVerify;
  constexpr uint64_t kStep = 64 * G;
  constexpr uint32_t kGroups = 64 / G;
  static_assert(kByteTab == kMainBytes + kLevels * kTreeBytes, "byte table follows the tree");
#ifdef NOVA_DIAG
  if (p.gate) {  // follow-up of the log-stream kernel
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
#endif
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
#ifdef NOVA_DIAG
  const bool sect = (MODE == kTrailer || MODE == kLogWrite) && G >= 8 && p.tr_flag &&
                    *p.tr_flag == 0;
#else
  constexpr bool sect = false;
#endif

  // ---- chunk claims (as the flat kernel) ---------------------------------------
  uint32_t victim = blockIdx.x, tried = 0, req = 0;
  auto claim = [&](uint32_t v) {
    uint32_t r = 0;
    if (lane == 0)
      r = __hip_atomic_fetch_add(p.sched + v * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    req = r;
  };
  auto chunk_of = [&](uint32_t v, uint32_t idx) -> uint64_t {
    const uint64_t c = ((uint64_t)idx + nwaves) * nwg + v;
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
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0, h5 = 0, h6 = 0;
  uint64_t n_u0 = 0, c_u0 = 0;
  uint32_t n_n = 0, n_rec = 0, n_aux = 0, c_n = 0, c_rec = 0, c_aux = 0;
  uint32_t t_ok = 0, n_ok = 0, c_ok = 0;  // slot holds a block of the batch
  uint32_t n_chunk = kNone, c_chunk = kNone, t_chunk = kNone;
  // wave-uniform state packed in one word (fewer scalar registers)
  constexpr uint32_t fReady = 1, fRefill = 2, fDry = 4, fDone = 8, fRoundDone = 16, fClaim = 32;
  uint32_t fl = 0;
  uint32_t stage = 0;  // next pipeline stage due (0: none)
  const uint32_t my = (uint32_t)lane < C ? (uint32_t)lane : C - 1;
  // Sort the loaded chunk's slots by step count, largest first (rank by
  // shuffles, inverse permutation through the wave's LDS scratch), so each
  // round's blocks have similar lengths while the chunk keeps its locality.
  uint32_t* const sortbuf = reinterpret_cast<uint32_t*>(lds + kByteTab + 1024u + 272u) + wave * 64;
  auto sort_nxt = [&]() {
    n_ok = t_ok;
    if (!p.sort_local) return;
    uint32_t S = 0;
    if (t_ok) {
      const uint64_t E = (n_u0 + n_n) & ~15ull;
      const uint64_t s64 = (E - (n_u0 & ~15ull) + kStep - 1) / kStep;
      S = s64 == 0 ? 1u : (s64 > 0xffffffffull ? 0xffffffffu : (uint32_t)s64);
    }
    uint32_t rank = 0;
    for (int j = 0; j < 64; j++) {
      // lane j's key as a wave-uniform scalar (v_readlane: no LDS round trip)
      const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)S, j);
      rank += (sj > S || (sj == S && j < lane)) ? 1u : 0u;
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
    n_ok = __shfl(t_ok, src);
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
      stage = 3;
    } else if (st == 3) {
      const uint64_t a = base + (((uint64_t)t_ohi << 32) | t_olo) + (uint64_t)t_rec * p.stride;
      if constexpr (kLog) {
        // a header past its log block / the image is not read (bounds, status)
        const uint64_t o = ((uint64_t)t_ohi << 32) | t_olo;
        const uint8_t* h = log_header_fits(o, p.buf_len) ? (const uint8_t*)a : p.zline;
        h4 = h[4];
        h5 = h[5];
        if constexpr (MODE == kLogVerify) {
          h0 = h[0];
          h1 = h[1];
          h2 = h[2];
          h3 = h[3];
          h6 = h[6];
        }
        stage = 4;
      } else {
        n_u0 = a;
        n_n = t_len + p.len + extra;
        n_rec = t_rec;
        n_aux = t_aux;
        n_chunk = t_chunk;
        sort_nxt();
        fl |= fReady;
        stage = 0;
      }
    } else if (st == 4) {
      const uint64_t o = ((uint64_t)t_ohi << 32) | t_olo;
      n_u0 = base + o + 6;  // CRC input: type byte + payload
      const uint32_t length = h4 | (h5 << 8);  // db/log_format.h:27-30
      const uint32_t ls = log_header_fits(o, p.buf_len)
                              ? log_status(o, length, MODE == kLogVerify ? h6 : 1u, p.buf_len)
                              : log_nohdr_status(o, p.buf_len);
      n_n = ls == NOVA_LOG_OK ? 1u + length : 0u;  // 0: not read, n_aux = status
      n_rec = t_rec;
      n_aux = ls == NOVA_LOG_OK ? (MODE == kLogWrite ? t_aux : (h0 | (h1 << 8) | (h2 << 16) | (h3 << 24)))
                                : ls;
      n_chunk = t_chunk;
      sort_nxt();
      fl |= fReady;
      stage = 0;
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
  uint32_t g_ninit = 0, g_st = 0;
  bool g_valid = false;
  uint32_t r_idx = R, r_step = 0, r_S = 0;
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
        c_u0 = n_u0;
        c_n = n_n;
        c_rec = n_rec;
        c_aux = n_aux;
        c_ok = n_ok;
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
      g_ninit = (raw || n < 4) ? 0u : ~((kLog || MODE == kTrailer) ? 0u : aux);
      g_st = aux;
      g_end = g_u1 & ~15ull;
      // steps on the group's 16G-byte line grid: lines from the one holding
      // the first byte to the one holding byte E-1 (load_step, kLines)
      g_le = (g_end + (kLine - 1)) & ~(kLine - 1);
      uint64_t S = (g_le - (a & ~(kLine - 1)) + kStep - 1) / kStep;
      if (S == 0) S = 1;
      uint32_t m = ok ? (uint32_t)S : 0u;
      m = wave_max(m);
      r_S = m;
      if (r_S != 0) break;  // an empty round (past the batch's end): next one
    }
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
    if (first) {
      asm volatile("" ::"v"(req), "v"(t_olo), "v"(t_ohi), "v"(t_len), "v"(t_aux));
      if (stage == 3) pipe(3);
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
        asm volatile("" ::"v"(h0), "v"(h1), "v"(h2), "v"(h3), "v"(h4), "v"(h5), "v"(h6));
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
    const bool live = !(fl & fDone);
    const bool run = r_S != 0;             // a round is active (else: stalled, empty step)
    const bool v = g_valid && run;
    const bool last = run && r_step + 1 == r_S;  // wave-uniform
    {
      const bool vz = g_nz && run;
      const uint32_t w = 4 * r_step;
      const uint64_t pa = g_lp + 16 * q;
      X.d0 = gload16<VAR>((vz && w >= g_w0) ? pa : zl);
      X.d1 = gload16<VAR>((vz && w + 1 >= g_w0) ? pa + 16 * G : zl);
      X.d2 = gload16<VAR>((vz && w + 2 >= g_w0) ? pa + 32 * G : zl);
      X.d3 = gload16<VAR>((vz && w + 3 >= g_w0 && (!last || g_l3)) ? pa + 48 * G : zl);
      const bool vl = v && last;
      if constexpr ((VAR & kVarNoTail) != 0) {  // timing ablation (diagnostics)
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
    X.rec = g_rec;
    // An invalid group's step (or a stalled one) reads zeros; with no init
    // xor-ed in it leaves the group's zero registers zero for its next block.
    X.ninit = v ? g_ninit : 0u;
    X.st = g_st;
    X.valid = v;
    X.last = last;
    if (run) {
      g_lp += kStep;
      if (++r_step == r_S) fl |= fRoundDone;
    }
    return live;
  };

  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  bool wb_on = false, wb_sec = false;
  uint64_t wb_a = 0;
  uint32_t wb_v = 0;
  uint4 wb_w = make_uint4(0, 0, 0, 0);  // trailer writer: the patched sector piece
  auto fold = [&](FlatSet& Y) {
    uint4 d0 = Y.d0, d1 = Y.d1, d2 = Y.d2, d3 = Y.d3;
    if (__builtin_amdgcn_ballot_w64(Y.head)) {  // wave-uniform: some group's head step
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
        const int32_t i4 = Y.ninit ? 4 : 0;
        auto mask = [&](uint4& d, int32_t hk) {
          const uint4 B = lds_u128(kLM + 16u * (uint32_t)clamp16(hk));
          const uint4 I = lds_u128(kLM + 16u * (uint32_t)clamp16(hk + i4));
          d.x = (d.x ^ I.x) & ~B.x;
          d.y = (d.y ^ I.y) & ~B.y;
          d.z = (d.z ^ I.z) & ~B.z;
          d.w = (d.w ^ I.w) & ~B.w;
        };
        mask(d0, h);
        mask(d1, h - 16 * G);
        mask(d2, h - 32 * G);
        mask(d3, h - 48 * G);
      }
    }
    if (Y.last) {  // wave-uniform: the region's last line may end past E
      swath4<VAR>(lds, c0, c1, c2, c3, d0, lo0, lo1, lo2, lo3);
      swath4<VAR>(lds, c0, c1, c2, c3, d1, lo0, lo1, lo2, lo3);
      swath4<VAR>(lds, c0, c1, c2, c3, d2, lo0, lo1, lo2, lo3);
      const uint32_t k0 = c0, k1 = c1, k2 = c2, k3 = c3;
      swath4<VAR>(lds, c0, c1, c2, c3, d3, lo0, lo1, lo2, lo3);
      if (!Y.l3) {  // piece at or after E: not in the region
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
    // the tail line(s) are used only on a block's last step: consume anyway, so
    // the compiler resolves their loads here with an exact count
    asm volatile("" ::"v"(Y.t.x), "v"(Y.t.y), "v"(Y.t.z), "v"(Y.t.w));
    if constexpr (kTail2) asm volatile("" ::"v"(Y.t2.x), "v"(Y.t2.y), "v"(Y.t2.z), "v"(Y.t2.w));
    if (Y.last) {  // wave-uniform: every group ends its block on this step
      // On the line grid lane q's pieces sit at position (q - e) mod G of the
      // 16G-byte swaths that end at E (e = (E mod 16G) / 16); group_fold wants
      // position p in lane p, which reads lane (p + e) mod G.
      const uint32_t e = (uint32_t)(Y.u1 >> 4) & (uint32_t)(G - 1);
      const int src = (grp * G) + (int)(((uint32_t)q + e) & (uint32_t)(G - 1));
      c0 = __shfl(c0, src);
      c1 = __shfl(c1, src);
      c2 = __shfl(c2, src);
      c3 = __shfl(c3, src);
      const uint32_t v = group_fold<G>(lds, c0, c1, c2, c3, q);
      c0 = c1 = c2 = c3 = 0;
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
#ifdef NOVA_DIAG
      if (p.wvar == 3) {  // timing ablation: no per-block epilogue, no result (WRONG)
        wb_a = 0;
        wb_v = v;
      } else
#endif
      finish_block<MODE>(lds, kByteTab, p, raw, v, Y, wb_a, wb_v);
      wb_on = q == 0 && Y.valid;  // written after the next step's loads are issued
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
      if ((MODE == kTrailer || MODE == kLogWrite) && wb_sec) {
        u32x4 w;
        w.x = wb_w.x;
        w.y = wb_w.y;
        w.z = wb_w.z;
        w.w = wb_w.w;
#ifdef NOVA_DIAG
        if (p.wvar == 1)
          __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)wb_a);
        else if (p.wvar != 2)
#endif
          *(__attribute__((address_space(1))) u32x4*)wb_a = w;
      } else {
#ifdef NOVA_DIAG
        if (p.wvar < 2)
#endif
          write_result<MODE>(p, wb_a, wb_v);
      }
      wb_on = false;
    }
  };

  // ---- prologue: the first chunk is implicit, the second is claimed; both are
  // loaded synchronously (stages back to back) ----------------------------------
  {
    uint64_t k0 = (uint64_t)wave * nwg + blockIdx.x;
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
  A.valid = A.last = A.head = A.l3 = A.wsec = false;
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
#ifdef NOVA_DIAG
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
#endif
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

template <int V, int MODE>
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
#ifdef NOVA_DIAG
  // per-wave phase stamps (s_memrealtime, 100 MHz): entry, descriptors used,
  // tables + first data landed, first block folded, first result written
  uint64_t st[5] = {0, 0, 0, 0, 0};
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p.stamps) st[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const bool live0 = bw < n_all;
  if (live0) start_blocks();
#ifdef NOVA_DIAG
  if (p.stamps) {
    asm volatile("" ::"v"((uint32_t)Kw));
    st[1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  // tables by LDS-DMA while the first block's loads are in flight
  glds_copy(0, p.tab_main, Cfg::kTree);
  glds_copy(Cfg::kTree, p.tab_tree, Cfg::kLevels * kTreeBytes);
  glds_copy(burst_byte_tab<V>(), p.tab_byte, 1024);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
#ifdef NOVA_DIAG
  if (p.stamps) st[2] = __builtin_amdgcn_s_memrealtime();
#endif
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
#ifdef NOVA_DIAG
    if (p.stamps && !st[3]) {
      asm volatile("" ::"v"(v));
      st[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    finish_block<MODE, Cfg::kTree>(lds, burst_byte_tab<V>(), p, raw, v, Y, wb_a, wb_v);
    if (q == 0 && Y.valid) write_result<MODE>(p, wb_a, wb_v);
#ifdef NOVA_DIAG
    if (p.stamps && !st[4]) {
      __builtin_amdgcn_s_waitcnt(0);
      st[4] = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) {
        for (int k = 0; k < 5; k++) p.stamps[8 * wid + k] = st[k];
        p.stamps[8 * wid + 5] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // XCC id
        p.stamps[8 * wid + 6] = Kw;
      }
    }
#endif
    bw += step_blocks;
    if (bw >= n_all) break;
    start_blocks();
  }
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

// Trailer writer, second pass: crc[i] = Mask(Extend(Value(block i), type))
// from the first pass (the rounds kernel in store mode); write the 5-byte
// trailer [type][LE32] at base + offsets[i] + sizes[i], with '!' over its last
// byte for TableBuilder's ordering (table/table_builder.cc:202-206,
// ltc/stoc_file_client_impl.cpp:713-719).  Inside the streaming kernel the
// trailer stores per block cost ~12 points of HBM throughput.
#ifdef NOVA_DIAG
// Store-form experiments for the trailer writer and log CRC fields (DESIGN.md
// 3.5b): measured, not faster than the CRC kernel's own byte stores.

// Trailer writer pre-pass.  HBM writes whole 64-B pieces; a store that
// covers only part of one (a 5-B trailer) costs a read-modify-write at the
// memory, so the rounds kernel rewrites the whole aligned
// 64-B piece(s) holding a trailer -- its "window", one piece or two when the
// trailer crosses a piece boundary -- patched with the trailer bytes.  The
// window's other bytes are stored back unchanged, which is safe when no other
// block's trailer lies in it: then nobody else writes those bytes (block data
// is only read) and no two windows share a piece (every window piece holds a
// byte of its own trailer).
//   *flag |= 1 unless the blocks are ascending and disjoint, trailer
//   included (offset[i+1] >= offset[i] + size[i] + 5): then only the
//   neighbours' trailers can reach a window, and
//   elig[i] = 1 iff block i's window holds neither neighbour's trailer, lies
//   above the first block's start (i == 0) and is not the last block's (its
//   window may run past the image).  Window bytes outside every block (gaps)
//   lie between two blocks of the image, so inside the caller's allocation.
//   Windows are aligned in absolute addresses (ba = the image base), as the
//   kernels that store them see them.
__global__ void __launch_bounds__(256) trailer_layout_kernel(uint64_t ba, const uint64_t* offsets,
                                                             uint64_t omask, const uint32_t* lengths,
                                                             uint64_t lmask, uint64_t stride,
                                                             uint32_t len, uint64_t n, uint32_t* elig,
                                                             uint32_t* flag) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  bool bad = false;
  auto u0_of = [&](uint64_t i) { return ba + offsets[i & omask] + i * stride; };
  auto u1_of = [&](uint64_t i) { return u0_of(i) + lengths[i & lmask] + len; };
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nth) {
    const uint64_t u0 = u0_of(i), u1 = u1_of(i);
    const uint64_t ws = u1 & ~63ull, we = ((u1 + 4) & ~63ull) + 64;
    bool e = i + 1 < n;
    if (i + 1 < n) {
      bad = bad || u0_of(i + 1) < u1 + 5;
      e = e && u1_of(i + 1) >= we;
    }
    e = e && (i == 0 ? ws >= u0 : u1_of(i - 1) + 5 <= ws);
    elig[i] = e ? 1u : 0u;
  }
  if (__builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// Log write pre-pass (same reasoning as trailer_layout_kernel): the rounds
// kernel rewrites the whole 64-B piece holding a record's 4-byte CRC field
// [o, o+4) (db/log_writer.cc:113) instead of storing 4 bytes into it.
//   *flag |= 1 unless the record offsets are non-decreasing (then only the
//   neighbours' CRC fields can reach a piece);
//   elig[i] = 1 iff the field lies in one piece, the piece lies inside the
//   image (buf_len) and holds neither neighbour's CRC field.  Every other byte
//   of the piece (payloads, length and type bytes, block padding) is only read
//   and is stored back unchanged.
__global__ void __launch_bounds__(256) log_window_kernel(const uint64_t* offs, uint64_t n,
                                                         uint64_t buf_len, uint32_t* elig,
                                                         uint32_t* flag) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nth) {
    const uint64_t o = offs[i], ws = o & ~63ull;
    bool e = (o & 63) <= 60 && ws + 64 <= buf_len;
    if (i + 1 < n) {
      const uint64_t on = offs[i + 1];
      bad = bad || on < o;
      e = e && on >= ws + 64;
    }
    if (i > 0) e = e && offs[i - 1] + 4 <= ws;
    elig[i] = e ? 1u : 0u;
  }
  if (__builtin_amdgcn_ballot_w64(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// Two-pass trailer writer with whole-piece stores, second pass: the CRC pass
// left crc[i] = Mask(crc) (type appended); block i's trailer [u1, u1+5) is
// patched into the aligned 64-B piece(s) holding it, which are read and
// stored whole when trailer_layout_kernel found them private to the block
// (*flag == 0, elig[i]); other blocks store their five bytes.  Eight lanes per
// block: lane k owns the piece line s0 + 16k (k < 4, or < 8 when the trailer
// crosses a piece).  The stores run after every read of the image, in their
// own launch.
__global__ void __launch_bounds__(256) trailer_rmw_kernel(uint8_t* base, const uint64_t* offsets,
                                                          uint64_t omask, const uint32_t* lengths,
                                                          uint64_t lmask, uint64_t stride, uint32_t len,
                                                          const uint32_t* crc, const uint32_t* elig,
                                                          const uint32_t* flag, uint64_t n,
                                                          uint32_t flags) {
  const uint64_t nth = ((uint64_t)gridDim.x * blockDim.x) >> 3;
  const uint32_t k = threadIdx.x & 7u;
  const bool layout_ok = *flag == 0;
  const bool quirk = (flags & NOVA_TRAILER_TB_QUIRK) != 0;
  const uint32_t type = (flags >> 8) & 0xffu;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; i < n; i += nth) {
    uint8_t* t = base + offsets[i & omask] + i * stride + lengths[i & lmask] + len;
    const uint32_t m = crc[i];
    if (layout_ok && elig[i]) {
      const uint64_t u1 = (uint64_t)t, s0 = u1 & ~63ull;
      const uint32_t np = ((u1 + 4) & ~63ull) != s0 ? 8u : 4u;
      if (k < np) {
        const uint32_t mq = quirk ? ((m & 0x00ffffffu) | ((uint32_t)'!' << 24)) : m;
        const uint64_t tv = (uint64_t)type | ((uint64_t)mq << 8);
        const uint64_t a = s0 + 16u * k;
        auto* pa = (__attribute__((address_space(1))) u32x4*)a;
        u32x4 w = *pa;
        const uint4 d = patch_trailer(make_uint4(w.x, w.y, w.z, w.w), a, u1, tv);
        w.x = d.x;
        w.y = d.y;
        w.z = d.z;
        w.w = d.w;
        *pa = w;
      }
    } else if (k == 0) {
      store_trailer(t, type, m, quirk);
    }
  }
}

__global__ void __launch_bounds__(256) trailer_scatter_kernel(uint8_t* base, const uint64_t* offsets,
                                                              const uint32_t* sizes,
                                                              const uint32_t* crc, uint64_t n,
                                                              uint32_t flags) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nth) {
    store_trailer(base + offsets[i] + sizes[i], (flags >> 8) & 0xffu, crc[i],
                  (flags & NOVA_TRAILER_TB_QUIRK) != 0);
  }
}
#endif  // NOVA_DIAG

#ifdef NOVA_DIAG
// ---- crc32c_logstream_kernel<MODE>: a whole log image, record CRCs ----------
// MANIFEST / write-ahead-log record CRCs for a log image
// whose record offsets are in file order.  Each lane group of 8 lanes streams
// one 32 KiB log block (db/log_format.h:27, kBlockSize) with the stream
// kernel's uniform schedule -- 4-swath steps of one 128-B line per swath,
// identical for every group of the wave, no per-record regions and no round
// padding -- and resolves the block's records on the fly:
//
//   * A record's CRC input is [a, b) = [header+6, header+7+length) (type byte +
//     payload, db/log_writer.cc:99-114).  The group's four stream registers per
//     lane hold the CURRENT record only.  A swath holding a, a byte of the init
//     window [a, a+4), or b takes the slow path: each lane masks its 16-B piece
//     to [a, b) with two 16-B prefix masks from LDS and xors ~0 into [a, a+4)
//     (Extend's init, as the units kernel); a record that starts in the swath
//     starts from zero.  Between records (headers, block trailers, records
//     left to the follow-up) the registers run on unmasked data: the next
//     record's first swath resets them.
//   * Only records of >= kLsMinN CRC bytes are streamed, so a group meets at
//     most one record end and one record start per 128-B swath and the slow
//     path is straight-line code (no loop, no global memory access -- either
//     would make the compiler drain the step's prefetch).  Shorter records,
//     records the reader would not read (bounds / zero records: status only)
//     and whole blocks of more than 64 records go to a leftover list that the
//     gated rounds kernel processes right after (crc32c_rounds_kernel, gate).
//   * At b the group spills its 32 stream words to a per-wave LDS slot
//     ("snapshot").  Streams whose word of the last swath lies entirely at or
//     after b keep their value from the swath before (the rounds kernel's
//     rotation), so the snapshot is a virtual 128-B message ending at the
//     4-byte word holding b-1: pad = 0..3 bytes.
//   * Snapshots are folded after the swath once a wave holds kLsFlush of them
//     (the fold phase): four lanes per record run one Horner chain each (M16
//     over every 4th word), a 3-step merge (M4) gives the pending word V,
//     register = M4(V), and `pad` inverse zero-byte steps (bitwise) give the
//     register at b.  Write: Mask(crc) into the header; verify: compare with
//     the stored CRC (one status byte per record, mismatches counted).
//   * Descriptors: a 64-record window per group (8 per lane), decoded at the
//     start of each block from the offsets and the 7-byte record headers.
//   * Preconditions (else the follow-up reruns the whole batch): offsets
//     ascending (pre-pass, flag bit 0) and no streamed record starting before
//     the previous one ended (flag bit 1).
// Fast swaths cost what the stream kernel's do; the per-record work runs
// wave-wide on the swaths that hold a record boundary.
constexpr int kLsG = 8;                      // lanes per group (one 128-B line per swath)
constexpr int kLsWaves = 8;                  // waves per workgroup
constexpr uint32_t kLsSlots = 16;            // snapshot slots per wave
constexpr uint32_t kLsFlush = kLsSlots - 8;  // fold after a swath leaving this many (<= 8 per swath)
constexpr uint32_t kLsSlotBytes = 144;       // 32 stream words + 16 B of meta (bank spread)
constexpr uint32_t kLsM4 = kMainBytes;       // LDS: M4 byte tables (4 KiB)
constexpr uint32_t kLsM16 = kMainBytes + 4096;
constexpr uint32_t kLsLM = kMainBytes + 8192;  // 17 x 16-B prefix masks: LM[n] = bytes [0, n)
constexpr uint32_t kLsTabBytes = 8192 + 17 * 16;
constexpr uint32_t kLsSlot0 = kMainBytes + kLsTabBytes;
constexpr uint32_t kLsLds = kLsSlot0 + kLsWaves * kLsSlots * kLsSlotBytes;
static_assert(kLsLds <= 160 * 1024, "log-stream LDS exceeds the CU");
static_assert(kLsSlot0 % 16 == 0, "slots are 16-B aligned");
constexpr int kLsWin = 8;                    // decoded descriptors per lane (64 per group)
constexpr uint32_t kLsMinN = 128;            // CRC bytes of a streamed record (>= one swath)
constexpr int32_t kLsFar = 1 << 28;          // "no record": past every swath


typedef __attribute__((address_space(1))) const u32_unaligned gcu32u;

// Pre-pass: first[k] = first record of log block k (record i belongs to block
// min(off_i / 32 KiB, nb - 1): a record past the image lands in the last block,
// whose status logic rejects it), first[nb] = n.  Unsorted offsets set bit 0
// of *flag (the log-stream kernel then leaves the batch to the follow-up).
__global__ void __launch_bounds__(256) log_first_kernel(const uint64_t* __restrict__ offs, uint64_t n,
                                                        uint64_t nb, uint32_t* __restrict__ first,
                                                        uint32_t* flag) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += nth) {
    const uint64_t o = i < n ? offs[i] : 0;
    const uint64_t k = i < n ? ((o >> 15) < nb - 1 ? (o >> 15) : nb - 1) : nb;
    uint64_t k_lo = 0;
    if (i > 0) {
      const uint64_t op = offs[i - 1];
      if (i < n && o < op) atomicOr(flag, 1u);
      k_lo = ((op >> 15) < nb - 1 ? (op >> 15) : nb - 1) + 1;
    }
    for (uint64_t kk = k_lo; kk <= k; kk++) first[kk] = (uint32_t)i;
  }
}

template <int MODE, int VAR = 0>
__global__ void __launch_bounds__(kLsWaves * 64) crc32c_logstream_kernel(CrcParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  static_assert(MODE == kLogWrite || MODE == kLogVerify, "log modes only");
  constexpr bool kVerifyMode = MODE == kLogVerify;
  if (*(volatile const uint32_t*)p.ls_flag & 1u) return;  // unsorted: the follow-up takes it
  lds_fill_tables(lds, p.tab_main, p.tab_tree, kLsTabBytes / 16, nullptr, 0);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane & 7;
  const int grp = lane >> 3;
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const uint64_t base = (uint64_t)p.base;
  const uint64_t nb = p.n_lblocks;
  const uint64_t R = (nb + 7) / 8;                     // rounds: 8 log blocks (one per group)
  const int32_t off0 = (int32_t)(base & 127u);         // every block starts off0 into its line
  const uint32_t KG = ((uint32_t)off0 + kLogBlock + 511u) / 512u;  // 4-line steps per block
  const uint64_t zl = (uint64_t)p.zline;
  const uint64_t lo_ok = base & ~15ull, hi_ok = (base + p.buf_len + 15) & ~15ull;
  const uint32_t slots = kLsSlot0 + (uint32_t)wave * kLsSlots * kLsSlotBytes;
  const uint32_t nwaves = blockDim.x >> 6;
  const uint32_t nwg = gridDim.x;
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  // ---- round claims (per-workgroup counters, bounded stealing)
  uint32_t victim = blockIdx.x, tried = 0, req = 0;
  auto claim = [&](uint32_t v) {
    uint32_t r = 0;
    if (lane == 0)
      r = __hip_atomic_fetch_add(p.sched + v * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    req = r;
  };
  auto round_of = [&](uint32_t v, uint32_t idx) -> uint64_t {
    const uint64_t r = ((uint64_t)idx + nwaves) * nwg + v;
    return r < R ? r : ~0ull;
  };
  auto collect = [&]() -> uint64_t {
    uint64_t r = round_of(victim, __builtin_amdgcn_readfirstlane(req));
    while (r == ~0ull && ++tried < p.steal_limit + 1) {
      victim = (victim + 1) % nwg;
      claim(victim);
      r = round_of(victim, __builtin_amdgcn_readfirstlane(req));
    }
    return r;
  };

  // ---- per-group block state (group-uniform values, in every lane of it)
  uint64_t k = 0;                      // log block of the group
  uint32_t r_lo = 0, nrec = 0;         // its records [r_lo, r_lo + nrec)
  uint32_t nwin = 0;                   // records in the window (0: dense block, all leftover)
  uint32_t j = 0;                      // current window position
  int32_t a_c = kLsFar, b_c = kLsFar;  // current record's CRC range, region-relative
  uint32_t n_c = 0, ax_c = 0;          // its CRC length, aux (stored CRC)
  int32_t prev_b = 0;                  // end of the previous streamed record (overlap check)
  uint32_t wd[kLsWin], wa[kLsWin];     // window: desc = b_rel | n << 16 (n = 0: not streamed), aux
  uint32_t np = 0;                     // pending snapshots of the wave (wave-uniform)
  uint32_t ovl = 0;                    // this lane saw overlapping records
  uint32_t nbad = 0;                   // this lane's mismatches (verify)
  uint32_t* const left = p.ls_left;    // leftover record list, count at ls_flag[2]

  // Decode the block's records (synchronous; once per block): offsets, then
  // the 7-byte headers (a header past its block or the image is not read).
  // Records not streamed here are appended to the leftover list.
  auto decode_block = [&](uint64_t bk) {
    const bool dense = nrec > 8u * kLsWin;
    nwin = dense ? 0u : nrec;
    uint64_t o[kLsWin];
#pragma unroll
    for (int m = 0; m < kLsWin; m++) {
      const uint32_t jj = 8u * m + (uint32_t)q;
      o[m] = jj < nwin ? p.offsets[r_lo + jj] : 0;
    }
    uint32_t nl = 0;  // this lane's leftovers
#pragma unroll
    for (int m = 0; m < kLsWin; m++) {
      const uint32_t jj = 8u * m + (uint32_t)q;
      const bool valid = jj < nwin;
      const bool fits = valid && log_header_fits(o[m], p.buf_len);
      const uint64_t h = fits ? base + o[m] : zl;
      const uint32_t w0 = kVerifyMode ? *(gcu32u*)h : 0u;  // stored masked CRC
      const uint32_t w1 = *(gcu32u*)(fits ? h + 4 : zl);    // length, type
      const uint32_t length = w1 & 0xffffu;
      const uint32_t st = fits ? log_status(o[m], length, kVerifyMode ? ((w1 >> 16) & 0xffu) : 1u,
                                            p.buf_len)
                               : (valid ? log_nohdr_status(o[m], p.buf_len) : NOVA_LOG_TRUNCATED);
      const bool elig = st == NOVA_LOG_OK && 1u + length >= kLsMinN;
      const uint64_t hrel = o[m] - bk * kLogBlock;
      wd[m] = elig ? ((uint32_t)hrel + 7u + length) | ((1u + length) << 16) : 0u;
      wa[m] = kVerifyMode ? w0 : 0u;
      nl += (valid && !elig) ? 1u : 0u;
    }
    // leftover list: the whole block if dense, else the records not streamed
    uint32_t cnt = dense ? (nrec > (uint32_t)q ? (nrec - 1u - (uint32_t)q) / 8u + 1u : 0u) : nl;
    uint32_t incl = cnt;  // inclusive prefix over the group's 8 lanes
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      const uint32_t y = __shfl_up(incl, (unsigned)d, 8);
      if (q >= d) incl += y;
    }
    const uint32_t total = __shfl(incl, (grp << 3) | 7);
    uint32_t at = 0;
    if (q == 0 && total) at = atomicAdd(p.ls_flag + 2, total);
    at = __shfl(at, grp << 3);
    if (dense) {
      for (uint32_t i = (uint32_t)q; i < nrec; i += 8) left[at + i] = r_lo + i;
    } else {
      uint32_t pos = at + incl - cnt;
#pragma unroll
      for (int m = 0; m < kLsWin; m++) {
        const uint32_t jj = 8u * m + (uint32_t)q;
        if (jj < nwin && (wd[m] >> 16) == 0) left[pos++] = r_lo + jj;
      }
    }
  };
  // Current record := the first streamed record at window position >= j.
  auto fetch = [&]() {
    for (;;) {
      if (j >= nwin) {
        a_c = b_c = kLsFar;
        n_c = 0;
        return;
      }
      const uint32_t m = j >> 3;
      uint32_t dsel = wd[0], asel = wa[0];
#pragma unroll
      for (int mm = 1; mm < kLsWin; mm++) {
        if (m == (uint32_t)mm) {
          dsel = wd[mm];
          asel = wa[mm];
        }
      }
      const int src = (grp << 3) | (int)(j & 7u);
      const uint32_t d = __shfl(dsel, src);
      if ((d >> 16) != 0) {
        n_c = d >> 16;
        b_c = off0 + (int32_t)(d & 0xffffu);
        a_c = b_c - (int32_t)n_c;
        ax_c = kVerifyMode ? __shfl(asel, src) : 0u;
        if (a_c - 6 < prev_b) ovl = 1;  // starts inside the previous streamed record
        prev_b = b_c;
        return;
      }
      j++;
    }
  };

  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;

  // ---- fold phase: four lanes per pending snapshot ----------------------------
  // A wave's LDS operations execute in order, so other lanes' snapshot stores
  // are visible to the reads below once the compiler keeps the order (memory
  // clobber); a wavefront-scope fence would also drain the step's data loads.
  auto lds_order = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  auto fold_phase = [&]() {
    lds_order();
    const uint32_t rec = (uint32_t)lane >> 2, sub = (uint32_t)lane & 3u;
    const bool act = rec < np;
    const uint32_t sa = slots + (act ? rec : 0u) * kLsSlotBytes;
    const uint4 meta = lds_u128(sa + 128);
    const uint32_t info = meta.w;
    const uint32_t kb = (info >> 16) & 31u, pad = (info >> 21) & 3u;
    // chain `sub`: words kb+1+jj (mod 32) of the rotated message, jj = sub, sub+4, ...
    uint32_t v = 0;
#pragma unroll
    for (uint32_t jj = 0; jj < 32; jj += 4)
      v = lds_apply(kLsM16, v) ^ lds_u32(nullptr, sa + (((kb + 1u + jj + sub) & 31u) << 2));
    const int b4 = lane & ~3;
    const uint32_t u0 = __shfl(v, b4), u1 = __shfl(v, b4 + 1), u2 = __shfl(v, b4 + 2);
    const uint32_t u3 = __shfl(v, b4 + 3);
    const uint32_t V = lds_apply(kLsM4, lds_apply(kLsM4, lds_apply(kLsM4, u0) ^ u1) ^ u2) ^ u3;
    uint32_t reg = lds_apply(kLsM4, V);
    if (pad >= 1) reg = unstep_byte(reg);
    if (pad >= 2) reg = unstep_byte(reg);
    if (pad >= 3) reg = unstep_byte(reg);
    const uint32_t crc = ~reg;
    if (act && sub == 0) {
      if constexpr (MODE == kLogWrite) {
        const uint64_t h = base + (uint64_t)meta.z * kLogBlock + (info & 0xffffu);
        store_u32_unaligned((uint8_t*)h, mask_crc(crc));
      } else {
        const bool ok = unmask_crc(meta.y) == crc;
        *(__attribute__((address_space(1))) uint8_t*)(p.ok_out + meta.x) =
            (uint8_t)(ok ? NOVA_LOG_OK : NOVA_LOG_CHECKSUM_MISMATCH);
        nbad += ok ? 0u : 1u;
      }
    }
    np = 0;
    lds_order();
  };

  // ---- one swath: line L0 (region-relative byte) of the group's block --------
  auto swath = [&](const uint4 d, int32_t L0) {
    const bool st = (a_c + 4 > L0) && (a_c < L0 + 128);
    const bool en = b_c <= L0 + 128;
    if ((VAR & kVarLsFast) != 0 || __builtin_amdgcn_ballot_w64(st || en) == 0) {
      swath4(lds, c0, c1, c2, c3, d, lo0, lo1, lo2, lo3);
      return;
    }
    // slow path: a record of some group starts or ends in this swath
    const int32_t P = L0 + 16 * q;
    const uint32_t o0 = c0, o1 = c1, o2 = c2, o3 = c3;
    uint32_t t0 = c0, t1 = c1, t2 = c2, t3 = c3;
    swath4(lds, t0, t1, t2, t3, zero4, lo0, lo1, lo2, lo3);  // T(c): the record goes on
    const bool cont = a_c < L0;  // the current record began in an earlier swath
    const uint32_t km = cont ? ~0u : 0u;
    uint32_t r0, r1, r2, r3;
    {  // r = (cont ? T(c) : 0) ^ (((d & LM[hi]) ^ LM[lo4]) & ~LM[lo])
      const int32_t lo = clamp16(a_c - P), hi = clamp16(b_c - P), lo4 = clamp16(a_c + 4 - P);
      const uint4 A = lds_u128(kLsLM + 16u * (uint32_t)hi);
      const uint4 B = lds_u128(kLsLM + 16u * (uint32_t)lo);
      const uint4 Cm = lds_u128(kLsLM + 16u * (uint32_t)lo4);
      r0 = (t0 & km) ^ (((d.x & A.x) ^ Cm.x) & ~B.x);
      r1 = (t1 & km) ^ (((d.y & A.y) ^ Cm.y) & ~B.y);
      r2 = (t2 & km) ^ (((d.z & A.z) ^ Cm.z) & ~B.z);
      r3 = (t3 & km) ^ (((d.w & A.w) ^ Cm.w) & ~B.w);
    }
    const uint64_t eb = __builtin_amdgcn_ballot_w64(en);
    if (eb == 0) {  // starts only
      c0 = r0;
      c1 = r1;
      c2 = r2;
      c3 = r3;
      return;
    }
    const uint64_t leaders = eb & 0x0101010101010101ull;
    if (en) {  // snapshot the ending record, then take the group's next one
      const int32_t kb = (b_c - 1 - L0) >> 2;  // stream holding byte b-1 (b > L0: n >= 128)
      const uint32_t pad = (uint32_t)(4 * (kb + 1) - (b_c - L0));
      const int k0 = 4 * q;
      uint4 sn;
      sn.x = (k0 + 0 > kb) ? (o0 & km) : r0;
      sn.y = (k0 + 1 > kb) ? (o1 & km) : r1;
      sn.z = (k0 + 2 > kb) ? (o2 & km) : r2;
      sn.w = (k0 + 3 > kb) ? (o3 & km) : r3;
      const uint64_t below = leaders & ((1ull << (grp * 8)) - 1ull);
      const uint32_t sa = slots + (np + (uint32_t)__popcll(below)) * kLsSlotBytes;
      lds_st128(sa + 16u * (uint32_t)q, sn);
      if (q == 0) {
        const uint32_t hrel = (uint32_t)(a_c - off0) - 6u;  // the record's header
        lds_st128(sa + 128, make_uint4(r_lo + j, ax_c, (uint32_t)k,
                                       hrel | ((uint32_t)kb << 16) | (pad << 21)));
      }
      j++;
      fetch();
    }
    np += (uint32_t)__popcll(leaders);
    // the ending groups' next record starts from zero (it may start in this swath;
    // it cannot also end in it)
    const int32_t lo = clamp16(a_c - P), hi = clamp16(b_c - P), lo4 = clamp16(a_c + 4 - P);
    const uint4 A = lds_u128(kLsLM + 16u * (uint32_t)hi);
    const uint4 B = lds_u128(kLsLM + 16u * (uint32_t)lo);
    const uint4 Cm = lds_u128(kLsLM + 16u * (uint32_t)lo4);
    c0 = en ? (((d.x & A.x) ^ Cm.x) & ~B.x) : r0;
    c1 = en ? (((d.y & A.y) ^ Cm.y) & ~B.y) : r1;
    c2 = en ? (((d.z & A.z) ^ Cm.z) & ~B.z) : r2;
    c3 = en ? (((d.w & A.w) ^ Cm.w) & ~B.w) : r3;
  };

  // ---- rounds ---------------------------------------------------------------
  uint64_t r = (uint64_t)wave * nwg + blockIdx.x;  // implicit first round
  if (r >= R) {
    claim(victim);
    r = collect();
  }
  while (r != ~0ull) {
    claim(victim);  // the next round (collected after this one)
    k = r * 8 + (uint64_t)grp;
    const bool act = k < nb;
    r_lo = act ? p.first[k] : 0u;
    nrec = act ? p.first[k + 1] - r_lo : 0u;
    const uint64_t bstart = k * kLogBlock;
    const uint32_t blen =
        act ? (uint32_t)(p.buf_len - bstart < kLogBlock ? p.buf_len - bstart : kLogBlock) : 0u;
    const uint64_t RS = base + bstart - (uint64_t)off0;  // region start: 128-B aligned
    const uint32_t lines = act ? ((uint32_t)off0 + blen + 127u) / 128u : 0u;
    decode_block(k);
    j = 0;
    prev_b = 0;
    fetch();
    c0 = c1 = c2 = c3 = 0;
    auto piece = [&](uint32_t line) -> uint64_t {
      const uint64_t a = RS + 128ull * line + 16u * (uint32_t)q;
      return (line < lines && a >= lo_ok && a < hi_ok) ? a : zl;
    };
    uint4 b0 = gload16(piece(0)), b1 = gload16(piece(1));
    uint4 b2 = gload16(piece(2)), b3 = gload16(piece(3));
    for (uint32_t s = 0; s < KG; s++) {
      const uint4 x0 = b0, x1 = b1, x2 = b2, x3 = b3;
      const uint32_t ln = 4 * s + 4;
      b0 = gload16(piece(ln));
      b1 = gload16(piece(ln + 1));
      b2 = gload16(piece(ln + 2));
      b3 = gload16(piece(ln + 3));
      const int32_t L = (int32_t)(512 * s);
      swath(x0, L);
      if (np >= kLsFlush) fold_phase();
      swath(x1, L + 128);
      if (np >= kLsFlush) fold_phase();
      swath(x2, L + 256);
      if (np >= kLsFlush) fold_phase();
      swath(x3, L + 384);
      if (np >= kLsFlush) fold_phase();
    }
    r = collect();
  }
  if (np) fold_phase();
  if constexpr ((VAR & kVarLsFast) != 0)  // keep the ablation's stream live
    if ((c0 ^ c1 ^ c2 ^ c3) == 0x9e3779b9u) atomicOr(p.ls_flag, 4u);
  if (__builtin_amdgcn_ballot_w64(ovl != 0) && lane == 0) atomicOr(p.ls_flag, 2u);
  if constexpr (kVerifyMode) {
    if (__builtin_amdgcn_ballot_w64(nbad != 0)) {
      uint32_t v = nbad;
      for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) atomicAdd(p.ls_bad, v);
    }
  }
  sched_release(p.sched);
}

#endif  // NOVA_DIAG

// ---- few large blocks: split and combine --------------------
// Every kernel above gives a block to one lane group or one wave, so a batch
// of a few large blocks (one 256 MiB buffer, 16 x 64 MiB) leaves the machine
// idle: one 256 MiB block ran at 3.7 GB/s.  The split path cuts block i (its
// n_i CRC input bytes: len_i, +1 type byte for verify) into pieces of S bytes
// (S a multiple of 16) counted from the block's END -- piece j >= 1 is
// [n_i - (K_i - j) S, n_i - (K_i - j - 1) S), piece 0 the head [0, n_i - (K_i - 1) S)
// -- with K_i = min(kmax, ceil(n_i / S)) and slots j >= K_i empty.  A batch of
// the pieces (the ordinary kernels, RAW) gives each piece's linear part raw_j;
//   raw(block)            = xor_j M_{(K_i - 1 - j) S}(raw_j)      (split_fold_kernel)
//   Extend(init, block)   = ~(M_{n_i}(~init) ^ raw(block))       (split_finish)
// (util/crc32c.cc:487-588 computes the same value in one pass), and the finish
// runs the mode's epilogue (store, trailer, verify) as the other kernels do.
__device__ __forceinline__ uint64_t split_block_off(const CrcParams& p, uint64_t i) {
  return p.offsets ? p.offsets[i] : i * p.stride;
}
__device__ __forceinline__ uint32_t split_block_len(const CrcParams& p, uint64_t i, uint32_t extra) {
  return (p.lengths ? p.lengths[i] : p.len) + extra;
}
__device__ __forceinline__ uint32_t split_pieces(uint32_t n, uint32_t S, uint32_t kmax) {
  const uint32_t k = n ? (uint32_t)(((uint64_t)n + S - 1) / S) : 1u;
  return k < kmax ? k : kmax;
}
// M_{16 m} through the binary powers M_{16 * 2^b} (sh16 tables).
__device__ __forceinline__ uint32_t shift16(const uint32_t* sh16, uint64_t m, uint32_t c) {
  while (m) {
    const int b = __builtin_ctzll(m);
    c = gapply(sh16 + b * 1024, c);
    m &= m - 1;
  }
  return c;
}

__global__ void __launch_bounds__(256) split_pieces_kernel(CrcParams p, uint32_t extra, uint32_t S,
                                                           uint32_t kshift, uint64_t* poff,
                                                           uint32_t* plen, uint32_t* acc) {
  const uint64_t slots = p.n_blocks << kshift;
  const uint32_t kmax = 1u << kshift;
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < slots; s += nth) {
    const uint64_t i = s >> kshift;
    const uint32_t j = (uint32_t)s & (kmax - 1);
    const uint64_t o = split_block_off(p, i);
    const uint32_t n = split_block_len(p, i, extra);
    const uint32_t k = split_pieces(n, S, kmax);
    uint64_t po = o;
    uint32_t pl = 0;
    if (j == 0) {
      pl = n - (k - 1) * S;
    } else if (j < k) {
      po = o + n - (uint64_t)(k - j) * S;
      pl = S;
    }
    poff[s] = po;
    plen[s] = pl;
    if (j == 0) acc[i] = 0;  // the block's xor word (split_fold_kernel, kmax > 64)
  }
}

// Extend's init and the mode epilogue for block i with raw(block) = x.
__device__ void split_finish(const CrcParams& p, int mode, uint32_t extra, uint64_t i, uint32_t x) {
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t type = (p.flags >> 8) & 0xffu;
  const uint32_t n = split_block_len(p, i, extra);
  uint32_t crc = x;
  if (!raw) {
    uint32_t l = ~(p.init ? p.init[i] : 0u);  // M_n(~init): n & 15 byte steps, then M_{16 (n >> 4)}
    for (uint32_t r = 0; r < (n & 15u); r++) l = byte_step(l, 0u);
    crc = ~(shift16(p.tab_sh16, n >> 4, l) ^ crc);
  }
  const uint8_t* d = p.base + split_block_off(p, i);
  if (mode == kVerify) {
    const uint32_t stored = (uint32_t)d[n] | ((uint32_t)d[n + 1] << 8) |
                            ((uint32_t)d[n + 2] << 16) | ((uint32_t)d[n + 3] << 24);
    const bool ok = unmask_crc(stored) == crc;  // table/table.cc:435-437
    p.ok_out[i] = ok ? 1 : 0;
    if (!ok && p.n_bad) atomicAdd(p.n_bad, 1u);
    return;
  }
  if (p.flags & NOVA_CRC32C_APPEND_TYPE) crc = ~byte_step(~crc, type);  // table/table_builder.cc:203
  if (mode == kTrailer) {
    store_trailer(const_cast<uint8_t*>(d) + n, type, mask_crc(crc), (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
  } else {
    if (p.flags & NOVA_CRC32C_MASK_OUTPUT) crc = mask_crc(crc);
    p.out[i] = crc;
  }
}

// One thread per piece slot; the grid covers the slots exactly (whole waves
// when kmax >= 64, whose 64 lanes then share one block).  The lanes of one
// block xor their shifted raws together; with kmax <= 64 one lane then holds
// the block's raw and finishes it, otherwise each wave xors its part into the
// block's word acc[i] (zeroed by split_pieces_kernel) and split_finish_kernel
// follows.  (A last-arriving wave finishing instead measured slower: 2048
// ordered atomics on one block's words for one 256 MiB block.)
__global__ void __launch_bounds__(256) split_fold_kernel(CrcParams p, int mode, uint32_t extra,
                                                         uint32_t S, uint32_t kshift,
                                                         const uint32_t* praw, uint32_t* acc) {
  const uint64_t slots = p.n_blocks << kshift;
  const uint32_t kmax = 1u << kshift;
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c = 0;
  uint64_t i = 0;
  uint32_t j = 0;
  if (s < slots) {
    i = s >> kshift;
    j = (uint32_t)s & (kmax - 1);
    const uint32_t k = split_pieces(split_block_len(p, i, extra), S, kmax);
    if (j < k) c = shift16(p.tab_sh16, (uint64_t)(k - 1 - j) * (S >> 4), praw[s]);
  }
  const uint32_t span = kmax < 64 ? kmax : 64u;
  for (uint32_t d = 1; d < span; d <<= 1) c ^= __shfl_xor(c, (int)d);
  if (s >= slots || (j & (span - 1)) != 0) return;
  if (kmax <= 64) {
    split_finish(p, mode, extra, i, c);
    return;
  }
  if (c) __hip_atomic_fetch_xor(acc + i, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) split_finish_kernel(CrcParams p, int mode, uint32_t extra,
                                                           const uint32_t* acc) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n_blocks; i += nth)
    split_finish(p, mode, extra, i, acc[i]);
}

// Synthetic data: splitmix64 counter stream (novalsm_amd/synth.py).
__global__ void fill_splitmix64_kernel(uint8_t* dst, uint64_t nbytes, uint64_t seed,
                                       uint64_t first_word) {
  const uint64_t nw = nbytes / 8;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = tid; k < nw; k += stride) {
    uint64_t z = seed + (first_word + k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    reinterpret_cast<uint64_t*>(dst)[k] = z;
  }
  if (tid == 0 && (nbytes & 7)) {
    uint64_t z = seed + (first_word + nw + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (uint64_t i = 0; i < (nbytes & 7); i++) dst[nw * 8 + i] = (uint8_t)(z >> (8 * i));
  }
}

#ifdef NOVA_DIAG
// Diagnostic: plain coalesced streaming read (grid-stride, 4 x 16 B per lane
// in flight), the chip's read ceiling for comparison with the CRC kernels.
__global__ void __launch_bounds__(256) read_stream_kernel(const uint8_t* base, uint64_t n16,
                                                          uint32_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t nth = (uint64_t)gridDim.x * 256;
  uint32_t acc = 0;
  uint64_t i = tid;
  const uint64_t b = (uint64_t)base;
  for (; i + 3 * nth < n16; i += 4 * nth) {
    const uint4 a0 = gload16(b + 16 * i), a1 = gload16(b + 16 * (i + nth));
    const uint4 a2 = gload16(b + 16 * (i + 2 * nth)), a3 = gload16(b + 16 * (i + 3 * nth));
    acc ^= a0.x ^ a0.y ^ a0.z ^ a0.w ^ a1.x ^ a1.y ^ a1.z ^ a1.w;
    acc ^= a2.x ^ a2.y ^ a2.z ^ a2.w ^ a3.x ^ a3.y ^ a3.z ^ a3.w;
  }
  for (; i < n16; i += nth) {
    const uint4 a = gload16(b + 16 * i);
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  out[tid] = acc;
}

// Diagnostic: read-ceiling probe.  U 16-byte loads per lane issued before any
// use, default or nt policy, for measuring how much memory-level parallelism
// the chip needs to approach its read peak.
template <int U, int NT>
__global__ void __launch_bounds__(1024) read_ceiling_kernel(const uint8_t* base, uint64_t n16,
                                                            uint32_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = tid;
  const uint64_t b = (uint64_t)base;
  for (; i + (U - 1) * nth < n16; i += U * nth) {
    uint4 a[U];
#pragma unroll
    for (int k = 0; k < U; k++) a[k] = gload16<NT ? 0 : kVarCached>(b + 16 * (i + k * nth));
#pragma unroll
    for (int k = 0; k < U; k++) acc ^= a[k].x ^ a[k].y ^ a[k].z ^ a[k].w;
  }
  for (; i < n16; i += nth) {
    const uint4 a = gload16(b + 16 * i);
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  out[tid] = acc;
}
#endif  // NOVA_DIAG

// ---- host: per-device tables ----------------------------------------------

struct DevTables {
  uint32_t* main[kNumG] = {};
  uint32_t* tree = nullptr;
  uint32_t* ft = nullptr;
  uint32_t* sh16 = nullptr;
  uint32_t* zero_word = nullptr;  // 16 zero bytes: the NULL-init stand-in
  uint32_t* byte8 = nullptr;      // M_1 byte table (flat kernel tail steps)
  uint32_t* byte8lm = nullptr;    // the same + 17 x 16-B prefix masks (rounds kernel head steps)
  uint32_t* op1024 = nullptr;     // M_1024 byte tables (burst kernel stream step)
  uint32_t* op1024r = nullptr;    // the same, 16-way bank-replicated
  uint32_t* ls_tabs = nullptr;    // log-stream kernel LDS tail: M4, M16 byte tables, 17 prefix masks
  int cus = 0;
  int err = 0;
  // Claim counters, one 16 KiB slot per HIP stream (256 workgroups x 64 B).
  // Launches on one stream run in order, so no two running launches share a
  // slot; each launch leaves its slot zeroed (sched_release).  A slot lives
  // until nova_stream_release(stream) (or process exit); the library's own
  // streams (port hook, host-streamed path) come from a pool and are reused.
  // The lock covers only the map: nothing waits on the GPU while holding it.
  std::mutex sched_mu;
  std::unordered_map<uint64_t, uint32_t*> sched_by_stream;
};

constexpr int kMaxDevices = 64;
constexpr int kSchedWords = 256 * 16;  // per stream: up to 256 workgroups x 64 B
thread_local std::atomic<int> g_tune_static_pct{-1};  // reused: steal probe limit (-1 = default)
DevTables g_dev[kMaxDevices];
std::once_flag g_once[kMaxDevices];

thread_local std::atomic<int> g_tune_g{0};
#ifdef NOVA_DIAG
thread_local std::atomic<int> g_tune_var{0};  // kernel variant (ablations)
#endif
thread_local std::atomic<int> g_tune_bpg{0};
thread_local std::atomic<int> g_tune_chunk{0};
thread_local std::atomic<int> g_tune_waves{0};  // waves per workgroup override (0 = per-kernel default)
thread_local std::atomic<int> g_tune_parity{0};  // XOR parity kernel variant (0 = default)

// Waves per workgroup.  The tables fill the CU's LDS, so a CU runs exactly one
// workgroup; fewer waves keep fewer HBM reads in flight per CU, which the
// streaming kernel prefers (tools/ceiling.py: 8 waves 2-3% faster than 16).
constexpr int kStreamWaves = 8;
constexpr int kUnitsWaves = 12;  // config 3 sweep: 12 > 16 > 8
int waves_per_wg(int def) {
  const int w = g_tune_waves.load();
  return (w > 0 && w <= kWaves) ? w : def;
}
#ifdef NOVA_DIAG
thread_local std::atomic<uint64_t*> g_diag_stamps{nullptr};
#endif
thread_local std::atomic<uint32_t> g_tune_seg{0};

void build_main_image(const nova::gf2::Lin& m, std::vector<uint32_t>& img) {
  uint32_t t[4][256];
  nova::gf2::byte_tables(m, t);
  img.assign(kMainBytes / 4, 0);
  for (int k = 0; k < 4; k++)
    for (int idx = 0; idx < 256; idx++)
      for (int c = 0; c < 32; c++) {
        const uint32_t byte = (uint32_t)((k >> 1) << 16) | (uint32_t)(idx << 8) |
                              (uint32_t)((k & 1) << 7) | (uint32_t)(c << 2);
        img[byte / 4] = t[k][idx];
      }
}

void append_op(const nova::gf2::Lin& m, std::vector<uint32_t>& v) {
  uint32_t t[4][256];
  nova::gf2::byte_tables(m, t);
  for (int k = 0; k < 4; k++) v.insert(v.end(), t[k], t[k] + 256);
}

template <typename T>
int upload(T** dst, const std::vector<uint32_t>& src) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, src.size() * 4);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpy(p, src.data(), src.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return (int)e;
  *dst = reinterpret_cast<T*>(p);
  return 0;
}

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

constexpr size_t kLdsMax = 160 * 1024;  // per CU on MI355X

// Flat kernel LDS: tables + byte table; the per-wave descriptor banks
// (2 x chunk x 16 B per wave) come on top (flat_lds_total).
template <int G>
constexpr size_t flat_lds() {
  return kMainBytes + (2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16)) * kTreeBytes + 1024;
}

#ifdef NOVA_DIAG
template <int G, int MODE, int VAR = 0>
int set_lds_attr_flat() {
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_flat_kernel<G, MODE, VAR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax);
}

template <int MODE, int VAR = 0>
int set_lds_attrs_flat() {
  int e = 0;
  if ((e = set_lds_attr_flat<1, MODE, VAR>())) return e;
  if ((e = set_lds_attr_flat<2, MODE, VAR>())) return e;
  if ((e = set_lds_attr_flat<4, MODE, VAR>())) return e;
  if ((e = set_lds_attr_flat<8, MODE, VAR>())) return e;
  return set_lds_attr_flat<16, MODE, VAR>();
}
#endif

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

template <int MODE>
int set_lds_attr_burst() {
  int e = (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_burst_kernel<64, MODE>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)burst_lds<64>());
  if (e) return e;
#ifdef NOVA_DIAG
  e = (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_burst_kernel<65, MODE>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)burst_lds<65>());
  if (e) return e;
  e = (int)hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_burst_kernel<16, MODE>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)burst_lds<16>());
#endif
  return e;
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

void init_device(int dev, DevTables* t) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) { t->err = (int)e; return; }
  t->cus = prop.multiProcessorCount;
  using namespace nova::gf2;
  const Lin m1 = zero_byte();
  std::vector<uint32_t> img;
  for (int gi = 0; gi < kNumG; gi++) {
    const int G = 1 << gi;
    build_main_image(power(m1, 16 * G), img);
    if ((t->err = upload(&t->main[gi], img))) return;
  }
  std::vector<uint32_t> tree;
  for (int l = 0; l < kTreeLevels; l++) append_op(power(m1, 4u << l), tree);
  if ((t->err = upload(&t->tree, tree))) return;
  std::vector<uint32_t> ft;
  const Lin m1inv = inverse(m1);
  const Lin m4 = power(m1, 4);
  for (int tt = 0; tt < 16; tt++) append_op(compose(power(m1inv, tt), m4), ft);
  if ((t->err = upload(&t->ft, ft))) return;
  std::vector<uint32_t> sh;
  Lin s = power(m1, 16);
  for (int b = 0; b < 32; b++) {
    append_op(s, sh);
    s = compose(s, s);
  }
  if ((t->err = upload(&t->sh16, sh))) return;
  if ((t->err = upload(&t->zero_word, std::vector<uint32_t>(4, 0u)))) return;
  {
    std::vector<uint32_t> b8(256);
    for (uint32_t b = 0; b < 256; b++) b8[b] = m1(b);
    if ((t->err = upload(&t->byte8, b8))) return;
    for (uint32_t nbytes = 0; nbytes <= 16; nbytes++)  // LM[n]: bytes [0, n) set
      for (uint32_t w = 0; w < 4; w++) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; b++)
          if (4 * w + b < nbytes) v |= 0xffu << (8 * b);
        b8.push_back(v);
      }
    if ((t->err = upload(&t->byte8lm, b8))) return;
  }
  {
    std::vector<uint32_t> op;
    append_op(power(m1, (uint32_t)kBurstSw), op);
    if ((t->err = upload(&t->op1024, op))) return;
#ifdef NOVA_DIAG
    std::vector<uint32_t> rep(16384);  // 4 tables x 256 entries x 16 replicas
    for (int k = 0; k < 4; k++)
      for (int idx = 0; idx < 256; idx++)
        for (int c = 0; c < 16; c++) rep[(k * 256 + idx) * 16 + c] = op[k * 256 + idx];
    if ((t->err = upload(&t->op1024r, rep))) return;
#endif
  }
#ifdef NOVA_DIAG  // log-stream experiment
  {
    std::vector<uint32_t> ls;
    append_op(power(m1, 4), ls);
    append_op(power(m1, 16), ls);
    for (uint32_t nbytes = 0; nbytes <= 16; nbytes++)
      for (uint32_t w = 0; w < 4; w++) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; b++)
          if (4 * w + b < nbytes) v |= 0xffu << (8 * b);
        ls.push_back(v);
      }
    if ((t->err = upload(&t->ls_tabs, ls))) return;
    for (const void* f : {reinterpret_cast<const void*>(&crc32c_logstream_kernel<kLogWrite>),
                          reinterpret_cast<const void*>(&crc32c_logstream_kernel<kLogVerify>),
#ifdef NOVA_DIAG
                          reinterpret_cast<const void*>(&crc32c_logstream_kernel<kLogWrite, kVarLsFast>),
#endif
                          })
      if ((t->err = (int)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)kLsLds)))
        return;
  }
#endif
  if ((t->err = set_lds_attrs_rounds<kStore>())) return;
  if ((t->err = set_lds_attrs_rounds<kStore, kVarInit>())) return;
  if ((t->err = set_lds_attrs_rounds<kTrailer>())) return;
  if ((t->err = set_lds_attrs_rounds<kVerify>())) return;
  if ((t->err = set_lds_attrs_rounds<kLogWrite>())) return;
  if ((t->err = set_lds_attrs_rounds<kLogVerify>())) return;
  if ((t->err = set_lds_attrs_mode<kStore>())) return;
  if ((t->err = set_lds_attrs_mode<kTrailer>())) return;
  if ((t->err = set_lds_attrs_mode<kVerify>())) return;
  if ((t->err = set_lds_attrs_mode<kLogWrite>())) return;
  if ((t->err = set_lds_attrs_mode<kLogVerify>())) return;
  if ((t->err = set_lds_attrs_stream<0>())) return;
  if ((t->err = set_lds_attr_burst<kStore>())) return;
  if ((t->err = set_lds_attr_burst<kTrailer>())) return;
  if ((t->err = set_lds_attr_burst<kVerify>())) return;
#ifdef NOVA_DIAG
  // timing ablations and alternative schedules (diagnostics build only)
  if ((t->err = set_lds_attrs_flat<kStore>())) return;
  if ((t->err = set_lds_attrs_flat<kTrailer>())) return;
  if ((t->err = set_lds_attrs_flat<kVerify>())) return;
  if ((t->err = set_lds_attrs_flat<kLogWrite>())) return;
  if ((t->err = set_lds_attrs_flat<kLogVerify>())) return;
  if ((t->err = set_lds_attrs_flat<kStore, kVarNoLookup>())) return;
  if ((t->err = set_lds_attrs_flat<kStore, kVarCached>())) return;
  if ((t->err = set_lds_attrs_rounds<kStore, kVarNoLookup>())) return;
  if ((t->err = set_lds_attrs_rounds<kStore, kVarNarrow>())) return;
  if ((t->err = set_lds_attrs_mode<kStore, kVarNoLookup>())) return;
  if ((t->err = set_lds_attrs_mode<kStore, kVarNarrow>())) return;
  if ((t->err = set_lds_attrs_mode<kStore, kVarCached>())) return;
  if ((t->err = set_lds_attrs_stream<kVarNoLookup>())) return;
  if ((t->err = set_lds_attrs_stream<kVarCached>())) return;
  if ((t->err = set_lds_attrs_stream<kVarWide>())) return;
  if ((t->err = set_lds_attrs_stream<kVarStamps>())) return;
  if ((t->err = set_lds_attrs_stream<kVarStamps | kVarStaticClaims>())) return;
#endif
}

DevTables* tables(int* err) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) { *err = NOVA_E_NODEV; return nullptr; }
  if (dev < 0 || dev >= kMaxDevices) { *err = NOVA_E_INVAL; return nullptr; }
  std::call_once(g_once[dev], [&] { init_device(dev, &g_dev[dev]); });
  if (g_dev[dev].err) { *err = g_dev[dev].err; return nullptr; }
  *err = 0;
  return &g_dev[dev];
}

// The calling stream's claim-counter slot, created zeroed (in stream order) on
// first use.  hipStreamPerThread names a different stream in every thread.
uint32_t* sched_slot(DevTables* t, hipStream_t stream) {
  uint64_t key = (uint64_t)(uintptr_t)stream;
  if (stream == hipStreamPerThread)
    key = (std::hash<std::thread::id>{}(std::this_thread::get_id()) << 1) | 1u;
  std::lock_guard<std::mutex> lk(t->sched_mu);
  auto it = t->sched_by_stream.find(key);
  if (it != t->sched_by_stream.end()) return it->second;
  void* d = nullptr;
  if (hipMalloc(&d, kSchedWords * sizeof(uint32_t)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(d, 0, kSchedWords * sizeof(uint32_t), stream) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  t->sched_by_stream.emplace(key, static_cast<uint32_t*>(d));
  return static_cast<uint32_t*>(d);
}

// Drop the stream's slot (nova_stream_release): waits for the stream's work,
// then frees the slot outside the lock.
int sched_release_stream(DevTables* t, hipStream_t stream) {
  uint64_t key = (uint64_t)(uintptr_t)stream;
  if (stream == hipStreamPerThread)
    key = (std::hash<std::thread::id>{}(std::this_thread::get_id()) << 1) | 1u;
  const hipError_t e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return (int)e;
  uint32_t* slot = nullptr;
  {
    std::lock_guard<std::mutex> lk(t->sched_mu);
    auto it = t->sched_by_stream.find(key);
    if (it == t->sched_by_stream.end()) return 0;
    slot = it->second;
    t->sched_by_stream.erase(it);
  }
  return (int)hipFree(slot);
}

size_t sched_slots(DevTables* t) {
  std::lock_guard<std::mutex> lk(t->sched_mu);
  return t->sched_by_stream.size();
}

int gindex(int G) { return G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : 4; }

// Dispatcher policy for batches the streaming kernel does not take.
// Kernels: rounds (sorted lockstep rounds of whole
// blocks, G = 8: the default), units (rounds of 32 KiB segments, G = 16: for
// batches of mostly >= 16 KiB blocks), flat (per-group block streams; on
// request), chosen with nova_diag_set_variable_kernel.  Lanes per block/unit
// and segment size can be forced with nova_crc32c_set_tuning.
constexpr int kFlatWaves = 12;  // sweep: 12 > 10 > 8 waves (more loads in flight)
uint64_t flat_waves() {
  const int w = waves_per_wg(kFlatWaves);
  return w > kFlatMaxWaves ? kFlatMaxWaves : w;
}
enum VarKernel { kAuto = 0, kUnitsK = 1, kFlatK = 2, kRoundsK = 3, kLogStreamK = 4 };
thread_local std::atomic<int> g_tune_kernel{0};
struct Plan {
  int kernel;
  int G;
  uint32_t seg;
  uint32_t chunk;  // rounds kernel: blocks per claimed chunk (0: the kernel's default)
};
// Measured (tools/sweep_flat.py, profiles/r01_sweep_lines.log):
//   SSTable-like 4096+U[0,255] B blocks: rounds G=8 73.7 %, units 53-57 %;
//   config 3 ({4,16,64} KiB + U[1,64]): units G=16/32 KiB segments 84.0 %,
//     rounds 75-78 %;
//   log records U[1,4096] B: rounds G=8, chunks of 64, 55.2 %.
// Blocks are checksummed whole in rounds unless the caller says most are
// >= 16 KiB (NOVA_CRC32C_HINT_LARGE_BLOCKS) or the fixed length is.
//
// Small batches (one SSTable per call, NovaLSM's pattern: ~4K blocks) are
// latency-bound: a wave walks its chunk's rounds one step at a time, so the
// launch lasts as long as the longest chunk.  Below ~2 chunks per wave slot
// the chunks shrink (32 -> 16 -> 8 blocks), and at <= 2 blocks per wave slot
// the groups widen to 16 lanes with 4-block chunks, halving the steps per
// block (tools/latency.py, profiles/r01_latency.log: 4K x 4 KiB verify
// 77 -> 31 us, 64K blocks 83 -> 70 us; 256K blocks unchanged).
Plan plan(uint64_t n_blocks, uint64_t bytes_per_block, bool uniform, int mode, bool large,
          uint32_t cus = 256) {
  const bool log = mode == kLogWrite || mode == kLogVerify;
  Plan pl{kRoundsK, 8, 0u, 0u};
  if (!log && ((uniform && bytes_per_block >= 16384) || (!uniform && large))) {
    pl.kernel = kUnitsK;
    pl.G = 16;
    pl.seg = 32768u;
  }
  const int tk = g_tune_kernel.load();
  const int tg = g_tune_g.load();
  const uint32_t ts = g_tune_seg.load();
  if (tk != kAuto && tk != kLogStreamK) pl.kernel = tk;
  if (ts) pl.kernel = kUnitsK;  // a forced segment size is a units-kernel setting
  if (tg == 1 || tg == 2 || tg == 4 || tg == 8 || tg == 16) pl.G = tg;
  if (ts) pl.seg = ts & ~15u;
  if (pl.kernel == kFlatK || pl.kernel == kRoundsK) {
    pl.seg = 0;
    if (pl.G == 1) pl.G = 2;  // at most 32 groups per wave (chunk >= 2 groups <= 64)
  }
  if (pl.kernel == kRoundsK && log && tk == kAuto && tg == 0 && g_tune_chunk.load() == 0) {
    // log records (~2 KiB): 16-record chunks below 32 chunks' worth per wave
    // slot (16 MiB log: 95 -> 40 us), the default 64 only for GiB-sized logs
    // (tools/latency_log.py, profiles/r01_latency_log.log)
    const uint64_t slots = 2ull * cus * flat_waves();
    pl.chunk = n_blocks >= 64 * slots ? 0u : (n_blocks >= 32 * slots ? 32u : 16u);
  }
  if (pl.kernel == kRoundsK && !log && tk == kAuto && tg == 0 && g_tune_chunk.load() == 0) {
    const uint64_t slots = 2ull * cus * flat_waves();  // two chunks per wave slot
    if (n_blocks <= slots) {
      pl.G = 16;
      pl.chunk = 4;
    } else {
      pl.chunk = n_blocks >= 32 * slots ? 32u : (n_blocks >= 16 * slots ? 16u : 8u);
    }
  }
  return pl;
}

size_t flat_lds_g(int G);
#ifdef NOVA_DIAG
// Blocks per claimed chunk of the flat kernel: one per lane group (the bank
// refill is one step old when read), four per group for log records (the
// header bytes need two more steps); at most 64 (one per lane).
uint32_t flat_chunk(int G, int mode) {
  const uint32_t groups = 64u / (uint32_t)G;
  const bool log = mode == kLogWrite || mode == kLogVerify;
  const int tc = g_tune_chunk.load();
  uint32_t c = tc > 0 ? (uint32_t)tc : (log ? 4 * groups : 2 * groups);
  // the descriptor banks must fit next to the tables
  const uint64_t room = (kLdsMax - flat_lds_g(G)) / (flat_waves() * 2 * 16);
  if (c > room) c = (uint32_t)room;
  if (c > 64) c = 64;
  if (c < 2 * groups) c = 2 * groups;  // the kernel relies on it (positions < 2C)
  return c;
}
#endif

size_t flat_lds_g(int G) {
  switch (G) {
    case 1: return flat_lds<1>();
    case 2: return flat_lds<2>();
    case 4: return flat_lds<4>();
    case 8: return flat_lds<8>();
    default: return flat_lds<16>();
  }
}

#ifdef NOVA_DIAG
template <int MODE, int VAR>
int launch_flat_g(int G, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const CrcParams& p) {
  switch (G) {
    case 1: hipLaunchKernelGGL((crc32c_flat_kernel<1, MODE, VAR>), grid, block, lds, stream, p); break;
    case 2: hipLaunchKernelGGL((crc32c_flat_kernel<2, MODE, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_flat_kernel<4, MODE, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_flat_kernel<8, MODE, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_flat_kernel<16, MODE, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
}

template <int MODE>
int launch_flat(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
  p.tab_main = t->main[gindex(G)];
  p.tab_tree = t->tree;
  p.tab_byte = t->byte8;
  p.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
  p.omask = p.lmask = p.imask = ~0ull;
  if (p.offsets) {
    p.stride = 0;
  } else {  // fixed stride: offset i * stride
    p.offsets = reinterpret_cast<const uint64_t*>(t->zero_word);
    p.omask = 0;
  }
  if (p.lengths) {
    p.len = 0;
  } else {  // fixed length p.len (log modes read the header instead)
    p.lengths = t->zero_word;
    p.lmask = 0;
  }
  if (!p.init) {
    p.init = t->zero_word;
    p.imask = 0;
  }
  p.chunk = flat_chunk(G, MODE);
  p.n_chunks = (p.n_blocks + p.chunk - 1) / p.chunk;
  uint64_t nwaves = flat_waves();
  while (nwaves > 1 && flat_lds_g(G) + nwaves * 2 * p.chunk * 16 > kLdsMax) nwaves--;  // G = 2
  uint64_t wgs = (p.n_chunks + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  if (wgs == 0) return 0;
  {
    const int sl = g_tune_static_pct.load();
    p.steal_limit = sl < 0 ? 8u : (uint32_t)sl;
    // The first nwaves x wgs chunks are implicit (one per wave): when they cover
    // the batch, a claim or a steal can only come back empty, and each of the
    // 8 probes is a serial device-scope atomic (~1.5 us) on the launch's tail.
    if (sl < 0 && p.n_chunks <= wgs * (uint64_t)nwaves) p.steal_limit = 0;
  }
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const dim3 block(64 * nwaves);
  const size_t lds = flat_lds_g(G) + nwaves * 2 * p.chunk * 16;
  if (lds > kLdsMax) return NOVA_E_INVAL;
  const int var = g_tune_var.load();
  if (MODE == kStore && var == kVarNoLookup) return launch_flat_g<kStore, kVarNoLookup>(G, dim3(wgs), block, lds, stream, p);
  if (MODE == kStore && var == kVarCached) return launch_flat_g<kStore, kVarCached>(G, dim3(wgs), block, lds, stream, p);
  return launch_flat_g<MODE, 0>(G, dim3(wgs), block, lds, stream, p);
}
#endif  // NOVA_DIAG

template <int MODE, int VAR>
int launch_g(int G, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const CrcParams& p) {
  switch (G) {
    case 1: hipLaunchKernelGGL((crc32c_units_kernel<1, MODE, VAR>), grid, block, lds, stream, p); break;
    case 2: hipLaunchKernelGGL((crc32c_units_kernel<2, MODE, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_units_kernel<4, MODE, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_units_kernel<8, MODE, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_units_kernel<16, MODE, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
}

template <int MODE>
int launch_mode(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
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
  const uint64_t nwaves = waves_per_wg(kUnitsWaves);
  uint64_t wgs = (p.n_chunks + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  if (wgs == 0) return 0;
  {
    const int sl = g_tune_static_pct.load();
    p.steal_limit = sl < 0 ? 8u : (uint32_t)sl;
    // The first nwaves x wgs chunks are implicit (one per wave): when they cover
    // the batch, a claim or a steal can only come back empty, and each of the
    // 8 probes is a serial device-scope atomic (~1.5 us) on the launch's tail.
    if (sl < 0 && p.n_chunks <= wgs * (uint64_t)nwaves) p.steal_limit = 0;
  }
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const int levels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  const size_t lds = kMainBytes + levels * kTreeBytes + kWaves * kWaveScratch;
  const dim3 block(64 * nwaves);
#ifdef NOVA_DIAG
  const int var = g_tune_var.load();
  if (MODE == kStore && var == kVarNoLookup) return launch_g<kStore, kVarNoLookup>(G, dim3(wgs), block, lds, stream, p);
  if (MODE == kStore && var == kVarNarrow) return launch_g<kStore, kVarNarrow>(G, dim3(wgs), block, lds, stream, p);
  if (MODE == kStore && var == kVarCached) return launch_g<kStore, kVarCached>(G, dim3(wgs), block, lds, stream, p);
#endif
  return launch_g<MODE, 0>(G, dim3(wgs), block, lds, stream, p);
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

// Lanes per block for the streaming kernel, or 0 if the batch is not eligible
// (unaligned base/stride, or len not a multiple of 128*G for any G).
// Measured on MI355X (tools/sweep.py): G = 16 for blocks >= 16 KiB, else 8.
int stream_lanes(const CrcParams& p) {
  if (((uint64_t)p.base & 15) || (p.stride & 15) || p.len == 0 || p.stride < p.len) return 0;
  int want = p.len >= 16384 ? 16 : 8;
  const int tg = g_tune_g.load();
  if (tg == 1 || tg == 2 || tg == 4 || tg == 8 || tg == 16) want = tg;
  for (int g = want; g >= 1; g >>= 1)
    if (p.len % (128u * g) == 0) return g;  // KG = len / 64G even
  return 0;
}

// Blocks per lane group per round: a wave-round of ~64 KiB measured best on
// MI355X at every block size tried (4 KiB: G=8 x 2 blocks, 76% of 8 TB/s vs
// 71% with 1; 16 KiB: G=16 x 1 block, 82%).
uint32_t stream_bpg(int G, uint32_t len) {
  const int tb = g_tune_bpg.load();
  if (tb > 0) return (uint32_t)tb;
  const uint64_t per_round = (uint64_t)(64 / G) * len;
  uint64_t b = 65536 / (per_round ? per_round : 1);
  return b < 1 ? 1u : (b > 64 ? 64u : (uint32_t)b);
}

// Scratch that lives between launches of ONE call is allocated and freed in
// stream order (hipMallocAsync / hipFreeAsync from the device's default
// pool): every call owns its own array, so calls from several host threads
// on one stream cannot see each other's scratch, and nothing is freed while
// a kernel still reads it.
struct StreamScratch {
  void* p = nullptr;
  hipStream_t s = nullptr;
  int alloc(size_t bytes, hipStream_t stream) {
    s = stream;
    if (hipMallocAsync(&p, bytes, stream) == hipSuccess) return 0;
    p = nullptr;
    (void)hipGetLastError();  // not sticky for the caller's next launch check
    return NOVA_E_NOMEM;
  }
  ~StreamScratch() {
    if (p) (void)hipFreeAsync(p, s);
  }
};

#ifdef NOVA_DIAG
template <int MODE>
int launch_sort(CrcParams& p, DevTables* t, hipStream_t stream, uint64_t kStep, StreamScratch& sc) {
  const size_t hist_bytes = 2 * kBins * sizeof(uint32_t);
  if (sc.alloc(hist_bytes + p.n_blocks * sizeof(uint32_t), stream)) return NOVA_E_NOMEM;
  uint32_t* hist = static_cast<uint32_t*>(sc.p);
  uint32_t* perm = hist + 2 * kBins;
  hipError_t e = hipMemsetAsync(hist, 0, kBins * sizeof(uint32_t), stream);
  if (e != hipSuccess) return (int)e;
  uint64_t wgs = (p.n_blocks + 255) / 256;
  const uint64_t cap = (uint64_t)t->cus * 4;
  if (wgs > cap) wgs = cap;
  hipLaunchKernelGGL(bin_count_kernel<MODE>, dim3(wgs), dim3(256), 0, stream, p, kStep, hist);
  hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(kBins), 0, stream, hist, hist + kBins);
  hipLaunchKernelGGL(bin_scatter_kernel<MODE>, dim3(wgs), dim3(256), 0, stream, p, kStep,
                     hist + kBins, perm);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  p.perm = perm;
  return 0;
}
#endif

thread_local std::atomic<int> g_tune_sort{2};  // rounds kernel: 0 in order, 1 whole-batch sort, 2 per chunk
#ifdef NOVA_DIAG
thread_local std::atomic<int> g_tune_trailer_1pass{0};  // diagnostics: trailer / log-write store forms (run())
constexpr uint64_t kLogWindowMin = 1u << 15;  // diagnostics: log records, whole-piece CRC-field stores from here
#endif

template <int MODE, int VAR>
int launch_rounds_g(int G, dim3 grid, dim3 block, size_t lds, hipStream_t stream, const CrcParams& p) {
  switch (G) {
    case 2: hipLaunchKernelGGL((crc32c_rounds_kernel<2, MODE, VAR>), grid, block, lds, stream, p); break;
    case 4: hipLaunchKernelGGL((crc32c_rounds_kernel<4, MODE, VAR>), grid, block, lds, stream, p); break;
    case 8: hipLaunchKernelGGL((crc32c_rounds_kernel<8, MODE, VAR>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((crc32c_rounds_kernel<16, MODE, VAR>), grid, block, lds, stream, p); break;
  }
  return (int)hipGetLastError();
}

template <int MODE>
int launch_rounds(int G, CrcParams& p, DevTables* t, hipStream_t stream, uint32_t chunk = 0) {
  if (G < 2) G = 2;
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
  if (!p.gate) p.perm = nullptr;  // (the log-stream follow-up passes its leftover list)
  const int sort = g_tune_sort.load();  // 0 none, 1 whole batch (pre-pass), 2 per chunk
  p.sort_local = sort == 2 ? 1u : 0u;
#ifdef NOVA_DIAG
  StreamScratch sort_sc;  // freed in stream order after the launch below
  if (sort == 1 && p.n_blocks >= 1024) {
    const int e = launch_sort<MODE>(p, t, stream, 64ull * G, sort_sc);
    if (e) return e;
  }
#endif
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
  const uint64_t nwaves = flat_waves();
  uint64_t wgs = (p.n_chunks + nwaves - 1) / nwaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  if (wgs == 0) return 0;
  {
    const int sl = g_tune_static_pct.load();
    p.steal_limit = sl < 0 ? 8u : (uint32_t)sl;
    // The first nwaves x wgs chunks are implicit (one per wave): when they cover
    // the batch, a claim or a steal can only come back empty, and each of the
    // 8 probes is a serial device-scope atomic (~1.5 us) on the launch's tail.
    if (sl < 0 && p.n_chunks <= wgs * (uint64_t)nwaves) p.steal_limit = 0;
  }
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const dim3 block(64 * nwaves);
  const size_t lds = flat_lds_g(G) + 272 + nwaves * 64 * 4;  // + prefix masks, per-wave sort scratch
#ifdef NOVA_DIAG
  if (MODE == kStore && g_tune_var.load() == kVarNoLookup)
    return launch_rounds_g<kStore, kVarNoLookup>(G, dim3(wgs), block, lds, stream, p);
  if (MODE == kStore && g_tune_var.load() == kVarNarrow)
    return launch_rounds_g<kStore, kVarNarrow>(G, dim3(wgs), block, lds, stream, p);
  if ((MODE == kVerify || MODE == kLogVerify) && g_tune_var.load() == kVarNoTail)
    return launch_rounds_g<MODE, kVarNoTail>(G, dim3(wgs), block, lds, stream, p);
#endif
  if (MODE == kStore && p.imask != 0)
    return launch_rounds_g<kStore, kVarInit>(G, dim3(wgs), block, lds, stream, p);
  return launch_rounds_g<MODE, 0>(G, dim3(wgs), block, lds, stream, p);
}

int launch_stream(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
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
  {
    const int sl = g_tune_static_pct.load();
    p.steal_limit = sl < 0 ? 8u : (uint32_t)sl;  // 8 probes = one victim per XCD
    // the first nwaves x wgs rounds are implicit: if they cover the batch no
    // claim or steal can find work (8 serial atomics on the tail otherwise)
    if (sl < 0 && rounds <= wgs * nwaves) p.steal_limit = 0;
  }
  // claim counters of this stream (left zeroed by the previous launch)
  p.sched = sched_slot(t, stream);
  if (!p.sched) return NOVA_E_NOMEM;
  const int levels = 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16);
  const size_t lds = kMainBytes + levels * kTreeBytes;
#ifdef NOVA_DIAG
  if (g_tune_var.load() == kVarNoLookup) return launch_stream_g<kVarNoLookup>(G, dim3(wgs), lds, stream, p);
  if (g_tune_var.load() == kVarCached) return launch_stream_g<kVarCached>(G, dim3(wgs), lds, stream, p);
  if (g_tune_var.load() == kVarWide) return launch_stream_g<kVarWide>(G, dim3(wgs), lds, stream, p);
  if (g_tune_var.load() == kVarStamps) {
    p.stamps = g_diag_stamps.load();
    return launch_stream_g<kVarStamps>(G, dim3(wgs), lds, stream, p);
  }
  if (g_tune_var.load() == (kVarStamps | kVarStaticClaims)) {
    p.stamps = g_diag_stamps.load();
    return launch_stream_g<kVarStamps | kVarStaticClaims>(G, dim3(wgs), lds, stream, p);
  }
#endif
  return launch_stream_g<0>(G, dim3(wgs), lds, stream, p);
}

// One SSTable per call: batches up to burst_max() blocks (two per wave slot of
// the rounds kernel, 6144 on 256 CUs) go to the burst kernel, one wave per
// block on the compact tables, unless tuning forces a kernel.
thread_local std::atomic<int> g_tune_burst{0};  // diagnostics: 0 auto, 16/64/65 force, -1 off
uint64_t burst_max(uint32_t cus) { return 2ull * cus * flat_waves(); }
int burst_lanes(int mode, uint64_t n_blocks, uint32_t cus) {
  if (mode != kStore && mode != kTrailer && mode != kVerify) return 0;
  const int tb = g_tune_burst.load();
  if (tb < 0) return 0;
  if (tb == 16 || tb == 64 || tb == 65) return tb;
  if (g_tune_g.load() || g_tune_seg.load() || g_tune_kernel.load()) return 0;
  return n_blocks <= burst_max(cus) ? 64 : 0;
}

template <int V, int MODE>
int launch_burst(CrcParams& p, DevTables* t, hipStream_t stream) {
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
#ifdef NOVA_DIAG
  if (g_tune_var.load() == kVarStamps) p.stamps = g_diag_stamps.load();
#endif
  hipLaunchKernelGGL((crc32c_burst_kernel<V, MODE>), dim3(wgs), dim3(64 * nw), burst_lds<V>(),
                     stream, p);
  return (int)hipGetLastError();
}

template <int MODE>
int launch_burst_g(int V, CrcParams& p, DevTables* t, hipStream_t stream) {
#ifdef NOVA_DIAG
  // measured slower at every batch size (profiles/r02_latency_burst_variants.log)
  if (V == 65) return launch_burst<65, MODE>(p, t, stream);
  if (V == 16) return launch_burst<16, MODE>(p, t, stream);
#endif
  return launch_burst<64, MODE>(p, t, stream);
}

#ifdef NOVA_DIAG
// Log-stream experiment (nova_diag_set_variable_kernel(4)):
// a pre-pass finds each 32 KiB block's first record, the log-stream kernel
// streams the image, and the rounds kernel follows, gated: the leftover list,
// or the whole batch if a precondition failed.  Measured slower than the
// rounds kernel on 2 KiB-average records, so the product does not use it.
template <int MODE>
int launch_logstream(CrcParams& p, DevTables* t, hipStream_t stream) {
  const uint64_t nb = (p.buf_len + kLogBlock - 1) / kLogBlock;
  // [flag, mismatches, leftovers, -, first[0..nb], leftover list[n]], freed in stream order
  StreamScratch sc;
  const uint64_t left_at = (4 + nb + 1 + 3) & ~3ull;
  if (sc.alloc((left_at + p.n_blocks) * sizeof(uint32_t), stream)) return NOVA_E_NOMEM;
  uint32_t* w = static_cast<uint32_t*>(sc.p);
  hipError_t e = hipMemsetAsync(w, 0, 16, stream);
  if (e != hipSuccess) return (int)e;
  uint32_t* first = w + 4;
  uint64_t fwgs = (p.n_blocks + 1 + 255) / 256;
  if (fwgs > (uint64_t)t->cus * 8) fwgs = (uint64_t)t->cus * 8;
  hipLaunchKernelGGL(log_first_kernel, dim3(fwgs), dim3(256), 0, stream, p.offsets, p.n_blocks, nb,
                     first, w);
  CrcParams s = p;
  s.first = first;
  s.n_lblocks = nb;
  s.ls_flag = w;
  s.ls_bad = w + 1;
  s.ls_left = w + left_at;
  s.tab_main = t->main[gindex(kLsG)];
  s.tab_tree = t->ls_tabs;
  s.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
  const uint64_t R = (nb + 7) / 8;
  uint64_t wgs = (R + kLsWaves - 1) / kLsWaves;
  if (wgs > (uint64_t)t->cus) wgs = t->cus;
  if (wgs > 256) wgs = 256;
  s.steal_limit = R <= wgs * kLsWaves ? 0u : 8u;
  s.sched = sched_slot(t, stream);
  if (!s.sched) return NOVA_E_NOMEM;
#ifdef NOVA_DIAG
  if (MODE == kLogWrite && g_tune_var.load() == kVarLsFast)
    hipLaunchKernelGGL((crc32c_logstream_kernel<kLogWrite, kVarLsFast>), dim3(wgs), dim3(64 * kLsWaves),
                       kLsLds, stream, s);
  else
#endif
    hipLaunchKernelGGL(crc32c_logstream_kernel<MODE>, dim3(wgs), dim3(64 * kLsWaves), kLsLds, stream, s);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  CrcParams f = p;  // follow-up: the leftover list, or the whole batch if flagged
  f.gate = w;
  f.ls_bad = w + 1;
  f.perm = w + left_at;
  const Plan pl = plan(p.n_blocks, 0, false, MODE, false, (uint32_t)t->cus);
  return launch_rounds<MODE>(pl.G, f, t, stream, pl.chunk);
}
#endif  // NOVA_DIAG

// Few large blocks -> the split-and-combine path (split_*_kernel): uniform
// blocks over kBurstMaxLen in a batch of at most kSplitMaxBlocks, or a batch of
// at most kSplitMaxHinted blocks the caller marks HINT_LARGE_BLOCKS (the host
// does not see variable lengths; read-verify takes the hint through
// nova_sstable_verify_blocks_ex).  tools/big_blocks.py measures both sides.
thread_local std::atomic<int> g_tune_split{0};  // 0 auto, 1 force, -1 off
constexpr uint64_t kBurstMaxLen = 65536;
constexpr uint64_t kSplitMaxBlocks = 8192, kSplitMaxHinted = 1024;
constexpr uint64_t kSplitTargetPieces = 65536;
bool split_wanted(int mode, const CrcParams& p, bool uniform, uint64_t len) {
  if (mode != kStore && mode != kTrailer && mode != kVerify) return false;
  const int ts = g_tune_split.load();
  if (ts) return ts > 0;
  if (g_tune_g.load() || g_tune_seg.load() || g_tune_kernel.load() || g_tune_burst.load()) return false;
  if (p.n_blocks > kSplitMaxBlocks) return false;
  if (uniform) return len > kBurstMaxLen;
  return (p.flags & NOVA_CRC32C_HINT_LARGE_BLOCKS) != 0 && p.n_blocks <= kSplitMaxHinted;
}
uint32_t ceil_log2(uint64_t x) {
  uint32_t k = 0;
  while ((1ull << k) < x) k++;
  return k;
}
// Piece size S and kmax = 2^kshift slots per block: about kSplitTargetPieces
// pieces of 4..64 KiB for a uniform batch; 16 KiB pieces and enough slots for
// 1 GiB of blocks in total otherwise.
void split_shape(uint64_t n, bool uniform, uint64_t len_in, uint32_t* S, uint32_t* kshift) {
  if (uniform) {
    const uint64_t total = n * (len_in ? len_in : 1);
    uint64_t s = 1ull << ceil_log2((total + kSplitTargetPieces - 1) / kSplitTargetPieces);
    s = s < 4096 ? 4096 : (s > 65536 ? 65536 : s);
    *S = (uint32_t)s;
    const uint32_t k = ceil_log2((len_in + s - 1) / s);
    *kshift = k > 16 ? 16u : k;
  } else {
    *S = 16384;
    const uint32_t k = ceil_log2((kSplitTargetPieces + n - 1) / n);
    *kshift = k > 16 ? 16u : k;
  }
}

// launch_split's "nothing launched" return: its scratch (or the stream's
// claim slot) could not be had before any kernel was queued, so the caller may
// still run the one-pass kernels.  Every later failure is the caller's error.
constexpr int kSplitNoScratch = -1000;

int launch_split(int mode, CrcParams& p, bool uniform, uint64_t len, DevTables* t, hipStream_t stream) {
  const uint32_t extra = mode == kVerify ? 1u : 0u;
  uint32_t S = 0, kshift = 0;
  split_shape(p.n_blocks, uniform, len + extra, &S, &kshift);
  const uint64_t slots = p.n_blocks << kshift;
  // [piece offsets u64][piece lengths u32][piece raws u32][per-block xor
  // word], freed in stream order after the last kernel
  StreamScratch sc;
  if (sc.alloc(slots * 16 + p.n_blocks * 4, stream)) return kSplitNoScratch;
  if (!sched_slot(t, stream)) return kSplitNoScratch;  // the pieces' launch needs it
  uint64_t* poff = static_cast<uint64_t*>(sc.p);
  uint32_t* plen = reinterpret_cast<uint32_t*>(poff + slots);
  uint32_t* praw = plen + slots;
  uint32_t* acc = praw + slots;
  p.tab_sh16 = t->sh16;
  const uint64_t cap = (uint64_t)t->cus * 8;
  const uint64_t wgs = (slots + 255) / 256;
  hipLaunchKernelGGL(split_pieces_kernel, dim3(wgs < cap ? wgs : cap), dim3(256), 0, stream, p, extra,
                     S, kshift, poff, plen, acc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  CrcParams q{};
  q.base = p.base;
  q.offsets = poff;
  q.lengths = plen;
  q.out = praw;
  q.n_blocks = slots;
  const bool big = S >= 16384;
  q.flags = NOVA_CRC32C_RAW | (big ? NOVA_CRC32C_HINT_LARGE_BLOCKS : 0u);
  const Plan pl = plan(slots, 0, false, kStore, big, (uint32_t)t->cus);
  q.seg = pl.seg;
  const int rc = pl.kernel == kRoundsK ? launch_rounds<kStore>(pl.G, q, t, stream, pl.chunk)
                                       : launch_mode<kStore>(pl.G, q, t, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(split_fold_kernel, dim3(wgs), dim3(256), 0, stream, p, mode, extra, S, kshift,
                     praw, acc);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if (kshift <= 6) return 0;  // kmax <= 64: the fold finished every block
  const uint64_t fwgs = (p.n_blocks + 255) / 256;
  hipLaunchKernelGGL(split_finish_kernel, dim3(fwgs < cap ? fwgs : cap), dim3(256), 0, stream, p, mode,
                     extra, acc);
  return (int)hipGetLastError();
}

int run(int mode, CrcParams& p, bool uniform, uint64_t bytes_per_block, hipStream_t stream) {
  int err = 0;
  DevTables* t = tables(&err);
  if (!t) return err;
  if (p.n_blocks == 0) return 0;
  if (split_wanted(mode, p, uniform, bytes_per_block)) {
    // no scratch for the pieces (nothing launched yet): the one-pass kernels
    // below; any failure after the first launch is returned as is
    const int rc = launch_split(mode, p, uniform, bytes_per_block, t, stream);
    if (rc != kSplitNoScratch) return rc;
  }
  if (const int bg = burst_lanes(mode, p.n_blocks, (uint32_t)t->cus)) {
    switch (mode) {
      case kStore: return launch_burst_g<kStore>(bg, p, t, stream);
      case kTrailer: return launch_burst_g<kTrailer>(bg, p, t, stream);
      default: return launch_burst_g<kVerify>(bg, p, t, stream);
    }
  }
#ifdef NOVA_DIAG
  if ((mode == kLogWrite || mode == kLogVerify) && p.n_blocks < (1ull << 31) &&
      g_tune_kernel.load() == kLogStreamK)
    return mode == kLogWrite ? launch_logstream<kLogWrite>(p, t, stream)
                             : launch_logstream<kLogVerify>(p, t, stream);
#endif
  if (mode == kStore && uniform && !g_tune_seg.load()) {
    const int sg = stream_lanes(p);
    if (sg) return launch_stream(sg, p, t, stream);
  }
  const Plan pl = plan(p.n_blocks, bytes_per_block, uniform, mode,
                       (p.flags & NOVA_CRC32C_HINT_LARGE_BLOCKS) != 0, (uint32_t)t->cus);
  const int G = pl.G;
  p.seg = pl.seg;
  // Batches that fit the implicit per-wave chunks (SSTable-sized, latency-bound)
  // write their trailers from the CRC kernel: a second launch would add its
  // whole fixed cost to the call.
  // Trailers and log CRC fields are stored by the CRC kernel itself (byte
  // stores).  The image writes cost ~13 points on SSTable-like images whatever
  // their form -- two passes, whole 64-B pieces, non-temporal -- while the
  // same kernels without the writes run at the verify rate;
  // those forms stay in the diagnostics build as measured experiments.
#ifdef NOVA_DIAG
  const bool small = p.n_blocks <= 2ull * t->cus * flat_waves();
  // g_tune_trailer_1pass: 2 = trailers in two passes; 3 = whole-64-B-piece
  // stores; 4 = the same non-temporal; 5 = whole-piece form without result
  // writes; 6 = no result writes (timing ablations: 5 and 6 write nothing)
  const int tkn = g_tune_trailer_1pass.load();
  p.wvar = tkn == 4 ? 1u : (tkn == 5 || tkn == 6) ? 2u : tkn == 7 ? 3u : 0u;
  const bool tk_piece = tkn == 3 || tkn == 4 || tkn == 5;
  if (pl.kernel == kRoundsK && mode == kTrailer && tk_piece && !small) {
    // whole-64-B-piece trailer stores where the layout allows it
    // (trailer_layout_kernel)
    StreamScratch sc;  // flag + eligibility, freed in stream order after the CRC kernel
    if (sc.alloc(sizeof(uint32_t) * (p.n_blocks + 1), stream)) return NOVA_E_NOMEM;
    uint32_t* flag = static_cast<uint32_t*>(sc.p);
    uint32_t* elig = flag + 1;
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return (int)e;
    uint64_t wgs = (p.n_blocks + 255) / 256;
    const uint64_t cap = (uint64_t)t->cus * 8;
    if (wgs > cap) wgs = cap;
    // descriptors as launch_rounds normalises them (absent arrays: stride / len)
    const uint64_t* lo = p.offsets ? p.offsets : reinterpret_cast<const uint64_t*>(t->zero_word);
    const uint32_t* ll = p.lengths ? p.lengths : t->zero_word;
    hipLaunchKernelGGL(trailer_layout_kernel, dim3(wgs), dim3(256), 0, stream, (uint64_t)p.base, lo,
                       p.offsets ? ~0ull : 0ull, ll, p.lengths ? ~0ull : 0ull,
                       p.offsets ? 0ull : p.stride, p.lengths ? 0u : p.len, p.n_blocks, elig, flag);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    CrcParams q = p;
    q.tr_flag = flag;
    q.init = elig;  // trailer mode reads each block's eligibility in place of an init
    return launch_rounds<kTrailer>(G, q, t, stream, pl.chunk);
  }
  if (pl.kernel == kRoundsK && mode == kLogWrite && tk_piece &&
      p.n_blocks >= kLogWindowMin && p.offsets) {
    // whole-64-B-piece CRC-field stores where the layout allows it
    // (log_window_kernel)
    StreamScratch sc;  // flag + eligibility, freed in stream order after the CRC kernel
    if (sc.alloc(sizeof(uint32_t) * (p.n_blocks + 1), stream)) return NOVA_E_NOMEM;
    uint32_t* flag = static_cast<uint32_t*>(sc.p);
    uint32_t* elig = flag + 1;
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return (int)e;
    uint64_t wgs = (p.n_blocks + 255) / 256;
    const uint64_t cap = (uint64_t)t->cus * 8;
    if (wgs > cap) wgs = cap;
    hipLaunchKernelGGL(log_window_kernel, dim3(wgs), dim3(256), 0, stream, p.offsets, p.n_blocks,
                       p.buf_len, elig, flag);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    CrcParams q = p;
    q.tr_flag = flag;
    q.init = elig;  // log write reads each record's eligibility in place of an init
    return launch_rounds<kLogWrite>(G, q, t, stream, pl.chunk);
  }
  if (pl.kernel == kRoundsK && mode == kTrailer && tkn == 8 && !small) {
    // Two passes: CRCs into this call's own stream-ordered array (with the
    // layout pre-pass's flag and eligibility), then trailer_rmw_kernel
    StreamScratch sc;  // flag, eligibility, CRCs; freed in stream order after the second pass
    if (sc.alloc(sizeof(uint32_t) * (2 * p.n_blocks + 1), stream)) return NOVA_E_NOMEM;
    uint32_t* flag = static_cast<uint32_t*>(sc.p);
    uint32_t* elig = flag + 1;
    uint32_t* tmp = elig + p.n_blocks;
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return (int)e;
    uint64_t wgs = (p.n_blocks + 255) / 256;
    const uint64_t cap = (uint64_t)t->cus * 8;
    if (wgs > cap) wgs = cap;
    const uint64_t* lo = p.offsets ? p.offsets : reinterpret_cast<const uint64_t*>(t->zero_word);
    const uint32_t* ll = p.lengths ? p.lengths : t->zero_word;
    const uint64_t om = p.offsets ? ~0ull : 0ull, lm = p.lengths ? ~0ull : 0ull;
    const uint64_t st = p.offsets ? 0ull : p.stride;
    const uint32_t ln = p.lengths ? 0u : p.len;
    hipLaunchKernelGGL(trailer_layout_kernel, dim3(wgs), dim3(256), 0, stream, (uint64_t)p.base, lo,
                       om, ll, lm, st, ln, p.n_blocks, elig, flag);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    CrcParams q = p;
    q.out = tmp;
    q.flags = (p.flags & 0xff00u) | NOVA_CRC32C_APPEND_TYPE | NOVA_CRC32C_MASK_OUTPUT;
    const int e2 = launch_rounds<kStore>(G, q, t, stream, pl.chunk);
    if (e2) return e2;
    uint64_t wgs8 = (p.n_blocks * 8 + 255) / 256;
    if (wgs8 > cap) wgs8 = cap;
    hipLaunchKernelGGL(trailer_rmw_kernel, dim3(wgs8), dim3(256), 0, stream,
                       const_cast<uint8_t*>(p.base), lo, om, ll, lm, st, ln, tmp, elig, flag,
                       p.n_blocks, p.flags);
    return (int)hipGetLastError();
  }
  if (pl.kernel == kRoundsK && mode == kTrailer && tkn == 2 && !small) {
    // Two passes: CRCs (type byte appended, masked) into this call's own
    // stream-ordered array, then the trailer bytes (trailer_scatter_kernel).
    StreamScratch sc;  // freed in stream order after the scatter
    if (sc.alloc(p.n_blocks * sizeof(uint32_t), stream)) return NOVA_E_NOMEM;
    uint32_t* tmp = static_cast<uint32_t*>(sc.p);
    CrcParams q = p;
    q.out = tmp;
    q.flags = (p.flags & 0xff00u) | NOVA_CRC32C_APPEND_TYPE | NOVA_CRC32C_MASK_OUTPUT;
    const int e = launch_rounds<kStore>(G, q, t, stream, pl.chunk);
    if (e) return e;
    uint64_t wgs = (p.n_blocks + 255) / 256;
    const uint64_t cap = (uint64_t)t->cus * 8;
    if (wgs > cap) wgs = cap;
    hipLaunchKernelGGL(trailer_scatter_kernel, dim3(wgs), dim3(256), 0, stream,
                       const_cast<uint8_t*>(p.base), p.offsets, p.lengths, tmp, p.n_blocks, p.flags);
    return (int)hipGetLastError();
  }
#endif
  if (pl.kernel == kRoundsK) {
    switch (mode) {
      case kStore: return launch_rounds<kStore>(G, p, t, stream, pl.chunk);
      case kTrailer: return launch_rounds<kTrailer>(G, p, t, stream, pl.chunk);
      case kLogWrite: return launch_rounds<kLogWrite>(G, p, t, stream, pl.chunk);
      case kLogVerify: return launch_rounds<kLogVerify>(G, p, t, stream, pl.chunk);
      default: return launch_rounds<kVerify>(G, p, t, stream, pl.chunk);
    }
  }
#ifdef NOVA_DIAG
  if (pl.kernel == kFlatK) {
    switch (mode) {
      case kStore: return launch_flat<kStore>(G, p, t, stream);
      case kTrailer: return launch_flat<kTrailer>(G, p, t, stream);
      case kLogWrite: return launch_flat<kLogWrite>(G, p, t, stream);
      case kLogVerify: return launch_flat<kLogVerify>(G, p, t, stream);
      default: return launch_flat<kVerify>(G, p, t, stream);
    }
  }
#endif
  switch (mode) {
    case kStore: return launch_mode<kStore>(G, p, t, stream);
    case kTrailer: return launch_mode<kTrailer>(G, p, t, stream);
    case kLogWrite: return launch_mode<kLogWrite>(G, p, t, stream);
    case kLogVerify: return launch_mode<kLogVerify>(G, p, t, stream);
    default: return launch_mode<kVerify>(G, p, t, stream);
  }
}

// The device's CU count for plan reports (the same value run() uses), without
// initialising the device: 256 (MI355X) when no table set exists yet.
uint32_t cus_hint() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return 256;
  }
  if (dev < 0 || dev >= kMaxDevices || g_dev[dev].cus <= 0) return 256;
  return (uint32_t)g_dev[dev].cus;
}

}  // namespace

extern "C" {

int nova_crc32c_abi_version(void) { return 2; }

int nova_device_init(void) {
  int err = 0;
  return tables(&err) ? 0 : err;
}

int nova_stream_release(void* stream) {
  int err = 0;
  DevTables* t = tables(&err);
  if (!t) return err;
  return sched_release_stream(t, (hipStream_t)stream);
}

size_t nova_stream_slots(void) {
  int err = 0;
  DevTables* t = tables(&err);
  return t ? sched_slots(t) : 0;
}

int nova_crc32c_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                      const uint32_t* init_or_null, uint32_t* out_crc, size_t n_blocks,
                      uint32_t flags, void* stream) {
  if (n_blocks && (!base || !offsets || !lengths || !out_crc)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)base;
  p.offsets = offsets;
  p.lengths = lengths;
  p.flags = flags;
  p.init = init_or_null;
  p.out = out_crc;
  p.n_blocks = n_blocks;
  return run(kStore, p, false, 0, (hipStream_t)stream);
}

int nova_crc32c_batch_strided(const void* base, uint64_t stride, uint32_t len, size_t n_blocks,
                              const uint32_t* init_or_null, uint32_t* out_crc, uint32_t flags,
                              void* stream) {
  if (n_blocks && (!base || !out_crc)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)base;
  p.stride = stride;
  p.len = len;
  p.flags = flags;
  p.init = init_or_null;
  p.out = out_crc;
  p.n_blocks = n_blocks;
  return run(kStore, p, true, len, (hipStream_t)stream);
}

int nova_sstable_write_trailers(void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                size_t n_blocks, uint32_t flags, void* stream) {
  if (n_blocks && (!buf || !offsets || !sizes)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)buf;
  p.offsets = offsets;
  p.lengths = sizes;
  p.flags = (flags & (0xff00u | NOVA_TRAILER_TB_QUIRK | NOVA_CRC32C_HINT_LARGE_BLOCKS)) |
            NOVA_CRC32C_APPEND_TYPE;
  p.n_blocks = n_blocks;
  return run(kTrailer, p, false, 0, (hipStream_t)stream);
}

int nova_sstable_verify_blocks_ex(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                  size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out,
                                  uint32_t flags, void* stream) {
  if (n_blocks && (!buf || !offsets || !sizes || !ok_out)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)buf;
  p.offsets = offsets;
  p.lengths = sizes;
  p.ok_out = ok_out;
  p.n_bad = n_bad_out;
  p.n_blocks = n_blocks;
  p.flags = flags & NOVA_CRC32C_HINT_LARGE_BLOCKS;
  return run(kVerify, p, false, 0, (hipStream_t)stream);
}

int nova_sstable_verify_blocks(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                               size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out,
                               void* stream) {
  return nova_sstable_verify_blocks_ex(buf, offsets, sizes, n_blocks, ok_out, n_bad_out, 0u, stream);
}

int nova_log_write_crcs(void* buf, size_t buf_len, const uint64_t* record_offsets,
                        size_t n_records, void* stream) {
  if (n_records && (!buf || !record_offsets)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)buf;
  p.buf_len = buf_len;
  p.offsets = record_offsets;
  p.n_blocks = n_records;
  return run(kLogWrite, p, false, 0, (hipStream_t)stream);
}

int nova_log_verify_records(const void* buf, size_t buf_len, const uint64_t* record_offsets,
                            size_t n_records, uint8_t* ok_out, uint32_t* n_bad_out, void* stream) {
  if (n_records && (!buf || !record_offsets || !ok_out)) return NOVA_E_INVAL;
  CrcParams p{};
  p.base = (const uint8_t*)buf;
  p.buf_len = buf_len;
  p.offsets = record_offsets;
  p.ok_out = ok_out;
  p.n_bad = n_bad_out;
  p.n_blocks = n_records;
  return run(kLogVerify, p, false, 0, (hipStream_t)stream);
}

int nova_xor_parity(const void* base, const uint64_t* frag_offsets, size_t n_frags,
                    size_t parity_len, void* out, void* stream) {
  if (!parity_len) return 0;
  if (!base || !frag_offsets || !out || n_frags == 0 || n_frags > 0xffffffffu) return NOVA_E_INVAL;
  int err = 0;
  DevTables* t = tables(&err);
  if (!t) return err;
  // variant: U (chunks per thread) x FU (fragments loaded together), grid cap
  // in workgroups per CU; default from the sweep in profiles.
  const int v = g_tune_parity.load();
  const int u = (v & 0xf) ? (v & 0xf) : 2;  // sweep (profiles/r01_parity_sweep.log): 2 x 1
  const int fu = ((v >> 4) & 0xf) ? ((v >> 4) & 0xf) : 1;  // x 8/CU best (71%), 4 x 2: 57%
  const int per_cu = ((v >> 8) & 0xff) ? ((v >> 8) & 0xff) : 8;
  uint64_t chunks = (parity_len + 15) / 16;
  uint64_t wgs = (chunks + 256 * (uint64_t)u - 1) / (256 * (uint64_t)u);
  const uint64_t cap = (uint64_t)t->cus * per_cu;
  if (wgs > cap) wgs = cap;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)base;
  const uint32_t nf = (uint32_t)n_frags;
  const uint64_t pl = (uint64_t)parity_len;
  uint8_t* o = (uint8_t*)out;
#define NOVA_XP(U_, FU_)                                                                      \
  if (u == U_ && fu == FU_) {                                                                 \
    hipLaunchKernelGGL((xor_parity_kernel<U_, FU_>), dim3(wgs), dim3(256), 0, st, b, frag_offsets, nf, pl, o); \
    return (int)hipGetLastError();                                                            \
  }
  NOVA_XP(1, 1) NOVA_XP(2, 1) NOVA_XP(4, 1) NOVA_XP(4, 2) NOVA_XP(4, 4) NOVA_XP(2, 4) NOVA_XP(2, 2)
  NOVA_XP(8, 1) NOVA_XP(8, 2)
#undef NOVA_XP
  return NOVA_E_INVAL;
}

int nova_fill_splitmix64(void* dev, size_t nbytes, uint64_t seed, uint64_t first_word,
                         void* stream) {
  if (!dev && nbytes) return NOVA_E_INVAL;
  if (!nbytes) return 0;
  uint64_t blocks = (nbytes / 8 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(fill_splitmix64_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)dev, (uint64_t)nbytes, seed, first_word);
  return (int)hipGetLastError();
}

int nova_crc32c_plan(size_t n_blocks, uint64_t bytes_per_block, int* lanes_per_unit,
                     uint32_t* seg_bytes) {
  // Plan for an aligned fixed-stride batch of bytes_per_block blocks.
  CrcParams p{};
  p.base = reinterpret_cast<const uint8_t*>(uintptr_t(256));
  p.len = (uint32_t)bytes_per_block;
  p.stride = bytes_per_block;
  p.n_blocks = n_blocks;
  if (split_wanted(kStore, p, true, bytes_per_block)) {
    uint32_t S = 0, ks = 0;
    split_shape(n_blocks, true, bytes_per_block, &S, &ks);
    if (lanes_per_unit) *lanes_per_unit = 0;
    if (seg_bytes) *seg_bytes = S;
    return 5;  // split and combine (pieces of S bytes)
  }
  if (const int bg = burst_lanes(kStore, n_blocks, cus_hint())) {
    if (lanes_per_unit) *lanes_per_unit = bg;
    if (seg_bytes) *seg_bytes = 0;
    return 4;  // burst kernel
  }
  const int sg = g_tune_seg.load() ? 0 : stream_lanes(p);
  if (sg) {
    if (lanes_per_unit) *lanes_per_unit = sg;
    if (seg_bytes) *seg_bytes = 0;
    return 1;  // streaming kernel
  }
  const Plan pl = plan(n_blocks, bytes_per_block, true, kStore, false, cus_hint());
  if (lanes_per_unit) *lanes_per_unit = pl.G;
  if (seg_bytes) *seg_bytes = pl.seg;
  return pl.kernel == kFlatK ? 2 : pl.kernel == kRoundsK ? 3 : 0;  // flat : rounds : units
}

int nova_crc32c_describe(size_t n_blocks, uint64_t len, uint64_t stride, int variable, char* buf,
                         size_t buflen) {
  CrcParams p{};
  p.base = reinterpret_cast<const uint8_t*>(uintptr_t(256));
  p.len = (uint32_t)len;
  p.stride = stride;
  p.n_blocks = n_blocks;
  int sg = 0;
  if (!variable && !g_tune_seg.load()) sg = stream_lanes(p);
  int n;
  if (variable == 0 || variable == 2) {
    p.flags = variable == 2 ? NOVA_CRC32C_HINT_LARGE_BLOCKS : 0u;
    if (split_wanted(kStore, p, variable == 0, len)) {
      uint32_t S = 0, ks = 0;
      split_shape(n_blocks, variable == 0, len, &S, &ks);
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"split\", \"piece_bytes\": %u, \"slots_per_block\": %u, "
                   "\"pieces\": \"%s\"}", S, 1u << ks,
                   S >= 16384 ? "crc32c_units_kernel<16, 0>" : "crc32c_rounds_kernel");
      return n;
    }
  }
  const int bg = variable == 3 ? 0 : burst_lanes(kStore, n_blocks, cus_hint());
  if (bg) {
    n = snprintf(buf, buflen,
                 "{\"kernel\": \"crc32c_burst_kernel<%d, 0>\", \"lanes_per_block\": %d, "
                 "\"swaths_per_pass\": %d}", bg, bg,
                 bg == 16 ? 16 : BurstCfg<64>::kK);
  } else if (sg) {
    n = snprintf(buf, buflen,
                 "{\"kernel\": \"crc32c_stream_kernel<%d, 0>\", \"lanes_per_block\": %d, "
                 "\"blocks_per_group\": %u, \"steal_probes\": %d}",
                 sg, sg, stream_bpg(sg, (uint32_t)len),
                 g_tune_static_pct.load() < 0 ? 8 : g_tune_static_pct.load());
  } else {
    const bool log = variable == 3;
    const int mode = log ? kLogWrite : kStore;
    const Plan pl = plan(n_blocks, len, !variable, mode, variable == 2, cus_hint());
    const int g = pl.G < 2 ? 2 : pl.G;
    // the chunk launch_rounds() runs when plan() leaves it to the default
    const uint32_t def_chunk = log ? 64u : 4u * (64u / (uint32_t)g);
    if (pl.kernel == kRoundsK)
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"crc32c_rounds_kernel<%d, %d>\", \"lanes_per_block\": %d, "
                   "\"sort\": %d, \"waves_per_wg\": %d, \"chunk_blocks\": %u}", g, mode,
                   g, g_tune_sort.load(), (int)flat_waves(), pl.chunk ? pl.chunk : def_chunk);
#ifdef NOVA_DIAG
    else if (pl.kernel == kFlatK)
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"crc32c_flat_kernel<%d, %d>\", \"lanes_per_block\": %d, "
                   "\"chunk_blocks\": %u, \"waves_per_wg\": %d}", pl.G, mode, pl.G,
                   flat_chunk(pl.G, mode), (int)flat_waves());
#endif
    else
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"crc32c_units_kernel<%d, %d>\", \"lanes_per_unit\": %d, "
                   "\"segment_bytes\": %u, \"waves_per_wg\": %d}", pl.G, mode, pl.G, pl.seg,
                   waves_per_wg(kUnitsWaves));
  }
  return n;
}

const char* nova_crc32c_kernel_name(int lanes_per_unit) {
  switch (lanes_per_unit) {
    case 1: return "crc32c_units_kernel<1, 0>";
    case 2: return "crc32c_units_kernel<2, 0>";
    case 4: return "crc32c_units_kernel<4, 0>";
    case 8: return "crc32c_units_kernel<8, 0>";
    case 16: return "crc32c_units_kernel<16, 0>";
    default: return "crc32c_units_kernel";
  }
}

void nova_crc32c_set_tuning(int lanes_per_unit, uint32_t seg_bytes) {
  g_tune_g.store(lanes_per_unit);
  g_tune_seg.store(seg_bytes);
}

#ifdef NOVA_DIAG
void nova_diag_set_variant(int variant) { g_tune_var.store(variant); }

void nova_diag_set_stamps(uint64_t* dev_stamps) { g_diag_stamps.store(dev_stamps); }

void nova_diag_set_static_pct(int pct) { g_tune_static_pct.store(pct); }

void nova_diag_set_blocks_per_group(int bpg) { g_tune_bpg.store(bpg); }

void nova_diag_set_chunk_blocks(int blocks) { g_tune_chunk.store(blocks); }

void nova_diag_set_stream_waves(int waves) { g_tune_waves.store(waves); }

void nova_diag_set_variable_kernel(int kernel) { g_tune_kernel.store(kernel); }

void nova_diag_set_parity_variant(int variant) { g_tune_parity.store(variant); }

void nova_diag_set_rounds_sort(int on) { g_tune_sort.store(on); }

void nova_diag_set_trailer_single_pass(int on) { g_tune_trailer_1pass.store(on); }

void nova_diag_set_burst_lanes(int lanes) { g_tune_burst.store(lanes); }
void nova_diag_set_split(int on) { g_tune_split.store(on); }

int nova_diag_read_stream(const void* base, size_t bytes, uint32_t* out_dev, int wgs,
                          void* stream) {
  if (!base || !out_dev || wgs <= 0) return NOVA_E_INVAL;
  hipLaunchKernelGGL(read_stream_kernel, dim3(wgs), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)base, (uint64_t)(bytes / 16), out_dev);
  return (int)hipGetLastError();
}

int nova_diag_read_ceiling(const void* base, size_t bytes, uint32_t* out_dev, int wgs,
                           int variant, void* stream) {
  if (!base || !out_dev || wgs <= 0) return NOVA_E_INVAL;
  const int u = variant & 0xff;
  const bool nt = (variant & 0x100) != 0;
  const int threads = (variant & 0x200) ? 1024 : 256;
  const uint8_t* b = (const uint8_t*)base;
  const uint64_t n16 = bytes / 16;
  hipStream_t st = (hipStream_t)stream;
#define NOVA_RC(U)                                                                        \
  if (u == U) {                                                                           \
    if (nt) hipLaunchKernelGGL((read_ceiling_kernel<U, 1>), dim3(wgs), dim3(threads), 0, st, b, n16, out_dev); \
    else hipLaunchKernelGGL((read_ceiling_kernel<U, 0>), dim3(wgs), dim3(threads), 0, st, b, n16, out_dev);   \
    return (int)hipGetLastError();                                                        \
  }
  NOVA_RC(2) NOVA_RC(4) NOVA_RC(8) NOVA_RC(16)
#undef NOVA_RC
  return NOVA_E_INVAL;
}

#endif  // NOVA_DIAG

const char* nova_error_string(int err) {
  switch (err) {
    case 0: return "success";
    case NOVA_E_INVAL: return "invalid argument";
    case NOVA_E_NODEV: return "no usable HIP device";
    case NOVA_E_NOMEM: return "allocation failed";
    default: return hipGetErrorString((hipError_t)err);
  }
}

}  // extern "C"
