// MI355X (gfx950) batched CRC-32C -- the product translation unit: the
// non-template kernels (XOR parity, split and combine, synthetic fill), the
// per-device tables, the dispatcher and the C-ABI batch entry points.  Drop-in
// for the per-SSTable-block checksum of NovaLSM (util/crc32c.cc:487-588 called
// from table/table_builder.cc:202-204, ltc/stoc_file_client_impl.cpp:713-719
// and table/table.cc:434-440).  The algorithm and the kernels that carry it
// are in crc32c_kernels.hpp; experiments and timing ablations live in
// crc32c_diag.hip (diagnostics library only), reached through g_diag.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "crc32c_kernels.hpp"
#include "gf2_crc32c.hpp"

namespace {

// (xor_parity_kernel: crc32c_kernels.hpp, shared with the diagnostics TU's A/B forms)



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

// ---- log records: windowed sort by line count ---------------
// The rounds kernel pads a round's kGroups records to the longest; sorting each
// claimed chunk of 64 records leaves ~21 % of the loaded step capacity as
// padding on U[1,4096] B records (tools/sim_rounds.py).  This pre-pass sorts
// windows of consecutive records (~512 KiB of log, log_sort_window(), so a
// chunk's records stay close together in memory) by line count, largest first,
// into perm[]; the kernel then takes chunks of that order.  The key comes from
// the offsets alone -- record i's length is at most the gap to the next
// record's header or to its 32 KiB block's end -- so the pre-pass reads 8 B
// per record and no header byte; a wrong estimate (unsorted offsets, a block
// trailer) only costs padding, never a wrong CRC.  One workgroup per window,
// counting sort in LDS (order within a line count is arbitrary).
constexpr uint32_t kLogSortWin = 1024;  // records per window (at most; g_tune_logwin)
constexpr uint32_t kLogSortBins = 288;  // line counts (a 32 KiB log block is 256 lines of 128 B)
// keymode (diagnostics A/B, nova_diag_set_log_key; product 0): 0 counting
// sort by line count, order within a count arbitrary; 1 the same, stable
// (file order within a count); 2 / 3 stable on the line count / 2 or / 4.
__global__ void __launch_bounds__(256) log_sort_kernel(uint64_t base, const uint64_t* __restrict__ offs,
                                                       uint64_t n, uint64_t buf_len, uint32_t line,
                                                       uint32_t win, uint32_t* __restrict__ perm,
                                                       uint32_t keymode) {
  __shared__ uint32_t cnt[kLogSortBins];
  __shared__ uint16_t kk[kLogSortWin];  // keymode > 0: every record's key, for the stable ranks
  // blockDim.x threads (64-256, log_sort_threads) take win / blockDim.x records each
  const uint32_t nt = blockDim.x;
  const uint64_t w0 = (uint64_t)blockIdx.x * win;
  for (uint32_t b = threadIdx.x; b < kLogSortBins; b += nt) cnt[b] = 0;
  __syncthreads();
  constexpr int kPer = kLogSortWin / 64;
  uint32_t key[kPer];
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint32_t j = threadIdx.x + nt * k;
    const uint64_t i = w0 + j;
    key[k] = 0;
    if (j < win && i < n) {
      const uint64_t o = offs[i];
      const uint64_t be = log_block_end(o, buf_len);
      uint64_t e = i + 1 < n ? offs[i + 1] : be;
      if (e > be || e < o) e = be;
      const uint64_t u0 = base + o + 6, u1 = base + (e > o + 7 ? e : o + 7);  // CRC input [u0, u1)
      const uint64_t E = u1 & ~15ull;
      const uint64_t first = (u0 & ~15ull) & ~(uint64_t)(line - 1);
      const uint64_t Le = (E + line - 1) & ~(uint64_t)(line - 1);
      const uint64_t S = Le > first ? (Le - first) / line : 1;  // lines (the rounds kernel's cost)
      key[k] = S < kLogSortBins ? (uint32_t)S : kLogSortBins - 1;
      if (keymode >= 2) key[k] >>= keymode - 1;
      atomicAdd(&cnt[key[k]], 1u);
      if (keymode) kk[j] = (uint16_t)key[k];
    }
  }
  __syncthreads();
  // Exclusive prefix in descending key order, by wave 0: lane l sums the
  // reversed bins [5l, 5l + 5) (320 >= kLogSortBins), one wave scan of those
  // sums, then it writes its five bins' starts.  (One thread walking the 288
  // bins was half the kernel's time: tools/logsort_probe.hip,
  // profiles/r06_logsort_probe.log.)
  static_assert(5 * 64 >= kLogSortBins, "five bins per lane");
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x;
    uint32_t c[5], sum = 0;
#pragma unroll
    for (int q = 0; q < 5; q++) {
      const int r = (int)(5 * l) + q;
      c[q] = r < (int)kLogSortBins ? cnt[kLogSortBins - 1 - r] : 0u;
      sum += c[q];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d);
      if ((int)l >= d) incl += o;
    }
    uint32_t run = incl - sum;
#pragma unroll
    for (int q = 0; q < 5; q++) {
      const int r = (int)(5 * l) + q;
      if (r < (int)kLogSortBins) cnt[kLogSortBins - 1 - r] = run;
      run += c[q];
    }
  }
  __syncthreads();
  if (keymode) {  // stable: rank = the bin's start + earlier records of the same key
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t j = threadIdx.x + nt * k;
      const uint64_t i = w0 + j;
      if (j < win && i < n) {
        uint32_t r = cnt[key[k]];
        for (uint32_t x = 0; x < j; x++) r += kk[x] == key[k] ? 1u : 0u;
        perm[w0 + r] = (uint32_t)i;
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint32_t j = threadIdx.x + nt * k;
    const uint64_t i = w0 + j;
    if (j < win && i < n) perm[w0 + atomicAdd(&cnt[key[k]], 1u)] = (uint32_t)i;
  }
}

// The sorted records ran position-indexed (kVarOutPos): per window, move each
// record's result from its position to the record, in record order -- verify:
// its status byte into status_out[i]; write: Mask(crc) into the header's CRC
// field when its status is OK (db/log_writer.cc:113).  Storing from the CRC
// kernel in sorted order scattered a window's stores over time and over 1 MiB
// of image (log write 52 % vs 63 % without the stores); here a
// window's stores issue together, in file order, and the status lines are
// written whole.
__global__ void __launch_bounds__(256) log_unperm_kernel(uint8_t* base, const uint64_t* __restrict__ offs,
                                                         uint64_t n, const uint32_t* __restrict__ perm,
                                                         const uint8_t* __restrict__ st_pos,
                                                         const uint32_t* __restrict__ crc_pos,
                                                         uint8_t* __restrict__ status_out, uint32_t win) {
  __shared__ uint16_t inv[kLogSortWin];
  const uint64_t w0 = (uint64_t)blockIdx.x * win;
  const uint32_t m = n - w0 < win ? (uint32_t)(n - w0) : win;
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) inv[perm[w0 + j] - w0] = (uint16_t)j;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
    const uint64_t pos = w0 + inv[j];
    const uint8_t st = st_pos[pos];
    if (status_out)
      status_out[w0 + j] = st;
    else if (st == NOVA_LOG_OK)
      store_u32_unaligned(base + offs[w0 + j], crc_pos[pos]);
  }
}

// ---- trailer writer: CRC pass, then whole-piece trailer stores
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
//   last (may be null): blocks that are never eligible (the first and last
//   block of each table of a coalesced batch: their windows may reach another
//   caller's memory, crc32c_queue.hip).
__global__ void __launch_bounds__(256) trailer_layout_kernel(uint64_t ba, const uint64_t* offsets,
                                                             uint64_t omask, const uint32_t* lengths,
                                                             uint64_t lmask, uint64_t stride,
                                                             uint32_t len, uint64_t n, uint32_t* elig,
                                                             uint32_t* flag, const uint8_t* last) {
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
    if (last) e = e && !last[i];
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


}  // namespace

// ---- shared state (crc32c_internal.hpp) -------------------------------------
namespace nova_dev {

thread_local std::atomic<int> g_tune_g{0};
thread_local std::atomic<uint32_t> g_tune_seg{0};
thread_local std::atomic<int> g_tune_static_pct{-1};
thread_local std::atomic<int> g_tune_var{0};
thread_local std::atomic<int> g_tune_bpg{0};
thread_local std::atomic<int> g_tune_chunk{0};
thread_local std::atomic<int> g_tune_waves{0};
thread_local std::atomic<int> g_tune_parity{0};
thread_local std::atomic<int> g_tune_kernel{0};
thread_local std::atomic<int> g_tune_sort{2};
thread_local std::atomic<int> g_tune_logwin{0};
thread_local std::atomic<int> g_tune_logkey{0};  // log_sort_kernel keymode (diagnostics)
thread_local std::atomic<int> g_tune_trailer_1pass{0};
thread_local std::atomic<int> g_tune_burst{0};
thread_local std::atomic<int> g_tune_split{0};
thread_local std::atomic<uint64_t*> g_diag_stamps{nullptr};
DiagHooks* g_diag = nullptr;

int waves_per_wg(int def) {
  const int w = g_tune_waves.load();
  return (w > 0 && w <= kWaves) ? w : def;
}

}  // namespace nova_dev

namespace {
using namespace nova_dev;

DevTables g_dev[kMaxDevices];
std::once_flag g_once[kMaxDevices];


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


void init_device(int dev, DevTables* t) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) { t->err = (int)e; return; }
  t->cus = prop.multiProcessorCount;
  {  // the scratch pool (DevTables::pool); without it scratch uses hipMallocAsync
    hipMemPoolProps pp{};
    pp.allocType = hipMemAllocationTypePinned;
    pp.handleTypes = hipMemHandleTypeNone;
    pp.location.type = hipMemLocationTypeDevice;
    pp.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &pp) == hipSuccess) {
      uint64_t keep = 512ull << 20;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      t->pool = pool;
    } else {
      (void)hipGetLastError();
    }
  }
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
  if ((t->err = upload(&t->zero_word, std::vector<uint32_t>(256, 0u)))) return;  // 1 KiB of zeros
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
  }
  if ((t->err = set_lds_attrs_rounds<kStore>())) return;
  if ((t->err = set_lds_attrs_rounds<kStore, kVarInit>())) return;
  if ((t->err = set_lds_attrs_rounds<kTrailer>())) return;
  if ((t->err = set_lds_attrs_rounds<kVerify>())) return;
  if ((t->err = set_lds_attrs_rounds<kLogWrite>())) return;
  if ((t->err = set_lds_attrs_rounds<kLogVerify>())) return;
  if ((t->err = set_lds_attr_rounds<8, kLogWrite, kVarOutPos>())) return;
  if ((t->err = set_lds_attr_rounds<8, kLogVerify, kVarOutPos>())) return;
  if ((t->err = set_lds_attr_rounds<2, kLogWrite, kVarCached>())) return;  // (2 and 4 lanes only)
  if ((t->err = set_lds_attr_rounds<4, kLogWrite, kVarCached>())) return;
  if ((t->err = set_lds_attr_rounds<2, kLogVerify, kVarCached>())) return;
  if ((t->err = set_lds_attr_rounds<4, kLogVerify, kVarCached>())) return;
  if ((t->err = set_lds_attrs_mode<kStore>())) return;
  if ((t->err = set_lds_attrs_mode<kTrailer>())) return;
  if ((t->err = set_lds_attrs_mode<kVerify>())) return;
  if ((t->err = set_lds_attrs_mode<kLogWrite>())) return;
  if ((t->err = set_lds_attrs_mode<kLogVerify>())) return;
  if ((t->err = set_lds_attrs_stream<0>())) return;
  if ((t->err = set_lds_attr_burst<64, kStore>())) return;
  if ((t->err = set_lds_attr_burst<64, kTrailer>())) return;
  if ((t->err = set_lds_attr_burst<64, kVerify>())) return;
  // the diagnostics library's tables and kernel attributes
  if (g_diag && (t->err = g_diag->init_device(t))) return;
}

}  // namespace

namespace nova_dev {

int upload_u32(uint32_t** dst, const uint32_t* src, size_t n) {
  return upload(dst, std::vector<uint32_t>(src, src + n));
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
//
// Logs pass their mean record span (bytes per record) as bytes_per_block.
// Short records run in narrower lane groups: more records per round, fewer
// padded steps per record.  Groups of 2 and 4 lanes load their records with
// the default policy (launch_rounds), which keeps the lines two records share
// in L2; with it the crossovers moved (round 5, payloads U[1,256] ..
// U[1,4096] B, % of 8 TB/s, profiles/r05_log_lanes_cached.log):
//   mean span      135 B  263 B  391 B  520 B  775 B  1031 B  2055 B
//   write G=2/4/8  25/22/15  38/36/26  43/43/33  44/46/37  45/49/44  45/49/48  49/52/57
//   verify G=2/4/8 26/22/14  42/38/25  47/47/33  47/50/39  48/55/50  50/57/56  52/57/66
// (round 3, nt loads: 4 lanes won below ~1 KiB for verify and only below
// ~400 B for write, profiles/r03_log_lanes_sweep.log).
constexpr uint64_t kLogNarrowVerify = 1280;  // 4 lanes below
constexpr uint64_t kLogNarrowWrite = 1280;
constexpr uint64_t kLogPairVerify = 420;  // 2 lanes below
constexpr uint64_t kLogPairWrite = 350;
Plan plan(uint64_t n_blocks, uint64_t bytes_per_block, bool uniform, int mode, bool large,
          uint32_t cus) {
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
  if (pl.kernel == kRoundsK && log && tk == kAuto && tg == 0 && bytes_per_block &&
      bytes_per_block < (mode == kLogVerify ? kLogNarrowVerify : kLogNarrowWrite)) {
    // short records: 4-lane groups, or 2 (log verify then runs without the pre-sort)
    pl.G = bytes_per_block < (mode == kLogVerify ? kLogPairVerify : kLogPairWrite) ? 2 : 4;
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

}  // namespace nova_dev

namespace {

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


// ---- product launches (the diagnostics library may take them over) ----------
template <int MODE>
int launch_mode(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
  int rc = 0;
  if (g_diag && g_diag->units(MODE, G, p, t, stream, &rc)) return rc;
  return launch_units_v<MODE, 0>(G, p, t, stream);
}

// p.perm: null, or the order to take the blocks in (log records: log_sort_kernel).
template <int MODE>
int launch_rounds(int G, CrcParams& p, DevTables* t, hipStream_t stream, uint32_t chunk = 0) {
  int rc = 0;
  if (g_diag && g_diag->rounds(MODE, G, p, t, stream, chunk, &rc)) return rc;
  if constexpr (MODE == kLogWrite || MODE == kLogVerify) {
    if (p.out_pos) return launch_rounds_v<MODE, kVarOutPos>(G, p, t, stream, chunk);
    // Short records (G <= 4 lanes each) share their first and last lines with
    // their neighbours, which the same wave reads in the same chunk: default-
    // policy loads keep those lines in L2 for the second reader (same-box A/B,
    // profiles/r05_log_cached_ab.log: log512 write 27.9 -> 36.7 %, verify
    // 36.8 -> 37.7 %; log4k at G = 8 loses 3-7 points with them and stays nt).
    if (G <= 4) return launch_rounds_v<MODE, kVarCached>(G, p, t, stream, chunk);
  }
  if (MODE == kStore && p.init)  // per-block init values: the general head masking
    return launch_rounds_v<kStore, kVarInit>(G, p, t, stream, chunk);
  return launch_rounds_v<MODE, 0>(G, p, t, stream, chunk);
}

int launch_stream(int G, CrcParams& p, DevTables* t, hipStream_t stream) {
  int rc = 0;
  if (g_diag && g_diag->stream(G, p, t, stream, &rc)) return rc;
  return launch_stream_v<0>(G, p, t, stream);
}

// SSTable-block batches up to 4 blocks per wave slot of the rounds kernel
// (12288 on 256 CUs x 12 waves) go to the burst kernel, one wave per block on
// the compact tables, unless tuning forces a kernel.  The
// crossover (tools/latency_burst.py, profiles/r03_latency_burst_mid.log): 8192
// blocks 26.1 us burst vs 34.4 us rounds, 16384 blocks 39.4 vs 35.4 us.
uint64_t burst_max(uint32_t cus) { return 4ull * cus * flat_waves(); }
int burst_lanes(int mode, uint64_t n_blocks, uint32_t cus) {
  if (mode != kStore && mode != kTrailer && mode != kVerify) return 0;
  const int tb = g_tune_burst.load();
  if (tb < 0) return 0;
  if (tb == 16 || tb == 64 || tb == 65) return tb;
  if (g_tune_g.load() || g_tune_seg.load() || g_tune_kernel.load()) return 0;
  return n_blocks <= burst_max(cus) ? 64 : 0;
}


template <int MODE>
int launch_burst_g(int V, CrcParams& p, DevTables* t, hipStream_t stream) {
  int rc = 0;
  if (g_diag && g_diag->burst(V, MODE, p, t, stream, &rc)) return rc;
  return launch_burst_v<64, MODE>(p, t, stream);
}


constexpr uint64_t kLogSortMin = 1u << 16;  // records: the log_sort_kernel pre-pass from here
constexpr uint64_t kTrailerTwoPassMin = 1u << 18;  // blocks: the trailer writer's two passes from here
// Records per sort window: the power of two nearest to ~512 KiB of log.  A wider
// window cuts more round padding but spreads a chunk's reads over more of the
// image; measured over payloads U[1,512] .. U[1,16384] B the best window spanned
// 0.25-1 MiB, and a fixed 512 records lost up to 15 points on large records
// (profiles/r03_logsort_sweep6.log).
// Threads per log_sort_kernel workgroup: a quarter of the window, 64 to 256
// (one wave takes four records per lane of a 256-record window).
// tools/logsort_probe.hip on 2M records in 8K windows: 36.6-36.9 us with 256
// threads and one thread's prefix, 28.7-29.1 with 64 threads, 16.9-17.2 with
// the wave's prefix, 13.1-13.3 with both (profiles/r06_logsort_probe.log); in
// the log4k verify line 30.8 -> 14.2 us.  (log_unperm_kernel at 64 threads
// measured the same 7.2-7.4 us and keeps 256.)
uint32_t log_sort_threads(uint32_t win) {
  const uint32_t t = win / 4;
  return t < 64 ? 64u : (t > 256 ? 256u : t);
}

uint32_t log_sort_window(uint64_t n, uint64_t bytes) {
  const uint64_t avg = n && bytes / n ? bytes / n : 1;
  const uint64_t w = (512u * 1024u) / avg;
  uint32_t win = 64;
  while (win < kLogSortWin && w >= win + win / 2) win *= 2;
  return win;
}

}  // namespace

namespace nova_dev {

int trailer_layout(const CrcParams& p, DevTables* t, hipStream_t stream, uint32_t* elig, uint32_t* flag) {
  hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), stream);
  if (e != hipSuccess) return (int)e;
  uint64_t wgs = (p.n_blocks + 255) / 256;
  const uint64_t cap = (uint64_t)t->cus * 8;
  if (wgs > cap) wgs = cap;
  // descriptors as the rounds kernel normalises them (absent arrays: stride / len)
  const uint64_t* lo = p.offsets ? p.offsets : reinterpret_cast<const uint64_t*>(t->zero_word);
  const uint32_t* ll = p.lengths ? p.lengths : t->zero_word;
  hipLaunchKernelGGL(trailer_layout_kernel, dim3(wgs), dim3(256), 0, stream, (uint64_t)p.base, lo,
                     p.offsets ? ~0ull : 0ull, ll, p.lengths ? ~0ull : 0ull, p.offsets ? 0ull : p.stride,
                     p.lengths ? 0u : p.len, p.n_blocks, elig, flag, p.tr_last);
  return (int)hipGetLastError();
}

// The trailer writer on rounds-kernel batches (round 3).  Storing the 5-B
// trailers from the CRC kernel cost ~16 points of HBM throughput on NovaLSM's
// block shape (partial 64-B pieces, each a read-modify-write at the memory,
// interleaved with the read stream); the CRC pass instead writes one word per
// block into a stream-ordered array, and trailer_rmw_kernel then rewrites the
// whole 64-B piece(s) holding each trailer (profiles/r03_ops_batchepi.log:
// 66 % -> 72 %).  Without scratch: the one-pass form.
int trailer_two_pass(CrcParams& p, int G, uint32_t chunk, DevTables* t, hipStream_t stream) {
  StreamScratch sc;  // flag, eligibility, CRCs; freed in stream order after the second pass
  if (sc.alloc(sizeof(uint32_t) * (2 * p.n_blocks + 1), stream))
    return launch_rounds_v<kTrailer, 0>(G, p, t, stream, chunk);
  uint32_t* flag = static_cast<uint32_t*>(sc.p);
  uint32_t* elig = flag + 1;
  uint32_t* tmp = elig + p.n_blocks;
  int e = trailer_layout(p, t, stream, elig, flag);
  if (e) return e;
  CrcParams q = p;
  q.out = tmp;
  q.flags = (p.flags & 0xff00u) | NOVA_CRC32C_APPEND_TYPE | NOVA_CRC32C_MASK_OUTPUT;
  if ((e = launch_rounds_v<kStore, 0>(G, q, t, stream, chunk))) return e;
  const uint64_t cap = (uint64_t)t->cus * 8;
  uint64_t wgs8 = (p.n_blocks * 8 + 255) / 256;
  if (wgs8 > cap) wgs8 = cap;
  const uint64_t* lo = p.offsets ? p.offsets : reinterpret_cast<const uint64_t*>(t->zero_word);
  const uint32_t* ll = p.lengths ? p.lengths : t->zero_word;
  hipLaunchKernelGGL(trailer_rmw_kernel, dim3(wgs8), dim3(256), 0, stream, const_cast<uint8_t*>(p.base), lo,
                     p.offsets ? ~0ull : 0ull, ll, p.lengths ? ~0ull : 0ull, p.offsets ? 0ull : p.stride,
                     p.lengths ? 0u : p.len, tmp, elig, flag, p.n_blocks, p.flags);
  return (int)hipGetLastError();
}

}  // namespace nova_dev

namespace {

// Few large blocks -> the split-and-combine path (split_*_kernel): uniform
// blocks over kBurstMaxLen in a batch of at most kSplitMaxBlocks, or a batch of
// at most kSplitMaxHinted blocks the caller marks HINT_LARGE_BLOCKS (the host
// does not see variable lengths; read-verify takes the hint through
// nova_sstable_verify_blocks_ex).  tools/big_blocks.py measures both sides.
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
  // the resident engine, if any, leaves the CUs to this call (crc32c_engine.hip)
  EngineYield yield_engine(stream);
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
  {
    int rc = 0;
    if (g_diag && g_diag->run_early(mode, p, t, stream, &rc)) return rc;
  }
  if (mode == kStore && uniform && !g_tune_seg.load()) {
    const int sg = stream_lanes(p);
    if (sg) return launch_stream(sg, p, t, stream);
  }
  const Plan pl = plan(p.n_blocks, bytes_per_block, uniform, mode,
                       (p.flags & NOVA_CRC32C_HINT_LARGE_BLOCKS) != 0, (uint32_t)t->cus);
  const int G = pl.G;
  p.seg = pl.seg;
  // Trailers and log CRC fields are stored by the CRC kernel itself (byte
  // stores).  The image writes cost ~13 points on SSTable-like images whatever
  // their form -- two passes, whole 64-B pieces, non-temporal -- while the
  // same kernels without the writes run at the verify rate;
  // those forms are measured experiments of the diagnostics library.
  {
    int rc = 0;
    if (g_diag && g_diag->run_planned(mode, p, pl, t, stream, &rc)) return rc;
  }
  // Large logs: records in step-count order (log_sort_kernel), results by
  // position, then log_unperm_kernel (small logs are latency-bound: two more
  // launches would add their fixed cost).  Without scratch the records run
  // unsorted (each claimed chunk still sorts itself).
  StreamScratch log_sc;  // order + position-indexed results, freed in stream order
  const int lsort = g_tune_sort.load();  // 2 default; 3-5 diagnostics A/B (crc32c_internal.hpp)
  // Log write stays in file order: every write-side sort form measured at or
  // below file order (profiles/r03_ops_logsort3.log) -- its CRC-field stores
  // cost ~7 points even in file order and more out of it; the
  // sort is a diagnostics option there.
  const bool lsort_mode = mode == kLogVerify || (mode == kLogWrite && g_diag && g_tune_logwin.load() < 0);
  // (diagnostics A/B, round 6: short records at 2-4 lanes in sorted windows
  // when a window is set, nova_diag_set_log_window)
  const bool lsort_g = G == 8 || (g_diag && G <= 4 && g_tune_logwin.load() != 0);
  if (pl.kernel == kRoundsK && lsort_mode && lsort_g &&
      p.n_blocks >= kLogSortMin && p.n_blocks < (1ull << 32) && lsort >= 2 &&
      !log_sc.alloc(p.n_blocks * (mode == kLogWrite ? 9 : 5), stream)) {
    const uint64_t n = p.n_blocks;
    const int tw = g_tune_logwin.load() < 0 ? -g_tune_logwin.load() : g_tune_logwin.load();
    const uint32_t win = (tw > 0 && tw <= (int)kLogSortWin) ? (uint32_t)tw : log_sort_window(n, p.buf_len);
    const bool by_pos = lsort == 2 || lsort == 3;
    uint32_t* perm = static_cast<uint32_t*>(log_sc.p);
    uint32_t* crc_pos = perm + n;  // log write only
    uint8_t* st_pos = reinterpret_cast<uint8_t*>(mode == kLogWrite ? crc_pos + n : perm + n);
    const uint64_t wgs = (n + win - 1) / win;
    const int km = g_diag ? g_tune_logkey.load() : 0;
    hipLaunchKernelGGL(log_sort_kernel, dim3(wgs), dim3(log_sort_threads(win)), 0, stream, (uint64_t)p.base, p.offsets, n,
                       (uint64_t)p.buf_len, 16u * (uint32_t)G, win, perm, (uint32_t)(km >= 0 && km <= 3 ? km : 0));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    CrcParams q = p;
    q.perm = perm;
    uint8_t* status_out = p.ok_out;  // verify: the caller's status array
    if (by_pos) {
      q.out_pos = 1;
      q.out = crc_pos;
      q.ok_out = st_pos;
    }
    const int rc = mode == kLogWrite ? launch_rounds<kLogWrite>(G, q, t, stream, pl.chunk)
                                     : launch_rounds<kLogVerify>(G, q, t, stream, pl.chunk);
    if (rc || !by_pos) return rc;
    hipLaunchKernelGGL(log_unperm_kernel, dim3(wgs), dim3(256), 0, stream, const_cast<uint8_t*>(p.base),
                       p.offsets, n, perm, st_pos, crc_pos, mode == kLogWrite ? nullptr : status_out, win);
    return (int)hipGetLastError();
  }
  // The trailer writer's two passes (CRC array, then whole-piece rewrite)
  // win from ~2^18 blocks; below, the CRC kernel's own trailer stores save two
  // launches and the scratch (a call waited on, sst4k blocks, events:
  // 16K blocks 33 vs 49 us, 64K 75 vs 90 us, 256K 238 vs 240 us, 1M 851 vs
  // 770 us; profiles/r04_trailer_forms_sizes_pool.log).
  if (pl.kernel == kRoundsK && mode == kTrailer && p.n_blocks >= kTrailerTwoPassMin)
    return trailer_two_pass(p, G, pl.chunk, t, stream);
  if (pl.kernel == kRoundsK) {
    switch (mode) {
      case kStore: return launch_rounds<kStore>(G, p, t, stream, pl.chunk);
      case kTrailer: return launch_rounds<kTrailer>(G, p, t, stream, pl.chunk);
      case kLogWrite: return launch_rounds<kLogWrite>(G, p, t, stream, pl.chunk);
      case kLogVerify: return launch_rounds<kLogVerify>(G, p, t, stream, pl.chunk);
      default: return launch_rounds<kVerify>(G, p, t, stream, pl.chunk);
    }
  }
  switch (mode) {
    case kStore: return launch_mode<kStore>(G, p, t, stream);
    case kTrailer: return launch_mode<kTrailer>(G, p, t, stream);
    case kLogWrite: return launch_mode<kLogWrite>(G, p, t, stream);
    case kLogVerify: return launch_mode<kLogVerify>(G, p, t, stream);
    default: return launch_mode<kVerify>(G, p, t, stream);
  }
}

}  // namespace

namespace nova_dev {
int dispatch(int mode, CrcParams& p, hipStream_t stream) { return run(mode, p, false, 0, stream); }
}  // namespace nova_dev

namespace {

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

int nova_crc32c_abi_version(void) { return 4; }

int nova_device_init(void) {
  int err = 0;
  return tables(&err) ? 0 : err;
}

int nova_stream_release(void* stream) {
  int err = 0;
  DevTables* t = tables(&err);
  if (!t) return err;
  const int rc = sched_release_stream(t, (hipStream_t)stream);
  engine_forget_stream((hipStream_t)stream);
  return rc;
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
  return run(kLogWrite, p, false, n_records ? buf_len / n_records : 0, (hipStream_t)stream);
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
  return run(kLogVerify, p, false, n_records ? buf_len / n_records : 0, (hipStream_t)stream);
}

int nova_xor_parity(const void* base, const uint64_t* frag_offsets, size_t n_frags,
                    size_t parity_len, void* out, void* stream) {
  if (!parity_len) return 0;
  if (!base || !frag_offsets || !out || n_frags == 0 || n_frags > 0xffffffffu) return NOVA_E_INVAL;
  int err = 0;
  DevTables* t = tables(&err);
  if (!t) return err;
  // variant (diagnostics knob): U (chunks per thread, bits 0-4) x FU
  // (fragments loaded together, bits 5-8), grid cap in workgroups per CU
  // (bits 9-16); 0 fields take the defaults below.
  const int v = g_tune_parity.load();
  // Default 8 chunks x 1 fragment per step over a one-pass grid (each lane's
  // 8 chunks in flight per fragment, no grid-stride loop): 79.6 %, against
  // 73.2 % for 2 x 1 and 71.1 % for the round-1 choice (2 x 1 on a grid
  // capped at 8 workgroups per CU, whose strided walk measured 52-54 % with
  // all 8 fragments' loads in flight) (profiles/r03_parity_sweep*.log).
  const int u = (v & 0x1f) ? (v & 0x1f) : 8;
  const int fu = ((v >> 5) & 0xf) ? ((v >> 5) & 0xf) : 1;
  const int per_cu = ((v >> 9) & 0xff) ? ((v >> 9) & 0xff) : 0xff;  // 0xff: no cap (one pass)
  uint64_t chunks = (parity_len + 15) / 16;
  uint64_t wgs = (chunks + 256 * (uint64_t)u - 1) / (256 * (uint64_t)u);
  const uint64_t cap = per_cu == 0xff ? (1ull << 31) - 1 : (uint64_t)t->cus * per_cu;
  if (wgs > cap) wgs = cap;
  hipStream_t st = (hipStream_t)stream;
  EngineYield yield_engine(st);
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
  NOVA_XP(8, 1) NOVA_XP(8, 2) NOVA_XP(1, 8) NOVA_XP(2, 8) NOVA_XP(1, 4) NOVA_XP(1, 2)
#undef NOVA_XP
  int rc = NOVA_E_INVAL;  // other forms: the diagnostics library's (g_diag->parity)
  if (g_diag && g_diag->parity && g_diag->parity(u, fu, b, frag_offsets, nf, pl, o, wgs, st, &rc)) return rc;
  return NOVA_E_INVAL;
}

int nova_fill_splitmix64(void* dev, size_t nbytes, uint64_t seed, uint64_t first_word,
                         void* stream) {
  if (!dev && nbytes) return NOVA_E_INVAL;
  if (!nbytes) return 0;
  uint64_t blocks = (nbytes / 8 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks == 0) blocks = 1;
  EngineYield yield_engine((hipStream_t)stream);
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
    // variable 3 / 4: log records (len = mean record span) written / verified
    const bool log = variable == 3 || variable == 4;
    const int mode = variable == 4 ? kLogVerify : log ? kLogWrite : kStore;
    const Plan pl = plan(n_blocks, len, !variable, mode, variable == 2, cus_hint());
    const int g = pl.G < 2 ? 2 : pl.G;
    // the chunk launch_rounds() runs when plan() leaves it to the default
    const uint32_t def_chunk = log ? 64u : 4u * (64u / (uint32_t)g);
    // log verify of large logs: windowed pre-sort by line count (run())
    const bool presort = mode == kLogVerify && g == 8 && n_blocks >= kLogSortMin && g_tune_sort.load() >= 2;
    if (pl.kernel == kRoundsK && presort)
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"crc32c_rounds_kernel<%d, %d>\", \"lanes_per_block\": %d, "
                   "\"sort\": %d, \"waves_per_wg\": %d, \"chunk_blocks\": %u, "
                   "\"kernels\": [\"log_sort_kernel\", \"crc32c_rounds_kernel<%d, %d>\", "
                   "\"log_unperm_kernel\"], \"sort_window\": %u}", g, mode, g, g_tune_sort.load(),
                   (int)flat_waves(), pl.chunk ? pl.chunk : def_chunk, g, mode,
                   log_sort_window(n_blocks, (uint64_t)n_blocks * len));
    else if (pl.kernel == kRoundsK)
      n = snprintf(buf, buflen,
                   "{\"kernel\": \"crc32c_rounds_kernel<%d, %d>\", \"lanes_per_block\": %d, "
                   "\"sort\": %d, \"waves_per_wg\": %d, \"chunk_blocks\": %u}", g, mode,
                   g, g_tune_sort.load(), (int)flat_waves(), pl.chunk ? pl.chunk : def_chunk);
    else if (pl.kernel == kFlatK && g_diag)
      n = g_diag->describe_flat(pl.G, mode, buf, buflen);
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

