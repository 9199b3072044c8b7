// Host-resident paths of the engine:
//   * nova_crc32c_stream_host -- BASELINE config 5: fixed-stride blocks in host
//     memory (the analogue of NovaLSM's RDMA-registered SSTable buffer,
//     backing_mem_ in ltc/stoc_file_client_impl.cpp:43-45 over nova_buf
//     registered in rdma/nova_rdma_rc_broker.cpp:31-35) stream H2D -> CRC
//     kernel -> D2H in chunks over several HIP streams so copies overlap the
//     kernels.
//   * nova_crc32c_batch_host / nova_sstable_write_trailers_host /
//     nova_sstable_verify_blocks_host -- the same for a real SSTable image:
//     variable-length blocks with 5-byte trailers, e.g. the Format() buffer
//     (ltc/stoc_file_client_impl.cpp:183-377) or the ReadAll() slab (:843-882).
//     Chunks are contiguous runs of blocks; each copies the byte span its
//     blocks cover.
//   * nova_port_accelerated_crc32c -- the reference's plug-in hook
//     port::AcceleratedCRC32C (port/port_stdcxx.h:179-189) backed by the GPU
//     for large buffers, by the host Extend otherwise and on any GPU error.
//
// The library's own HIP streams come from a per-device pool (created once,
// reused): a stream per call would also leave one claim-counter slot per
// stream address behind (crc32c_device.hip, sched_slot).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nova_crc32c.h"
#include "gf2_crc32c.hpp"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  ~DevBuf() { reset(); }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  int ensure(size_t bytes) {
    if (bytes <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
      (void)hipGetLastError();
      return NOVA_E_NOMEM;
    }
    n = bytes;
    return 0;
  }
};

struct PinBuf {
  void* p = nullptr;
  size_t n = 0;
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  PinBuf(PinBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  ~PinBuf() { reset(); }
  void reset() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  int ensure(size_t bytes) {
    if (bytes <= n) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return NOVA_E_NOMEM;
    }
    n = bytes;
    return 0;
  }
};

bool is_pinned(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeDevice ||
         attr.type == hipMemoryTypeManaged;
}

// ---- library-owned stream pool ----------------------------------------------
constexpr int kMaxDevices = 64;
struct StreamPool {
  std::mutex mu;
  std::vector<hipStream_t> idle[kMaxDevices];
};
StreamPool& pool() {
  static StreamPool* p = new StreamPool;  // never destroyed: streams outlive exit order
  return *p;
}

// A pooled stream of the current device, or nullptr.
hipStream_t acquire_stream(int* dev_out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
    (void)hipGetLastError();
    return nullptr;
  }
  *dev_out = dev;
  {
    std::lock_guard<std::mutex> lk(pool().mu);
    auto& v = pool().idle[dev];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return s;
}

void release_stream(int dev, hipStream_t s) {
  if (!s) return;
  std::lock_guard<std::mutex> lk(pool().mu);
  pool().idle[dev].push_back(s);
}

// RAII set of pooled streams for one call.
struct Streams {
  std::vector<hipStream_t> s;
  int dev = 0;
  int get(int n) {
    for (int i = 0; i < n; i++) {
      hipStream_t x = acquire_stream(&dev);
      if (!x) return NOVA_E_NODEV;
      s.push_back(x);
    }
    return 0;
  }
  int sync() {
    int rc = 0;
    for (hipStream_t x : s) {
      const hipError_t e = hipStreamSynchronize(x);
      if (!rc && e != hipSuccess) rc = (int)e;
    }
    return rc;
  }
  ~Streams() {
    (void)sync();  // never hand back a stream with work in flight
    for (hipStream_t x : s) release_stream(dev, x);
  }
};

// Registers pageable host memory for the duration of a call (no-op if the
// caller pinned it).  Registrations are shared between concurrent calls and
// reference-counted by range: a call whose range lies inside one
// this library registered takes a reference to it, so the registering call's
// end cannot unregister memory another call's DMA still reads; a call whose
// range partly overlaps a live registration waits until that one is released
// (hipHostRegister rejects overlapping ranges), then registers its own.
// hipHostRegister pins whole pages, so every range is rounded out to pages
// before it is compared: two calls on disjoint byte ranges that
// share a page share (or wait for) one registration.  Otherwise the second
// call found its pages pinned -- by the first call -- took them for
// caller-pinned memory without a reference, and the first call's end could
// unregister a page the second call's DMA still read.
struct RegEntry {
  uintptr_t lo, hi;  // page-aligned
  int refs;
};
struct RegTable {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<RegEntry> live;
};
RegTable& reg_table() {
  static RegTable* t = new RegTable;  // never destroyed (exit order)
  return *t;
}
uintptr_t page_bytes() {
  static const uintptr_t p = [] {
    const long v = sysconf(_SC_PAGESIZE);
    return v > 0 ? (uintptr_t)v : (uintptr_t)4096;
  }();
  return p;
}

struct HostReg {
  uintptr_t key = 0;  // lo of the entry this call holds a reference to (0: none)
  int reg(const void* base, size_t len) {
    if (!len) return 0;
    const uintptr_t pg = page_bytes();
    const uintptr_t lo = (uintptr_t)base & ~(pg - 1);
    const uintptr_t hi = ((uintptr_t)base + len + pg - 1) & ~(pg - 1);
    RegTable& t = reg_table();
    std::unique_lock<std::mutex> lk(t.mu);
    for (;;) {
      bool overlap = false;
      for (RegEntry& e : t.live) {
        if (e.lo <= lo && hi <= e.hi) {  // inside a live registration: share it
          e.refs++;
          key = e.lo;
          return 0;
        }
        overlap |= e.lo < hi && lo < e.hi;
      }
      if (!overlap) break;
      t.cv.wait(lk);  // a partly overlapping registration is still in use
    }
    // No live registration of this library touches these pages, so pinned
    // pages here were pinned by the caller.
    if (is_pinned(base) && is_pinned((const uint8_t*)base + len - 1)) return 0;
    if (hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return NOVA_E_NOMEM;
    }
    t.live.push_back({lo, hi, 1});
    key = lo;
    return 0;
  }
  ~HostReg() {
    if (!key) return;
    RegTable& t = reg_table();
    std::lock_guard<std::mutex> lk(t.mu);
    for (size_t i = 0; i < t.live.size(); i++) {
      if (t.live[i].lo != key) continue;
      if (--t.live[i].refs == 0) {
        (void)hipHostUnregister(reinterpret_cast<void*>(key));
        t.live.erase(t.live.begin() + (long)i);
        t.cv.notify_all();
      }
      break;
    }
  }
};

// ---- variable-length host images --------------------------------------------
enum HostOp { kHostCrc = 0, kHostTrailers = 1, kHostVerify = 2 };

// Per-stream staging of one chunk: its byte span and rebased descriptors.
struct Stage {
  DevBuf data, offs, lens, init, out;
  PinBuf hoffs, hlens;  // rebased descriptors (pinned: async H2D)
};

// The calling thread's staging, kept between calls (hipMalloc / hipHostMalloc
// cost milliseconds: per call they were most of a one-SSTable call's time).
// Grows to the largest chunk seen; nova_host_staging_release() frees it.
struct HostStaging {
  std::vector<Stage> stage;
  PinBuf pres;
};
HostStaging& host_staging() {
  thread_local HostStaging h;
  return h;
}

// Runs a batch over blocks that live in host memory.  Blocks [b0, b1) form a
// chunk when their spanned bytes fit chunk_bytes (a single larger block gets a
// chunk of its own); the span [lo, hi) is copied H2D, the chunk's offsets are
// rebased to it, the kernel runs on the device copy and the per-block results
// (CRCs or verify flags) come back D2H into pinned memory.
int host_batch(HostOp op, const void* host_base, const uint64_t* offsets, const uint32_t* lengths,
               const uint32_t* init, size_t n_blocks, uint32_t flags, uint32_t* crc_out,
               uint8_t* ok_out, size_t chunk_bytes, int n_streams) {
  if (n_blocks == 0) return 0;
  if (!host_base || !offsets || !lengths) return NOVA_E_INVAL;
  n_streams = std::max(1, std::min(n_streams, 8));
  int err = nova_device_init();
  if (err) return err;
  const uint64_t tail = op == kHostVerify ? 5 : 0;  // verify reads the trailer too
  if (chunk_bytes == 0) {
    // about two chunks per stream so copies and kernels overlap, 4..64 MiB
    uint64_t lo = ~0ull, hi = 0;
    for (size_t b = 0; b < n_blocks; b++) {
      lo = std::min(lo, offsets[b]);
      hi = std::max(hi, offsets[b] + lengths[b] + tail);
    }
    chunk_bytes = std::max<uint64_t>(4ull << 20, std::min<uint64_t>(64ull << 20,
                                                                     (hi - lo) / (2 * n_streams)));
  }
  // chunk boundaries and spans
  struct Chunk { size_t b0, b1; uint64_t lo, hi; };
  std::vector<Chunk> chunks;
  uint64_t span_max = 0;
  size_t blocks_max = 0;
  uint64_t glo = ~0ull, ghi = 0;
  for (size_t b = 0; b < n_blocks;) {
    Chunk c{b, b, offsets[b], offsets[b] + lengths[b] + tail};
    while (c.b1 < n_blocks) {
      const uint64_t lo = std::min(c.lo, offsets[c.b1]);
      const uint64_t hi = std::max(c.hi, offsets[c.b1] + lengths[c.b1] + tail);
      if (c.b1 > c.b0 && hi - lo > chunk_bytes) break;
      c.lo = lo;
      c.hi = hi;
      c.b1++;
    }
    span_max = std::max(span_max, c.hi - c.lo);
    blocks_max = std::max(blocks_max, c.b1 - c.b0);
    glo = std::min(glo, c.lo);
    ghi = std::max(ghi, c.hi);
    chunks.push_back(c);
    b = c.b1;
  }
  HostReg hr;
  if ((err = hr.reg(static_cast<const uint8_t*>(host_base) + glo, ghi - glo))) return err;
  Streams st;
  if ((err = st.get(n_streams))) return err;
  HostStaging& hsg = host_staging();
  if (hsg.stage.size() < (size_t)n_streams) hsg.stage.resize(n_streams);
  std::vector<Stage>& stage = hsg.stage;
  PinBuf& pres = hsg.pres;  // results for the whole batch
  const size_t res_bytes = op == kHostVerify ? n_blocks : n_blocks * 4;
  if ((err = pres.ensure(res_bytes))) return err;
  for (int si = 0; si < n_streams; si++) {
    Stage& s = stage[si];
    if ((err = s.data.ensure(span_max + 16))) return err;
    if ((err = s.offs.ensure(blocks_max * 8)) || (err = s.lens.ensure(blocks_max * 4)) ||
        (err = s.out.ensure(op == kHostVerify ? blocks_max + 4 : blocks_max * 4)) ||
        (err = s.hoffs.ensure(blocks_max * 8)) || (err = s.hlens.ensure(blocks_max * 4)))
      return err;
    if (init && (err = s.init.ensure(blocks_max * 4))) return err;
  }
  const uint8_t* hb = static_cast<const uint8_t*>(host_base);
  int rc = 0;
  for (size_t k = 0; k < chunks.size() && !rc; k++) {
    const Chunk& c = chunks[k];
    const int si = (int)(k % n_streams);
    Stage& s = stage[si];
    hipStream_t hs = st.s[si];
    const size_t m = c.b1 - c.b0;
    // the stream's previous chunk must be done with the pinned descriptors
    if (k >= (size_t)n_streams && (rc = (int)hipStreamSynchronize(hs))) break;
    uint64_t* ho = static_cast<uint64_t*>(s.hoffs.p);
    for (size_t i = 0; i < m; i++) ho[i] = offsets[c.b0 + i] - c.lo;
    std::memcpy(s.hlens.p, lengths + c.b0, m * 4);
    hipError_t e = hipMemcpyAsync(s.data.p, hb + c.lo, c.hi - c.lo, hipMemcpyHostToDevice, hs);
    if (e == hipSuccess) e = hipMemcpyAsync(s.offs.p, ho, m * 8, hipMemcpyHostToDevice, hs);
    if (e == hipSuccess) e = hipMemcpyAsync(s.lens.p, s.hlens.p, m * 4, hipMemcpyHostToDevice, hs);
    if (e == hipSuccess && init)
      e = hipMemcpyAsync(s.init.p, init + c.b0, m * 4, hipMemcpyHostToDevice, hs);
    if (e != hipSuccess) { rc = (int)e; break; }
    const uint64_t* doffs = static_cast<const uint64_t*>(s.offs.p);
    const uint32_t* dlens = static_cast<const uint32_t*>(s.lens.p);
    // the host sees the lengths: a chunk of >= 16 KiB blocks on average gets the
    // large-blocks hint (segments; a few big blocks: pieces over the device)
    const uint32_t hint = (c.hi - c.lo) / m >= 16384 ? NOVA_CRC32C_HINT_LARGE_BLOCKS : 0u;
    if (op == kHostVerify) {
      rc = nova_sstable_verify_blocks_ex(s.data.p, doffs, dlens, m, static_cast<uint8_t*>(s.out.p),
                                         nullptr, hint, hs);
      if (!rc) rc = (int)hipMemcpyAsync(static_cast<uint8_t*>(pres.p) + c.b0, s.out.p, m,
                                        hipMemcpyDeviceToHost, hs);
    } else {
      // trailers: CRCs (type byte appended, masked) come back; the host writes
      // the 5 trailer bytes into its own image
      const uint32_t f = (op == kHostTrailers
                              ? ((flags & 0xff00u) | NOVA_CRC32C_APPEND_TYPE | NOVA_CRC32C_MASK_OUTPUT |
                                 (flags & NOVA_CRC32C_HINT_LARGE_BLOCKS))
                              : flags) |
                         hint;
      rc = nova_crc32c_batch(s.data.p, doffs, dlens,
                             init ? static_cast<const uint32_t*>(s.init.p) : nullptr,
                             static_cast<uint32_t*>(s.out.p), m, f, hs);
      if (!rc) rc = (int)hipMemcpyAsync(static_cast<uint32_t*>(pres.p) + c.b0, s.out.p, m * 4,
                                        hipMemcpyDeviceToHost, hs);
    }
  }
  const int rs = st.sync();
  if (!rc) rc = rs;
  if (rc) return rc;
  if (op == kHostVerify) {
    std::memcpy(ok_out, pres.p, n_blocks);
  } else if (op == kHostCrc) {
    std::memcpy(crc_out, pres.p, n_blocks * 4);
  } else {  // table/table_builder.cc:200-206, ltc/stoc_file_client_impl.cpp:713-719
    uint8_t* img = static_cast<uint8_t*>(const_cast<void*>(host_base));
    const uint32_t* m = static_cast<const uint32_t*>(pres.p);
    const uint8_t type = (uint8_t)((flags >> 8) & 0xffu);
    const bool quirk = (flags & NOVA_TRAILER_TB_QUIRK) != 0;
    for (size_t i = 0; i < n_blocks; i++) {
      uint8_t* t = img + offsets[i] + lengths[i];
      t[0] = type;
      t[1] = (uint8_t)m[i];
      t[2] = (uint8_t)(m[i] >> 8);
      t[3] = (uint8_t)(m[i] >> 16);
      t[4] = quirk ? (uint8_t)'!' : (uint8_t)(m[i] >> 24);
    }
  }
  return 0;
}

// ---- port hook ----------------------------------------------------------------
std::atomic<uint64_t> g_hook_host{0}, g_hook_device{0}, g_hook_fallback{0};

size_t env_size(const char* name, size_t def) {
  const char* v = std::getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  const unsigned long long x = std::strtoull(v, &end, 0);
  return end && *end == 0 ? (size_t)x : def;
}

// Below this size Extend stays on the host.  Measured on the GPU box
// (tools/hook_crossover.py, profiles/r03_hook_crossover.log): the host Extend
// runs ~33 GiB/s (4 MiB: 117 us), the device path (H2D + kernels + fold) 146 us
// at 4 MiB and 399 us vs 468 us at 16 MiB: the crossover is ~9 MiB.
size_t hook_min_bytes() {
  static const size_t v = env_size("NOVA_HOOK_MIN_BYTES", 8u << 20);
  return v;
}
// Largest device staging buffer the hook allocates (a larger call runs on the host).
size_t hook_max_staging() {
  static const size_t v = env_size("NOVA_HOOK_MAX_STAGING", 1ull << 30);
  return v;
}

// Staging a thread keeps between hook calls; a larger call's staging is freed
// when the call ends, so many threads that occasionally Extend() a big buffer
// do not each pin up to NOVA_HOOK_MAX_STAGING of HBM.
size_t hook_keep_staging() {
  static const size_t v = env_size("NOVA_HOOK_KEEP_STAGING", 64u << 20);
  return v;
}

// Per-thread device state of the hook: one pooled stream, staging buffers.
struct HookState {
  hipStream_t s = nullptr;
  int dev = -1;
  DevBuf dbuf, dout;
  ~HookState() {
    if (s) {
      (void)hipStreamSynchronize(s);
      release_stream(dev, s);
    }
  }
};
HookState& hook_state() {
  thread_local HookState hs;
  return hs;
}

// Extend(crc, buf, size) on the GPU: the buffer is cut into 4 KiB sub-blocks
// whose linear ("raw") CRCs the kernels compute; the host folds them with the
// GF(2) shift.  Returns nonzero on any failure (the caller falls back).
int device_extend(uint32_t crc, const char* buf, size_t size, uint32_t* out) {
  if (size > hook_max_staging()) return NOVA_E_NOMEM;
  if (nova_device_init() != 0) return NOVA_E_NODEV;
  HookState& hs = hook_state();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  if (!hs.s || hs.dev != dev) {
    if (hs.s) release_stream(hs.dev, hs.s);
    hs.s = acquire_stream(&hs.dev);
    if (!hs.s) return NOVA_E_NODEV;
    hs.dbuf.reset();
    hs.dout.reset();
  }
  constexpr uint32_t kSub = 4096;
  const size_t nsub = (size + kSub - 1) / kSub;
  const size_t full = size / kSub;
  if (hs.dbuf.ensure(size) || hs.dout.ensure(nsub * 4)) return NOVA_E_NOMEM;
  std::vector<uint32_t> raw(nsub);
  int rc = (int)hipMemcpyAsync(hs.dbuf.p, buf, size, hipMemcpyHostToDevice, hs.s);
  if (!rc && full)
    rc = nova_crc32c_batch_strided(hs.dbuf.p, kSub, kSub, full, nullptr,
                                   static_cast<uint32_t*>(hs.dout.p), NOVA_CRC32C_RAW, hs.s);
  const uint32_t tail = (uint32_t)(size - full * kSub);
  if (!rc && tail)
    rc = nova_crc32c_batch_strided(static_cast<uint8_t*>(hs.dbuf.p) + full * kSub, tail, tail, 1,
                                   nullptr, static_cast<uint32_t*>(hs.dout.p) + full,
                                   NOVA_CRC32C_RAW, hs.s);
  if (!rc) rc = (int)hipMemcpyAsync(raw.data(), hs.dout.p, nsub * 4, hipMemcpyDeviceToHost, hs.s);
  const hipError_t se = hipStreamSynchronize(hs.s);
  if (!rc && se != hipSuccess) rc = (int)se;
  if (hs.dbuf.n > hook_keep_staging()) {  // (the stream is idle: synchronized above)
    hs.dbuf.reset();
    hs.dout.reset();
  }
  if (rc) {
    (void)hipGetLastError();
    return rc;
  }
  // raw(D) = fold of sub-block raws; Extend(crc, D) = ~(M_size(~crc) ^ raw(D)).
  using namespace nova::gf2;
  const Lin m_sub = shift_bytes(kSub);
  uint32_t acc = 0;
  for (size_t i = 0; i < full; i++) acc = m_sub(acc) ^ raw[i];
  if (tail) acc = shift_bytes(tail)(acc) ^ raw[full];
  *out = ~(shift_bytes(size)(~crc) ^ acc);
  return 0;
}

// nova_crc32c_stream_host's pipelined form (NOVA_STREAM_HOST_PIPE).
int stream_host_pipe(const void* host_base, uint64_t stride, uint32_t len, size_t n_blocks, uint32_t* host_out,
                     uint32_t flags, size_t chunk_blocks, int nb, size_t span, size_t chunk_span, HostReg& hr) {
  (void)span;
  (void)hr;  // (registered by the caller for the whole call)
  Streams st;
  int rc = st.get(2);
  if (rc) return rc;
  hipStream_t sc = st.s[0], sk = st.s[1];  // copy, compute
  std::vector<DevBuf> dbuf(nb), dout(nb);
  std::vector<hipEvent_t> landed(nb, nullptr), freed(nb, nullptr);
  PinBuf pout;
  rc = pout.ensure(n_blocks * 4);
  for (int b = 0; b < nb && !rc; b++) {
    rc = dbuf[b].ensure(chunk_span);
    if (!rc) rc = dout[b].ensure(chunk_blocks * 4);
    if (!rc && (hipEventCreateWithFlags(&landed[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&freed[b], hipEventDisableTiming) != hipSuccess))
      rc = NOVA_E_NOMEM;
  }
  const uint8_t* hb = static_cast<const uint8_t*>(host_base);
  size_t k = 0;
  for (size_t b0 = 0; b0 < n_blocks && !rc; b0 += chunk_blocks, k++) {
    const size_t m = (n_blocks - b0 < chunk_blocks) ? n_blocks - b0 : chunk_blocks;
    const int b = (int)(k % (size_t)nb);
    const size_t bytes = (m - 1) * stride + len;
    hipError_t e = hipSuccess;
    if (k >= (size_t)nb) e = hipStreamWaitEvent(sc, freed[b], 0);  // its previous chunk was read
    if (e == hipSuccess) e = hipMemcpyAsync(dbuf[b].p, hb + b0 * stride, bytes, hipMemcpyHostToDevice, sc);
    if (e == hipSuccess) e = hipEventRecord(landed[b], sc);
    if (e == hipSuccess) e = hipStreamWaitEvent(sk, landed[b], 0);
    if (e != hipSuccess) {
      rc = (int)e;
      break;
    }
    rc = nova_crc32c_batch_strided(dbuf[b].p, stride, len, m, nullptr, static_cast<uint32_t*>(dout[b].p), flags,
                                   sk);
    if (rc) break;
    e = hipMemcpyAsync(static_cast<uint32_t*>(pout.p) + b0, dout[b].p, m * 4, hipMemcpyDeviceToHost, sk);
    if (e == hipSuccess) e = hipEventRecord(freed[b], sk);
    if (e != hipSuccess) rc = (int)e;
  }
  const int rs = st.sync();
  if (!rc) rc = rs;
  for (int b = 0; b < nb; b++) {
    if (landed[b]) (void)hipEventDestroy(landed[b]);
    if (freed[b]) (void)hipEventDestroy(freed[b]);
  }
  if (rc) (void)hipGetLastError();
  if (!rc) std::memcpy(host_out, pout.p, n_blocks * 4);
  return rc;
}

}  // namespace

extern "C" {

int nova_crc32c_stream_host(const void* host_base, uint64_t stride, uint32_t len,
                            size_t n_blocks, uint32_t* host_out, uint32_t flags,
                            size_t chunk_blocks, int n_streams) {
  if (n_blocks == 0) return 0;
  if (!host_base || !host_out || stride < len) return NOVA_E_INVAL;
  if (chunk_blocks == 0) chunk_blocks = 4096;
  n_streams = std::max(1, std::min(n_streams, 8));
  int err = nova_device_init();
  if (err) return err;

  const size_t span = (n_blocks - 1) * stride + len;
  HostReg hr;
  if ((err = hr.reg(host_base, span))) return err;
  const size_t chunk_span = (chunk_blocks - 1) * stride + len;
  // NOVA_STREAM_HOST_PIPE (default 1): every H2D copy on ONE copy stream,
  // back to back, so the link is fed as by a single large copy; a compute
  // stream runs each chunk's kernel once its copy has landed (an event) and
  // copies its CRCs back; n_streams device buffers rotate, a copy into one
  // waiting for the kernel that read it before (an event).  0: the round-1
  // form, each of n_streams streams copying, checksumming and returning its
  // own chunks (copies from several streams compete for the link).
  static const bool pipe = env_size("NOVA_STREAM_HOST_PIPE", 1) != 0;
  if (pipe) return stream_host_pipe(host_base, stride, len, n_blocks, host_out, flags, chunk_blocks,
                                    std::max(2, n_streams), span, chunk_span, hr);
  Streams st;
  if ((err = st.get(n_streams))) return err;
  std::vector<DevBuf> dbuf(n_streams), dout(n_streams);
  PinBuf pout;
  int rc = pout.ensure(n_blocks * 4);
  for (int s = 0; s < n_streams && !rc; s++) {
    rc = dbuf[s].ensure(chunk_span);
    if (!rc) rc = dout[s].ensure(chunk_blocks * 4);
  }
  const uint8_t* hb = static_cast<const uint8_t*>(host_base);
  size_t k = 0;
  for (size_t b0 = 0; b0 < n_blocks && !rc; b0 += chunk_blocks, k++) {
    const size_t m = (n_blocks - b0 < chunk_blocks) ? n_blocks - b0 : chunk_blocks;
    const int s = (int)(k % n_streams);
    const size_t bytes = (m - 1) * stride + len;
    hipError_t e = hipMemcpyAsync(dbuf[s].p, hb + b0 * stride, bytes, hipMemcpyHostToDevice,
                                  st.s[s]);
    if (e != hipSuccess) { rc = (int)e; break; }
    rc = nova_crc32c_batch_strided(dbuf[s].p, stride, len, m, nullptr,
                                   static_cast<uint32_t*>(dout[s].p), flags, st.s[s]);
    if (rc) break;
    e = hipMemcpyAsync(static_cast<uint32_t*>(pout.p) + b0, dout[s].p, m * 4,
                       hipMemcpyDeviceToHost, st.s[s]);
    if (e != hipSuccess) rc = (int)e;
  }
  const int rs = st.sync();
  if (!rc) rc = rs;
  if (!rc) std::memcpy(host_out, pout.p, n_blocks * 4);
  return rc;
}

int nova_crc32c_batch_host(const void* host_base, const uint64_t* offsets, const uint32_t* lengths,
                           const uint32_t* init_or_null, uint32_t* out_crc, size_t n_blocks,
                           uint32_t flags, size_t chunk_bytes, int n_streams) {
  if (n_blocks && !out_crc) return NOVA_E_INVAL;
  return host_batch(kHostCrc, host_base, offsets, lengths, init_or_null, n_blocks, flags, out_crc,
                    nullptr, chunk_bytes, n_streams);
}

int nova_sstable_write_trailers_host(void* host_buf, const uint64_t* offsets, const uint32_t* sizes,
                                     size_t n_blocks, uint32_t flags, size_t chunk_bytes,
                                     int n_streams) {
  return host_batch(kHostTrailers, host_buf, offsets, sizes, nullptr, n_blocks, flags, nullptr,
                    nullptr, chunk_bytes, n_streams);
}

int nova_sstable_verify_blocks_host(const void* host_buf, const uint64_t* offsets,
                                    const uint32_t* sizes, size_t n_blocks, uint8_t* ok_out,
                                    uint32_t* n_bad_out, size_t chunk_bytes, int n_streams) {
  if (n_blocks && !ok_out) return NOVA_E_INVAL;
  const int rc = host_batch(kHostVerify, host_buf, offsets, sizes, nullptr, n_blocks, 0, nullptr,
                            ok_out, chunk_bytes, n_streams);
  if (!rc && n_bad_out) {
    uint32_t bad = 0;
    for (size_t i = 0; i < n_blocks; i++) bad += ok_out[i] ? 0u : 1u;
    *n_bad_out = bad;
  }
  return rc;
}

uint32_t nova_port_accelerated_crc32c(uint32_t crc, const char* buf, size_t size) {
  // Contract of port::AcceleratedCRC32C: the extended CRC.  Once the reference
  // adopts the hook (util/crc32c.cc:487-491) every Extend() comes here, so the
  // hook never answers "cannot accelerate" (0) with a wrong CRC: small buffers
  // and any GPU failure take the host Extend.
  if (size == 0) return crc;
  if (buf && size >= hook_min_bytes()) {
    uint32_t out = 0;
    if (device_extend(crc, buf, size, &out) == 0) {
      g_hook_device.fetch_add(1, std::memory_order_relaxed);
      return out;
    }
    g_hook_fallback.fetch_add(1, std::memory_order_relaxed);
  } else {
    g_hook_host.fetch_add(1, std::memory_order_relaxed);
  }
  return nova_crc32c_extend(crc, buf, size);
}

void nova_host_staging_release(void) {
  HostStaging& h = host_staging();
  h.stage.clear();
  h.pres.reset();
  HookState& hs = hook_state();  // the port hook's staging too
  if (hs.s) (void)hipStreamSynchronize(hs.s);
  hs.dbuf.reset();
  hs.dout.reset();
}

void nova_port_stats(uint64_t* host_calls, uint64_t* device_calls, uint64_t* fallback_calls) {
  if (host_calls) *host_calls = g_hook_host.load();
  if (device_calls) *device_calls = g_hook_device.load();
  if (fallback_calls) *fallback_calls = g_hook_fallback.load();
}

}  // extern "C"
