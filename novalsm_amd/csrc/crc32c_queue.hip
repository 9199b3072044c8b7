// Coalescing submission queue for per-SSTable callers.
//
// NovaLSM checksums one SSTable per call, from many threads at once: every
// compaction thread finishing a table (TableBuilder::Finish ->
// StoCWritableFileClient::Format, ltc/stoc_file_client_impl.cpp:274-289) and
// every reader verifying a fetched table (table/table.cc:425-441).  One
// ~16 MiB table is ~2 us of HBM time at 8 TB/s, well under a launch's fixed
// cost, so callers that each launch on their own stream leave the device
// mostly idle (tools/concurrent_sst.py: 16 threads reach ~27 % of peak).
//
// nova_sst_queue_* put concurrent calls into one launch, the way LevelDB's
// DBImpl::Write groups concurrent writers (db/db_impl.cc, the writers_ deque):
// a caller enqueues its table; the caller at the front of the queue, while a
// launch slot is free, becomes the leader, takes every compatible request
// queued behind it (same operation and flags, up to kMaxReqs tables and
// kMaxBlocks blocks) and runs them as one batch:
//   1. qgather_kernel: the batch's block descriptors into one array of
//      absolute addresses (base 0) and sizes, from each table's own arrays;
//   2. the product dispatch (run(): rounds / burst kernels) over that array;
//   3. verify: qscatter_kernel copies each table's ok flags back to its own
//      array and adds its mismatches to its own counter.
// A batch of one (no other caller waiting) is the plain call on the caller's
// own stream.  The leader waits for the batch, marks its requests done and
// wakes each follower (one condition variable per request: no thundering
// herd).  kSlots batches may be in flight at once (one stream and one scratch
// set each), so the next batch forms and launches while one runs.
// Results are identical to the per-table calls: each block's checksum is
// computed by the same kernels from the same bytes.
//
// Round 4: by default the queue entry points run on the persistent engine
// (crc32c_engine.hip), which pays no launch per table; the
// coalescing batches below serve NOVA_SST_ENGINE=0, and the plain call any
// request the engine cannot run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <mutex>

#include "crc32c_internal.hpp"

namespace nova_dev {
// engine_submit's code for a request declined during a yield storm
// (crc32c_engine.hip): nothing was published, the caller runs the plain call,
// and it is not counted as a fallback.
bool engine_declined(int rc);
}  // namespace nova_dev

namespace {

using namespace nova_dev;

constexpr int kMaxReqs = 32;                 // tables per batch (kernel-argument table)
constexpr uint64_t kMaxBlocks = 1ull << 20;  // blocks per batch (scratch per slot: 13 MiB)
constexpr int kSlots = 4;                    // batches in flight (at most)
constexpr int kDefaultSlots = 4;  // tools/concurrent_sst.py: 4 beat 2 in most rows

struct QTable {
  uint64_t base;          // the table image's device address
  const uint64_t* offs;   // its block offsets (relative to base)
  const uint32_t* sizes;  // its block sizes
  uint8_t* ok;            // verify: its ok flags
  uint32_t* bad;          // verify: its mismatch counter (may be null)
  uint64_t start;         // first index in the batch's arrays
};
struct QBatch {
  QTable t[kMaxReqs];
  uint32_t n_tables;
  uint64_t n_blocks;
};

// Combined index i -> (table r, block j).  The table list is kernel-argument
// (scalar) data; a linear scan over <= 32 starts.
__device__ __forceinline__ uint32_t qtable_of(const QBatch& b, uint64_t i) {
  uint32_t r = 0;
  for (uint32_t k = 1; k < b.n_tables; k++) r = i >= b.t[k].start ? k : r;
  return r;
}

// last[i] = 1 at every table's first and last block: the batched trailer
// writer must not rewrite those blocks' whole 64-B trailer pieces, which may
// reach past the end of the table's image (last block) or before its start (a
// first block shorter than the piece) into memory of another caller (ADVICE
// r03; the plain call never does: its image's edge blocks are never eligible).
__global__ void __launch_bounds__(256) qgather_kernel(QBatch b, uint64_t* offs, uint32_t* sizes,
                                                      uint8_t* last) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n_blocks) return;
  const uint32_t r = qtable_of(b, i);
  const QTable& T = b.t[r];
  const uint64_t j = i - T.start;
  offs[i] = T.base + T.offs[j];
  sizes[i] = T.sizes[j];
  const bool end = r + 1 < b.n_tables ? i + 1 == b.t[r + 1].start : i + 1 == b.n_blocks;
  last[i] = (end || j == 0) ? 1 : 0;
}

__global__ void __launch_bounds__(256) qscatter_kernel(QBatch b, const uint8_t* ok) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = i < b.n_blocks;
  const uint32_t r = in ? qtable_of(b, i) : 0;
  const QTable& T = b.t[r];
  const uint8_t v = in ? ok[i] : 1;
  if (in) T.ok[i - T.start] = v;
  if (in && v == 0 && T.bad) atomicAdd(T.bad, 1u);  // a corrupt block: rare
}

struct Req {
  int mode;
  uint32_t flags;
  const uint8_t* buf;
  const uint64_t* offs;
  const uint32_t* sizes;
  uint64_t n;
  uint8_t* ok;
  uint32_t* bad;
  hipStream_t stream;           // the caller's: idle when the request is queued
  std::condition_variable cv;   // woken when done, or when it may lead
  bool done = false;
  int rc = 0;
};

struct Slot {
  hipStream_t stream = nullptr;
  uint64_t* offs = nullptr;
  uint32_t* sizes = nullptr;
  uint8_t* ok = nullptr;
  uint8_t* last = nullptr;  // 1 at each table's first and last block (trailer writer)
  bool busy = false;
};

struct Queue {
  std::mutex mu;
  std::deque<Req*> q;
  Slot slot[kSlots];
  uint64_t batches = 0, requests = 0, max_tables = 0;

  // A slot counts as set up only once every one of its allocations succeeded
  // (ADVICE r03): a partial failure frees what it got and leaves the slot
  // empty, so a later batch retries instead of gathering through null arrays.
  int init_slot(Slot& s) {
    if (s.stream && s.offs && s.sizes && s.ok && s.last) return 0;
    Slot n{};
    hipError_t e = hipStreamCreateWithFlags(&n.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&n.offs, kMaxBlocks * 8);
    if (e == hipSuccess) e = hipMalloc(&n.sizes, kMaxBlocks * 4);
    if (e == hipSuccess) e = hipMalloc(&n.ok, kMaxBlocks);
    if (e == hipSuccess) e = hipMalloc(&n.last, kMaxBlocks);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (n.last) (void)hipFree(n.last);
      if (n.ok) (void)hipFree(n.ok);
      if (n.sizes) (void)hipFree(n.sizes);
      if (n.offs) (void)hipFree(n.offs);
      if (n.stream) (void)hipStreamDestroy(n.stream);
      (void)hipGetLastError();
      return NOVA_E_NOMEM;
    }
    n.busy = s.busy;
    s = n;
    return 0;
  }

  // One batch (the leader, without the lock).  A batch of one runs as the
  // plain call on its caller's stream; a larger one on the slot's stream:
  // gather, the product dispatch over absolute addresses, scatter.
  int run_batch(Slot& s, Req** rs, int nr) {
    if (nr == 1) {
      CrcParams p{};
      p.base = rs[0]->buf;
      p.offsets = rs[0]->offs;
      p.lengths = rs[0]->sizes;
      p.n_blocks = rs[0]->n;
      p.flags = rs[0]->flags;
      p.ok_out = rs[0]->ok;
      p.n_bad = rs[0]->bad;
      const int rc = dispatch(rs[0]->mode, p, rs[0]->stream);
      return rc ? rc : (int)hipStreamSynchronize(rs[0]->stream);
    }
    int rc = init_slot(s);
    if (rc) return rc;
    // tables in address order: the batch's blocks ascend when each table's
    // do, which the trailer writer's whole-piece pass needs (trailer_layout)
    std::sort(rs, rs + nr, [](const Req* a, const Req* b) { return a->buf < b->buf; });
    QBatch b{};
    uint64_t total = 0;
    for (int k = 0; k < nr; k++) {
      b.t[k] = QTable{(uint64_t)rs[k]->buf, rs[k]->offs, rs[k]->sizes, rs[k]->ok, rs[k]->bad, total};
      total += rs[k]->n;
    }
    b.n_tables = (uint32_t)nr;
    b.n_blocks = total;
    const uint64_t wgs = (total + 255) / 256;
    hipLaunchKernelGGL(qgather_kernel, dim3((uint32_t)wgs), dim3(256), 0, s.stream, b, s.offs, s.sizes,
                       s.last);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    CrcParams p{};
    p.base = nullptr;  // offsets are absolute addresses
    p.offsets = s.offs;
    p.lengths = s.sizes;
    p.n_blocks = total;
    p.flags = rs[0]->flags;
    const int mode = rs[0]->mode;
    if (mode == kVerify) p.ok_out = s.ok;
    if (mode == kTrailer) p.tr_last = s.last;
    rc = dispatch(mode, p, s.stream);
    if (rc) return rc;
    if (mode == kVerify) {
      hipLaunchKernelGGL(qscatter_kernel, dim3((uint32_t)wgs), dim3(256), 0, s.stream, b, s.ok);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    e = hipStreamSynchronize(s.stream);
    return e == hipSuccess ? 0 : (int)e;
  }

  // Batches in flight: NOVA_SST_QUEUE_SLOTS (1..4, default 4, read once) or
  // nova_sst_queue_set_slots (0 restores that default).
  static int env_slots() {
    static const int n = [] {
      const char* v = getenv("NOVA_SST_QUEUE_SLOTS");
      const int x = v ? atoi(v) : kDefaultSlots;
      return x >= 1 && x <= kSlots ? x : kDefaultSlots;
    }();
    return n;
  }
  int set_slots = 0;  // under mu
  // Test hook (nova_sst_queue_hold): while held no request leads, so callers
  // queue up deterministically; releasing wakes the front one.
  bool held = false;  // under mu
  int slots() const { return set_slots ? set_slots : env_slots(); }
  int free_slot(int ns) const {
    for (int k = 0; k < ns; k++)
      if (!slot[k].busy) return k;
    return -1;
  }
  void wake_front() {
    if (!q.empty()) q.front()->cv.notify_one();
  }

  int submit(Req& r) {
    std::unique_lock<std::mutex> lk(mu);
    q.push_back(&r);
    int si = -1;
    for (;;) {
      if (r.done) return r.rc;
      // (a popped request waits for done; front() of an empty deque is undefined;
      // the slot count is read on every wake: nova_sst_queue_set_slots may raise it)
      if (!held && !q.empty() && q.front() == &r && (si = free_slot(slots())) >= 0) break;
      r.cv.wait(lk);
    }
    // leader: take the compatible requests at the queue's front (r first)
    Req* rs[kMaxReqs];
    int nr = 0;
    uint64_t blocks = 0;
    while (!q.empty() && nr < kMaxReqs) {
      Req* x = q.front();
      if (x->mode != r.mode || x->flags != r.flags || (nr && blocks + x->n > kMaxBlocks)) break;
      rs[nr++] = x;
      blocks += x->n;
      q.pop_front();
    }
    slot[si].busy = true;
    batches++;
    requests += (uint64_t)nr;
    if ((uint64_t)nr > max_tables) max_tables = (uint64_t)nr;
    wake_front();  // it may lead on another free slot
    lk.unlock();
    const int rc = run_batch(slot[si], rs, nr);
    lk.lock();
    slot[si].busy = false;
    for (int k = 0; k < nr; k++) {  // under the lock: a woken caller's Req ends with its call
      rs[k]->rc = rc;
      rs[k]->done = true;
      if (rs[k] != &r) rs[k]->cv.notify_one();
    }
    wake_front();
    return r.rc;
  }
};

constexpr int kMaxDev = 16;
Queue g_q[kMaxDev];

int enqueue(Req& r, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  int err = 0;
  if (!tables(&err)) return err;
  // Work queued on the caller's stream (the image, its descriptors) finishes
  // before the request can join a batch on another stream.  Done here, in the
  // caller's thread, so the leader issues no per-request wait.
  hipError_t e = hipStreamQuery(stream);
  if (e == hipErrorNotReady) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return (int)e;
  r.stream = stream;
  bool plain = r.n > kMaxBlocks;  // larger than one batch: the plain call (one launch is efficient)
  if (!plain && engine_enabled()) {
    // the persistent engine (crc32c_engine.hip); if it did not run the
    // request and has let go of it, the plain call computes it (after zeroing
    // a verify counter the engine may have added to)
    const int erc = engine_submit(r.mode, r.buf, r.offs, r.sizes, r.n, r.flags,
                                  r.mode == kVerify ? (void*)r.ok : nullptr, r.bad);
    if (erc == 0) return 0;
    // the engine may still write this request's outputs: no plain call
    if (engine_unsafe(erc)) return NOVA_E_NODEV;
    if (!engine_declined(erc)) {  // (declined in a yield storm: the engine never saw the request)
      engine_count_fallback();
      if (r.mode == kVerify && r.bad && (e = hipMemsetAsync(r.bad, 0, sizeof(uint32_t), stream)) != hipSuccess)
        return (int)e;
    }
    plain = true;
  }
  if (plain) {
    CrcParams p{};
    p.base = r.buf;
    p.offsets = r.offs;
    p.lengths = r.sizes;
    p.n_blocks = r.n;
    p.flags = r.flags;
    p.ok_out = r.ok;
    p.n_bad = r.bad;
    const int rc = dispatch(r.mode, p, stream);
    return rc ? rc : (int)hipStreamSynchronize(stream);
  }
  return g_q[dev].submit(r);
}

}  // namespace

extern "C" {

int nova_sst_queue_write_trailers(void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                  size_t n_blocks, uint32_t flags, void* stream) {
  if (n_blocks == 0) return 0;
  if (!buf || !offsets || !sizes) return NOVA_E_INVAL;
  Req r{};
  r.mode = kTrailer;
  r.flags = (flags & (0xff00u | NOVA_TRAILER_TB_QUIRK)) | NOVA_CRC32C_APPEND_TYPE;
  r.buf = (const uint8_t*)buf;
  r.offs = offsets;
  r.sizes = sizes;
  r.n = n_blocks;
  return enqueue(r, (hipStream_t)stream);
}

int nova_sst_queue_verify_blocks(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                 size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out, void* stream) {
  if (n_blocks == 0) return 0;
  if (!buf || !offsets || !sizes || !ok_out) return NOVA_E_INVAL;
  Req r{};
  r.mode = kVerify;
  r.flags = 0;
  r.buf = (const uint8_t*)buf;
  r.offs = offsets;
  r.sizes = sizes;
  r.n = n_blocks;
  r.ok = ok_out;
  r.bad = n_bad_out;
  return enqueue(r, (hipStream_t)stream);
}

int nova_sst_queue_set_slots(int slots) {
  if (slots < 0 || slots > kSlots) return NOVA_E_INVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  Queue& q = g_q[dev];
  std::lock_guard<std::mutex> lk(q.mu);
  q.set_slots = slots;
  q.wake_front();  // more slots: the front request may lead now
  return 0;
}

int nova_sst_queue_hold(int hold, uint64_t* queued) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  Queue& q = g_q[dev];
  std::lock_guard<std::mutex> lk(q.mu);
  if (hold >= 0) {
    q.held = hold != 0;
    if (!q.held) q.wake_front();
  }
  if (queued) *queued = (uint64_t)q.q.size();
  return 0;
}

int nova_sst_queue_stats(uint64_t* batches, uint64_t* requests, uint64_t* max_tables_per_batch) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  Queue& q = g_q[dev];
  std::lock_guard<std::mutex> lk(q.mu);
  if (batches) *batches = q.batches;
  if (requests) *requests = q.requests;
  if (max_tables_per_batch) *max_tables_per_batch = q.max_tables;
  return 0;
}

}  // extern "C"
