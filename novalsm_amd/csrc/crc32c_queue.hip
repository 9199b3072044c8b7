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
// The leader waits for its slot's stream, marks the batch done and wakes the
// followers.  kSlots batches may be in flight at once (one stream and one
// scratch set each), so the next batch forms and launches while one runs.
// Results are identical to the per-table calls: each block's checksum is
// computed by the same kernels from the same bytes.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <mutex>

#include "crc32c_internal.hpp"

namespace {

using namespace nova_dev;

constexpr int kMaxReqs = 32;                 // tables per batch (kernel-argument table)
constexpr uint64_t kMaxBlocks = 1ull << 20;  // blocks per batch (scratch per slot: 13 MiB)
constexpr int kSlots = 2;                    // batches in flight (at most)

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

__global__ void __launch_bounds__(256) qgather_kernel(QBatch b, uint64_t* offs, uint32_t* sizes) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n_blocks) return;
  const QTable& T = b.t[qtable_of(b, i)];
  const uint64_t j = i - T.start;
  offs[i] = T.base + T.offs[j];
  sizes[i] = T.sizes[j];
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
  hipEvent_t ready;  // recorded on the caller's stream at submission
  bool done = false;
  int rc = 0;
};

struct Slot {
  hipStream_t stream = nullptr;
  uint64_t* offs = nullptr;
  uint32_t* sizes = nullptr;
  uint8_t* ok = nullptr;
  bool busy = false;
};

struct Queue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Req*> q;
  Slot slot[kSlots];
  uint64_t batches = 0, requests = 0, max_tables = 0;

  int init_slot(Slot& s) {
    if (s.stream) return 0;
    hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&s.offs, kMaxBlocks * 8);
    if (e == hipSuccess) e = hipMalloc(&s.sizes, kMaxBlocks * 4);
    if (e == hipSuccess) e = hipMalloc(&s.ok, kMaxBlocks);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return NOVA_E_NOMEM;
    }
    return 0;
  }

  // One batch on slot s (the leader, without the lock).
  int run_batch(Slot& s, Req** rs, int nr) {
    int rc = init_slot(s);
    if (rc) return rc;
    QBatch b{};
    uint64_t total = 0;
    for (int k = 0; k < nr; k++) {
      const hipError_t e = hipStreamWaitEvent(s.stream, rs[k]->ready, 0);
      if (e != hipSuccess) return (int)e;
      b.t[k] = QTable{(uint64_t)rs[k]->buf, rs[k]->offs, rs[k]->sizes, rs[k]->ok, rs[k]->bad, total};
      total += rs[k]->n;
    }
    b.n_tables = (uint32_t)nr;
    b.n_blocks = total;
    const uint64_t wgs = (total + 255) / 256;
    hipLaunchKernelGGL(qgather_kernel, dim3((uint32_t)wgs), dim3(256), 0, s.stream, b, s.offs, s.sizes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    CrcParams p{};
    p.base = nullptr;  // offsets are absolute addresses
    p.offsets = s.offs;
    p.lengths = s.sizes;
    p.n_blocks = total;
    const int mode = rs[0]->mode;
    if (mode == kTrailer) {
      p.flags = rs[0]->flags;
    } else {
      p.ok_out = s.ok;
      p.flags = rs[0]->flags;
    }
    rc = dispatch(mode, p, s.stream);
    if (rc) return rc;
    if (mode == kVerify) {
      hipLaunchKernelGGL(qscatter_kernel, dim3((uint32_t)wgs), dim3(256), 0, s.stream, b, s.ok);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    e = hipStreamSynchronize(s.stream);
    return e == hipSuccess ? 0 : (int)e;
  }

  // NOVA_SST_QUEUE_SLOTS=1 keeps one batch in flight (read once)
  static int slots() {
    static const int n = [] {
      const char* v = getenv("NOVA_SST_QUEUE_SLOTS");
      const int x = v ? atoi(v) : kSlots;
      return x >= 1 && x <= kSlots ? x : kSlots;
    }();
    return n;
  }

  int submit(Req& r) {
    const int ns = slots();
    std::unique_lock<std::mutex> lk(mu);
    q.push_back(&r);
    int si = -1;
    for (;;) {
      if (r.done) return r.rc;
      if (q.front() == &r) {
        for (int k = 0; k < ns; k++)
          if (!slot[k].busy) {
            si = k;
            break;
          }
        if (si >= 0) break;
      }
      cv.wait(lk);
    }
    // leader: take the compatible requests at the queue's front
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
    cv.notify_all();  // the next front may lead on the other slot
    lk.unlock();
    const int rc = run_batch(slot[si], rs, nr);
    lk.lock();
    slot[si].busy = false;
    for (int k = 0; k < nr; k++) {
      rs[k]->rc = rc;
      rs[k]->done = true;
    }
    cv.notify_all();
    return r.rc;
  }
};

constexpr int kMaxDev = 16;
Queue g_q[kMaxDev];

thread_local hipEvent_t t_ev[kMaxDev] = {};

int enqueue(Req& r, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return NOVA_E_NODEV;
  }
  int err = 0;
  if (!tables(&err)) return err;
  if (r.n > kMaxBlocks) {  // larger than one batch: the direct path (one launch is efficient)
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
  hipEvent_t& ev = t_ev[dev];
  if (!ev) {
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      ev = nullptr;
      return (int)e;
    }
  }
  const hipError_t e = hipEventRecord(ev, stream);
  if (e != hipSuccess) return (int)e;
  r.ready = ev;
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
