// Native caller threads for the per-SSTable paths -- the shape NovaLSM calls
// them in: T host threads (flush / compaction EnvBGThreads finishing tables,
// ltc/compaction_thread.h:77-107 -> StoCWritableFileClient::Format,
// ltc/stoc_file_client_impl.cpp:183-377; readers verifying a fetched table,
// ReadAll :843-882 -> table/table.cc:425-441), each with its own HIP stream and
// its own device-resident SSTable image of `blocks` blocks of 4096+U[0,255] B
// with 5-B trailers, each checksumming its table and waiting for the result,
// back to back.  Optionally one more thread makes plain calls of the other
// entry points (block verify, log-record verify, CRC batch) on its own stream,
// as the log writer (db/log_writer.cc:99-125) and the parity build
// (ltc/stoc_file_client_impl.cpp:334-349) do beside the compaction threads.
//
// Used by bench.py (the sst_engine secondary), tools/concurrent_sst.py and the
// mixed-caller GPU test; linked against libnova_crc32c.so (libnova_sst_callers.so).
// Native threads: the host cost measured is the library's, not an
// interpreter lock's.
//
// What is checked (stated exactly):
//   * verify: each table has one corrupted block.  Call i of a thread counts
//     its mismatches into its own zeroed counter (i % 2^20) and writes its
//     flags into its own flag set (i % S, S = 65536 sets, or fewer when a set
//     of a large table would exceed 256 MiB per thread).  After the run every
//     counter must hold exactly one mismatch per call that used it, and a
//     device pass checks every flag set used: exactly the corrupted block
//     flagged.  So every call's count and every call's flags are checked as
//     long as a thread makes at most S calls (the bench's windows make fewer);
//     beyond S, a reused set shows its last call's flags only;
//   * trailers: every call rewrites the same trailers in place, so what is
//     checked is the FINAL image (trailers scrambled before the first call,
//     compared byte for byte with a plain-call reference image afterwards):
//     a wrong trailer that a later call rewrote correctly is not detected;
//   * plain calls: each result is copied back and compared with the expected
//     one the caller passed (computed and checked against the oracle first).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nova_crc32c.h"

namespace {

using Clock = std::chrono::steady_clock;

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr uint64_t kMaxSets = 1u << 16;          // verify flag sets per thread (one per call)
constexpr uint64_t kSetBytes = 256ull << 20;     // ... within this many bytes per thread
constexpr uint64_t kCounters = 1u << 20;  // verify: one zeroed mismatch counter per call (4 MiB per thread)

struct Call {
  double t0, t1;  // seconds after the window's start
  uint64_t lc[8];  // engine path: nova_sst_engine_last_call
};

struct Table {
  hipStream_t stream = nullptr;
  uint8_t* img = nullptr;
  uint64_t* offs = nullptr;
  uint32_t* lens = nullptr;
  uint8_t* ok = nullptr;    // sets x n
  uint64_t sets = 0;
  uint32_t* bad = nullptr;  // kCounters counters, call i's at i % kCounters
  uint64_t n = 0, bytes = 0, algo_bytes = 0, victim = 0;
  std::vector<uint64_t> h_offs;
  std::vector<uint32_t> h_lens;
  std::vector<uint8_t> expect_img;  // trailers: the reference image
  std::vector<Call> calls;
  uint64_t ncalls = 0;
  int rc = 0;
};

#define CKH(x)                            \
  do {                                    \
    hipError_t e_ = (x);                  \
    if (e_ != hipSuccess) return (int)e_; \
  } while (0)
#define CKN(x)               \
  do {                       \
    int r_ = (x);            \
    if (r_ != 0) return r_;  \
  } while (0)

int make_table(Table& tb, uint64_t n, uint64_t seed, bool verify) {
  uint64_t s = seed;
  tb.n = n;
  tb.h_offs.resize(n);
  tb.h_lens.resize(n);
  uint64_t pos = 0, sum_len = 0;
  for (uint64_t i = 0; i < n; i++) {
    tb.h_lens[i] = 4096 + (uint32_t)(splitmix(s) & 255);
    tb.h_offs[i] = pos;
    pos += tb.h_lens[i] + 5;
    sum_len += tb.h_lens[i];
  }
  tb.bytes = pos;
  tb.algo_bytes = sum_len + n * (verify ? 6 : 5);
  tb.victim = splitmix(s) % n;
  CKH(hipStreamCreateWithFlags(&tb.stream, hipStreamNonBlocking));
  CKH(hipMalloc(&tb.img, pos + 64));
  CKH(hipMalloc(&tb.offs, n * 8));
  CKH(hipMalloc(&tb.lens, n * 4));
  tb.sets = verify ? std::min<uint64_t>(kMaxSets, std::max<uint64_t>(64, kSetBytes / n)) : 1;
  CKH(hipMalloc(&tb.ok, n * tb.sets));
  CKH(hipMalloc(&tb.bad, 4 * kCounters));
  CKH(hipMemcpy(tb.offs, tb.h_offs.data(), n * 8, hipMemcpyHostToDevice));
  CKH(hipMemcpy(tb.lens, tb.h_lens.data(), n * 4, hipMemcpyHostToDevice));
  CKN(nova_fill_splitmix64(tb.img, pos + 64, seed * 7 + 1, 0, tb.stream));
  CKN(nova_sstable_write_trailers(tb.img, tb.offs, tb.lens, n, 0, tb.stream));
  CKH(hipMemsetAsync(tb.bad, 0, 4 * kCounters, tb.stream));
  CKH(hipStreamSynchronize(tb.stream));
  if (verify) {  // one corrupted byte in the victim block
    uint8_t b = 0;
    uint8_t* at = tb.img + tb.h_offs[tb.victim] + 17;
    CKH(hipMemcpy(&b, at, 1, hipMemcpyDeviceToHost));
    b ^= 0x20;
    CKH(hipMemcpy(at, &b, 1, hipMemcpyHostToDevice));
  } else {  // the reference image, then every trailer scrambled
    tb.expect_img.resize(pos);
    CKH(hipMemcpy(tb.expect_img.data(), tb.img, pos, hipMemcpyDeviceToHost));
    std::vector<uint8_t> scr(tb.expect_img);
    for (uint64_t i = 0; i < n; i++)
      for (int k = 0; k < 5; k++) scr[tb.h_offs[i] + tb.h_lens[i] + k] ^= (uint8_t)(0x5Au + k);
    CKH(hipMemcpy(tb.img, scr.data(), pos, hipMemcpyHostToDevice));
  }
  return 0;
}

void free_table(Table& tb) {
  if (tb.stream) {
    (void)nova_stream_release(tb.stream);
    (void)hipStreamDestroy(tb.stream);
  }
  (void)hipFree(tb.img);
  (void)hipFree(tb.offs);
  (void)hipFree(tb.lens);
  (void)hipFree(tb.ok);
  (void)hipFree(tb.bad);
}

// Every flag of the first `sets` flag sets: 1, except 0 at the victim block.
__global__ void check_flag_sets(const uint8_t* ok, uint64_t n, uint64_t sets, uint64_t victim,
                                unsigned long long* wrong_sets) {
  const uint64_t s = blockIdx.x;  // one workgroup per set
  if (s >= sets) return;
  bool bad = false;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) bad = bad || ok[s * n + i] != (i == victim ? 0 : 1);
  if (bad) atomicAdd(wrong_sets, 1ull);  // (counts threads that saw a wrong flag; 0 iff all are right)
}

double pct(std::vector<double>& v, double p) {
  if (v.empty()) return 0;
  return v[std::min(v.size() - 1, (size_t)(p * (double)v.size()))];
}

bool read_cpu_stat(uint64_t* throttled, uint64_t* throttled_us) {
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return false;
  char k[64];
  unsigned long long v = 0;
  *throttled = *throttled_us = 0;
  while (fscanf(f, "%63s %llu", k, &v) == 2) {
    if (!strcmp(k, "nr_throttled")) *throttled = v;
    if (!strcmp(k, "throttled_usec")) *throttled_us = v;
  }
  fclose(f);
  return true;
}

}  // namespace

extern "C" {

// The plain-call thread's inputs (device pointers; expected results on the host).
typedef struct {
  const void* v_img;  // SSTable verify (nova_sstable_verify_blocks)
  const uint64_t* v_offs;
  const uint32_t* v_lens;
  uint64_t v_n;
  const uint8_t* v_expect_ok;
  uint32_t v_expect_bad;
  const void* l_img;  // log verify (nova_log_verify_records)
  uint64_t l_len;
  const uint64_t* l_offs;
  uint64_t l_n;
  const uint8_t* l_expect;
  uint32_t l_expect_bad;
  const void* b_img;  // CRC batch (nova_crc32c_batch)
  const uint64_t* b_offs;
  const uint32_t* b_lens;
  uint64_t b_n;
  const uint32_t* b_expect;
  double gap_us;  // pause between plain calls
} nova_callers_plain;

typedef struct {
  int op;          // 0 verify, 1 trailers
  int threads;     // table callers (0: only the plain thread)
  uint64_t blocks; // blocks per table
  double warm_s;   // callers run this long before the window opens
  double secs;     // the measured window
  int path;        // 0 direct calls + stream sync, 1 nova_sst_queue_* (engine), 2 nova_sst_queue_* (coalescing queue)
  uint64_t seed;
  const nova_callers_plain* plain;  // may be null
} nova_callers_cfg;

int nova_callers_run(const nova_callers_cfg* cfg, char* json, size_t cap) {
  if (!cfg || !json || cap < 64 || cfg->threads < 0 || cfg->threads > 64 || cfg->blocks > (1u << 20) ||
      cfg->secs <= 0 || cfg->warm_s < 0 || (cfg->threads && cfg->blocks == 0))
    return NOVA_E_INVAL;
  const bool verify = cfg->op == 0;
  const int T = cfg->threads;
  CKN(nova_device_init());
  // NOVA_CALLERS_TRACE=1: the engine's per-request spans (nova_sst_engine_set_trace) in the JSON
  const bool trace = getenv("NOVA_CALLERS_TRACE") && atoi(getenv("NOVA_CALLERS_TRACE")) != 0;
  // The routing (and tracing) this harness sets is put back on EVERY return
  // (ADVICE r05): later calls of the process go by NOVA_SST_ENGINE again.
  struct Restore {
    bool trace;
    ~Restore() {
      (void)nova_sst_engine_set_enabled(-1);
      if (trace) (void)nova_sst_engine_set_trace(0);
    }
  } restore{cfg->path == 1 && trace};
  if (cfg->path == 1) CKN(nova_sst_engine_set_enabled(1));
  if (cfg->path == 1 && trace) CKN(nova_sst_engine_set_trace(1));
  if (cfg->path == 2) CKN(nova_sst_engine_set_enabled(0));
  std::vector<Table> tabs(T);
  int rc = 0;
  for (int t = 0; t < T && !rc; t++) rc = make_table(tabs[t], cfg->blocks, cfg->seed * 1000 + 17 * t + 1, verify);
  const nova_callers_plain* pl = cfg->plain;
  hipStream_t pstream = nullptr;
  uint8_t *p_ok = nullptr, *p_lst = nullptr;
  uint32_t *p_bad = nullptr, *p_crc = nullptr;
  std::vector<uint8_t> h_ok, h_lst;
  std::vector<uint32_t> h_crc;
  if (!rc && pl) {
    if (hipStreamCreateWithFlags(&pstream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&p_ok, std::max<uint64_t>(1, pl->v_n)) != hipSuccess ||
        hipMalloc(&p_lst, std::max<uint64_t>(1, pl->l_n)) != hipSuccess ||
        hipMalloc(&p_bad, 8) != hipSuccess || hipMalloc(&p_crc, 4 * std::max<uint64_t>(1, pl->b_n)) != hipSuccess)
      rc = NOVA_E_NOMEM;
    h_ok.resize(pl->v_n);
    h_lst.resize(pl->l_n);
    h_crc.resize(pl->b_n);
  }
  if (rc) {
    for (auto& tb : tabs) free_table(tb);
    return rc;
  }

  auto call = [&](Table& tb, uint64_t i) -> int {
    const uint64_t set = i % tb.sets;
    if (cfg->path != 0) {  // host-synchronous: returns with the results written
      if (verify)
        return nova_sst_queue_verify_blocks(tb.img, tb.offs, tb.lens, tb.n, tb.ok + (uint64_t)set * tb.n,
                                            tb.bad + i % kCounters, tb.stream);
      return nova_sst_queue_write_trailers(tb.img, tb.offs, tb.lens, tb.n, 0, tb.stream);
    }
    int r = verify ? nova_sstable_verify_blocks(tb.img, tb.offs, tb.lens, tb.n, tb.ok + (uint64_t)set * tb.n,
                                                tb.bad + i % kCounters, tb.stream)
                   : nova_sstable_write_trailers(tb.img, tb.offs, tb.lens, tb.n, 0, tb.stream);
    return r ? r : (int)hipStreamSynchronize(tb.stream);
  };

  // plain-call thread state
  struct PStat {
    std::vector<double> lat[3];
    uint64_t bad[3] = {0, 0, 0};
    int rc = 0;
  } ps;

  std::atomic<int> ready{0};
  std::atomic<bool> go{false}, stop{false};
  Clock::time_point t_start{};  // the window opens (written before go)
  const double window = cfg->secs;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) {
    th.emplace_back([&, t] {
      Table& tb = tabs[t];
      tb.calls.reserve(1 << 17);
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      while (!stop.load(std::memory_order_relaxed)) {
        const auto a = Clock::now();
        const int r = call(tb, tb.ncalls);
        const auto b = Clock::now();
        if (r) {
          tb.rc = r;
          break;
        }
        tb.ncalls++;
        Call cl{std::chrono::duration<double>(a - t_start).count(), std::chrono::duration<double>(b - t_start).count(), {}};
        if (cfg->path == 1) (void)nova_sst_engine_last_call(cl.lc, 8);
        tb.calls.push_back(cl);
      }
    });
  }
  if (pl) {
    th.emplace_back([&] {
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (uint64_t k = 0; !stop.load(std::memory_order_relaxed); k++) {
        const int op = (int)(k % 3);
        if ((op == 0 && !pl->v_n) || (op == 1 && !pl->l_n) || (op == 2 && !pl->b_n)) continue;
        if (hipMemsetAsync(p_bad, 0, 8, pstream) != hipSuccess || hipStreamSynchronize(pstream) != hipSuccess) {
          ps.rc = NOVA_E_NODEV;
          break;
        }
        const auto a = Clock::now();
        int r = 0;
        if (op == 0)
          r = nova_sstable_verify_blocks(pl->v_img, pl->v_offs, pl->v_lens, pl->v_n, p_ok, p_bad, pstream);
        else if (op == 1)
          r = nova_log_verify_records(pl->l_img, pl->l_len, pl->l_offs, pl->l_n, p_lst, p_bad, pstream);
        else
          r = nova_crc32c_batch(pl->b_img, pl->b_offs, pl->b_lens, nullptr, p_crc, pl->b_n, 0, pstream);
        if (!r) r = (int)hipStreamSynchronize(pstream);
        const auto b = Clock::now();
        if (r) {
          ps.rc = r;
          break;
        }
        const double t0 = std::chrono::duration<double>(a - t_start).count();
        const double t1 = std::chrono::duration<double>(b - t_start).count();
        if (t0 >= 0 && t1 <= window) ps.lat[op].push_back((t1 - t0) * 1e6);
        // check (outside the timed call)
        uint32_t nb = 0;
        bool good = hipMemcpy(&nb, p_bad, 4, hipMemcpyDeviceToHost) == hipSuccess;
        if (op == 0) {
          good = good && hipMemcpy(h_ok.data(), p_ok, pl->v_n, hipMemcpyDeviceToHost) == hipSuccess &&
                 nb == pl->v_expect_bad && !memcmp(h_ok.data(), pl->v_expect_ok, pl->v_n);
        } else if (op == 1) {
          good = good && hipMemcpy(h_lst.data(), p_lst, pl->l_n, hipMemcpyDeviceToHost) == hipSuccess &&
                 nb == pl->l_expect_bad && !memcmp(h_lst.data(), pl->l_expect, pl->l_n);
        } else {
          good = good && hipMemcpy(h_crc.data(), p_crc, 4 * pl->b_n, hipMemcpyDeviceToHost) == hipSuccess &&
                 !memcmp(h_crc.data(), pl->b_expect, 4 * pl->b_n);
        }
        if (!good) ps.bad[op]++;
        if (pl->gap_us > 0) std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(pl->gap_us));
      }
    });
  }
  const int nthreads = (int)th.size();
  while (ready.load() < nthreads) std::this_thread::yield();
  uint64_t c0[NOVA_ENGINE_COUNTERS] = {}, c1[NOVA_ENGINE_COUNTERS] = {};
  uint64_t thr0 = 0, thr_us0 = 0, thr1 = 0, thr_us1 = 0;
  t_start = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(cfg->warm_s));
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_until(t_start);
  (void)nova_sst_engine_counters(c0, NOVA_ENGINE_COUNTERS);
  const bool have_cpu = read_cpu_stat(&thr0, &thr_us0);
  std::this_thread::sleep_until(t_start + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(window)));
  (void)nova_sst_engine_counters(c1, NOVA_ENGINE_COUNTERS);
  if (have_cpu) read_cpu_stat(&thr1, &thr_us1);
  stop.store(true);
  for (auto& x : th) x.join();

  // ---- results -----------------------------------------------------------
  std::vector<double> lat;
  double bytes = 0;
  uint64_t calls_in = 0, total_calls = 0;
  std::vector<std::pair<double, double>> slow;  // (latency us, start s)
  std::vector<std::pair<double, const Call*>> slowc;  // (latency us, call)
  for (auto& tb : tabs) {
    if (tb.rc && !rc) rc = tb.rc;
    total_calls += tb.ncalls;
    for (const Call& c : tb.calls) {
      if (c.t1 > 0 && c.t1 <= window) bytes += (double)tb.algo_bytes;  // completions inside the window
      if (c.t0 >= 0 && c.t1 <= window) {
        lat.push_back((c.t1 - c.t0) * 1e6);
        slow.push_back({(c.t1 - c.t0) * 1e6, c.t0});
        slowc.push_back({(c.t1 - c.t0) * 1e6, &c});
        calls_in++;
      }
    }
  }
  if (ps.rc && !rc) rc = ps.rc;
  // every call's result
  bool verified = rc == 0;
  uint64_t wrong = 0, checked_sets = 0;
  for (auto& tb : tabs) {
    if (!verified) break;
    if (verify) {
      std::vector<uint32_t> bad(kCounters);
      if (hipMemcpy(bad.data(), tb.bad, 4 * kCounters, hipMemcpyDeviceToHost) != hipSuccess) {
        verified = false;
        break;
      }
      // call i counted one mismatch into counter i % kCounters
      for (uint64_t i = 0; i < std::min<uint64_t>(tb.ncalls, kCounters); i++)
        if (bad[i] != (tb.ncalls - i + kCounters - 1) / kCounters) wrong++;
      // every flag set a call wrote (each call its own while calls <= sets)
      const uint64_t used = std::min<uint64_t>(tb.ncalls, tb.sets);
      if (used) {
        unsigned long long* dw = nullptr;
        unsigned long long hw = 0;
        if (hipMalloc(&dw, 8) != hipSuccess || hipMemset(dw, 0, 8) != hipSuccess) {
          verified = false;
          (void)hipFree(dw);
          break;
        }
        hipLaunchKernelGGL(check_flag_sets, dim3((uint32_t)used), dim3(256), 0, 0, tb.ok, tb.n, used, tb.victim, dw);
        const bool okc = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                         hipMemcpy(&hw, dw, 8, hipMemcpyDeviceToHost) == hipSuccess;
        (void)hipFree(dw);
        if (!okc) {
          verified = false;
          break;
        }
        wrong += hw;
      }
      checked_sets += used;
    } else {
      std::vector<uint8_t> img(tb.bytes);
      if (hipMemcpy(img.data(), tb.img, tb.bytes, hipMemcpyDeviceToHost) != hipSuccess) {
        verified = false;
        break;
      }
      if (tb.ncalls && memcmp(img.data(), tb.expect_img.data(), tb.bytes)) wrong++;
    }
  }
  verified = verified && wrong == 0 && ps.bad[0] + ps.bad[1] + ps.bad[2] == 0;
  std::sort(lat.begin(), lat.end());
  std::sort(slow.begin(), slow.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  std::string sl = "[";
  for (size_t i = 0; i < slow.size() && i < 5; i++) {
    char b[64];
    snprintf(b, sizeof b, "%s[%.1f, %.4f]", i ? ", " : "", slow[i].first, slow[i].second);
    sl += b;
  }
  sl += "]";
  // the slowest engine calls, where their host time went (us): lock wait,
  // lock held, completion wait, sleeps, relaunches in the wait, spun at the end
  std::sort(slowc.begin(), slowc.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  std::string sd = "[";
  for (size_t i = 0; cfg->path == 1 && i < slowc.size() && i < 5; i++) {
    const uint64_t* l = slowc[i].second->lc;
    char b[256];
    snprintf(b, sizeof b, "%s{\"us\": %.1f, \"at_s\": %.4f, \"lock_us\": %.1f, \"held_us\": %.1f, \"wait_us\": %.1f, "
             "\"sleeps\": %llu, \"relaunched\": %llu, \"spun\": %llu}", i ? ", " : "", slowc[i].first,
             slowc[i].second->t0, l[0] / 1e3, l[1] / 1e3, l[2] / 1e3, (unsigned long long)l[3],
             (unsigned long long)l[4], (unsigned long long)l[7]);
    sd += b;
  }
  sd += "]";
  std::string plain = "null";
  if (pl) {
    const char* names[3] = {"verify_blocks", "log_verify_records", "crc32c_batch"};
    plain = "{";
    for (int op = 0; op < 3; op++) {
      auto& v = ps.lat[op];
      std::sort(v.begin(), v.end());
      char b[256];
      snprintf(b, sizeof b, "%s\"%s\": {\"calls\": %zu, \"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, "
               "\"wrong\": %llu}", op ? ", " : "", names[op], v.size(), pct(v, 0.5), pct(v, 0.99),
               v.empty() ? 0.0 : v.back(), (unsigned long long)ps.bad[op]);
      plain += b;
    }
    plain += "}";
  }
  std::string eng = "{";
  const char* cn[NOVA_ENGINE_COUNTERS] = {"requests", "launches", "fallbacks", "running", "exits_idle",
                                          "exits_yield", "exits_stop", "exits_lost", "timeouts", "errors",
                                          "taken_back", "unsafe", "yield_waits", "yield_bumps", "broken",
                                          "backing_off", "exits_slice", "launch_us_max", "launch_slow",
                                          "poll_gap_us_max", "sleep_waits", "max_spinners",
                                          "ring_device", "host_marked_done", "waves", "storm_declined"};
  for (int i = 0; i < NOVA_ENGINE_COUNTERS; i++) {
    if (i == 3 || i == 14 || i == 15) continue;  // states, not counts
    char b[64];
    // launch_us_max, poll_gap_us_max, max_spinners, ring_device, waves: not counts
    snprintf(b, sizeof b, "%s\"%s\": %llu", eng.size() > 1 ? ", " : "", cn[i],
             (unsigned long long)(i == 17 || i == 19 || i == 21 || i == 22 || i == 24 ? c1[i] : c1[i] - c0[i]));
    eng += b;
  }
  eng += "}";
  std::string tr = "null";
  if (trace) {
    uint64_t tn = 0, dn = 0;
    double ts[5] = {}, td[11] = {};
    (void)nova_sst_engine_trace_stats(&tn, ts);
    (void)nova_sst_engine_trace_detail(&dn, td);
    char b[768];
    snprintf(b, sizeof b,
             "{\"requests\": %llu, \"host_submit_to_done_us\": %.2f, \"gpu_dispatch_to_first_chunk_us\": %.2f, "
             "\"gpu_first_to_last_chunk_us\": %.2f, \"gpu_dispatch_to_last_us\": %.2f, \"chunk0_us\": {\"seen\": %.2f, "
             "\"slot\": %.2f, \"body\": %.2f, \"drained\": %.2f, \"counted\": %.2f}, \"last_us\": {\"seen\": %.2f, "
             "\"slot\": %.2f, \"body\": %.2f, \"drained\": %.2f, \"counted\": %.2f, \"done\": %.2f}}",
             (unsigned long long)tn, ts[0], ts[1], ts[2], ts[3], td[2], td[0], td[3], td[4], td[5], td[6], td[7],
             td[8], td[9], td[10], td[1]);
    tr = b;
  }
  const double p50 = pct(lat, 0.5);
  const int n = snprintf(
      json, cap,
      "{\"op\": \"%s\", \"path\": \"%s\", \"threads\": %d, \"blocks_per_table\": %llu, \"table_bytes\": %llu, "
      "\"window_s\": %.3f, \"warm_s\": %.3f, \"calls\": %llu, \"calls_in_window\": %llu, "
      "\"aggregate_GBps\": %.1f, \"frac_of_8TBps\": %.4f, \"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, "
      "\"p999_us\": %.1f, \"max_us\": %.1f, \"max_over_p50\": %.2f, \"slowest_us_at_s\": %s, \"slowest_detail\": %s, "
      "\"engine\": %s, \"trace\": %s, \"cpu_throttled_periods\": %llu, \"cpu_throttled_us\": %llu, \"plain\": %s, "
      "\"wrong_results\": %llu, \"flag_sets_checked\": %llu, \"verified\": %s, \"rc\": %d}",
      verify ? "verify" : "trailers", cfg->path == 0 ? "direct" : cfg->path == 1 ? "engine" : "queue", T,
      (unsigned long long)cfg->blocks, (unsigned long long)(T ? tabs[0].algo_bytes : 0), window, cfg->warm_s,
      (unsigned long long)total_calls, (unsigned long long)calls_in, bytes / window / 1e9,
      bytes / window / 8e12, p50, pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.999), lat.empty() ? 0.0 : lat.back(),
      p50 > 0 ? (lat.empty() ? 0.0 : lat.back()) / p50 : 0.0, sl.c_str(), sd.c_str(), eng.c_str(), tr.c_str(),
      (unsigned long long)(thr1 - thr0), (unsigned long long)(thr_us1 - thr_us0), plain.c_str(),
      (unsigned long long)wrong, (unsigned long long)checked_sets, verified ? "true" : "false", rc);
  for (auto& tb : tabs) free_table(tb);
  if (pstream) {
    (void)nova_stream_release(pstream);
    (void)hipStreamDestroy(pstream);
  }
  (void)hipFree(p_ok);
  (void)hipFree(p_lst);
  (void)hipFree(p_bad);
  (void)hipFree(p_crc);
  return n < 0 || (size_t)n >= cap ? NOVA_E_INVAL : rc;
}

}  // extern "C"
