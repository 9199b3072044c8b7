// Concurrent per-SSTable callers: T host threads, each
// with its own HIP stream and its own device-resident SSTable image (n blocks
// of 4096+U[0,255] B with 5-B trailers, the sst4k layout), each calling
// nova_sstable_write_trailers or nova_sstable_verify_blocks on its table and
// waiting for it (hipStreamSynchronize): the way NovaLSM's compaction and
// read threads would call the library, one SSTable per call
// (ltc/stoc_file_client_impl.cpp:274-289 write side, table/table.cc:425-441
// read side).  Native threads, so the host cost measured is the library's,
// not an interpreter lock's.
//
// Prints one JSON line: aggregate algorithmic GB/s over all threads (verify:
// sum(len + 6) per block; trailers: sum(len + 5)), per-call latency p50/p99/max
// over every call of every thread, calls per thread.  Every verify call's
// result is checked (n_bad must stay 0; all ok flags set at the end).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/bin/concurrent_sst
//        tools/concurrent_sst.cpp -Lnovalsm_amd/lib -lnova_crc32c -Wl,-rpath,'$ORIGIN/../../novalsm_amd/lib' -lpthread
// Run:   tools/bin/concurrent_sst <verify|trailers> <threads> <blocks per table> <seconds>
//        [direct|queue|engine|engine_trace]   (nova_sst_queue_*: queue = the coalescing
//        queue, engine = the persistent engine; engine_trace: with its
//        per-request spans, nova_sst_engine_set_trace, printed as a second JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "nova_crc32c.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      std::exit(3);                                                                   \
    }                                                                                 \
  } while (0)
#define CKN(x)                                                                        \
  do {                                                                                \
    int r_ = (x);                                                                     \
    if (r_ != 0) {                                                                    \
      fprintf(stderr, "%s:%d nova rc %d\n", __FILE__, __LINE__, r_);                  \
      std::exit(3);                                                                   \
    }                                                                                 \
  } while (0)

using Clock = std::chrono::steady_clock;

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Table {
  hipStream_t stream;
  uint8_t* img;
  uint64_t* offs;
  uint32_t* lens;
  uint8_t* ok;
  uint32_t* bad;
  uint64_t algo_bytes;
  std::vector<double> lat_us;
};

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s <verify|trailers> <threads> <blocks> <seconds>\n", argv[0]);
    return 2;
  }
  const bool verify = !strcmp(argv[1], "verify");
  const int T = atoi(argv[2]);
  const size_t n = strtoull(argv[3], nullptr, 10);
  const double secs = atof(argv[4]);
  const bool trace = argc > 5 && !strcmp(argv[5], "engine_trace");
  const bool engine = trace || (argc > 5 && !strcmp(argv[5], "engine"));
  const bool queue = engine || (argc > 5 && !strcmp(argv[5], "queue"));
  if (T < 1 || T > 64 || n < 1 || n > (1u << 20) || secs <= 0) return 2;
  CKN(nova_device_init());
  CKN(nova_sst_engine_set_enabled(engine ? 1 : 0));
  CKN(nova_sst_engine_set_trace(trace ? 1 : 0));

  std::vector<Table> tabs(T);
  for (int t = 0; t < T; t++) {
    Table& tb = tabs[t];
    uint64_t s = 1000 + t;
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    uint64_t pos = 0, sum_len = 0;
    for (size_t i = 0; i < n; i++) {
      lens[i] = 4096 + (uint32_t)(splitmix(s) & 255);
      offs[i] = pos;
      pos += lens[i] + 5;
      sum_len += lens[i];
    }
    tb.algo_bytes = sum_len + n * (verify ? 6 : 5);
    CK(hipStreamCreateWithFlags(&tb.stream, hipStreamNonBlocking));
    CK(hipMalloc(&tb.img, pos + 64));
    CK(hipMalloc(&tb.offs, n * 8));
    CK(hipMalloc(&tb.lens, n * 4));
    CK(hipMalloc(&tb.ok, n));
    CK(hipMalloc(&tb.bad, 4));
    CK(hipMemcpy(tb.offs, offs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(tb.lens, lens.data(), n * 4, hipMemcpyHostToDevice));
    CKN(nova_fill_splitmix64(tb.img, pos + 64, 77 + t, 0, tb.stream));
    CKN(nova_sstable_write_trailers(tb.img, tb.offs, tb.lens, n, 0, tb.stream));
    CK(hipMemsetAsync(tb.bad, 0, 4, tb.stream));
    CK(hipStreamSynchronize(tb.stream));
  }

  auto call = [&](Table& tb) {
    if (queue) {  // host-synchronous: returns with the results written
      if (verify)
        CKN(nova_sst_queue_verify_blocks(tb.img, tb.offs, tb.lens, n, tb.ok, tb.bad, tb.stream));
      else
        CKN(nova_sst_queue_write_trailers(tb.img, tb.offs, tb.lens, n, 0, tb.stream));
      return;
    }
    if (verify)
      CKN(nova_sstable_verify_blocks(tb.img, tb.offs, tb.lens, n, tb.ok, tb.bad, tb.stream));
    else
      CKN(nova_sstable_write_trailers(tb.img, tb.offs, tb.lens, n, 0, tb.stream));
    CK(hipStreamSynchronize(tb.stream));
  };
  for (auto& tb : tabs)  // warm: per-stream claim slots, code objects
    for (int k = 0; k < 20; k++) call(tb);

  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  Clock::time_point t_end_all[64];
  Clock::time_point t_start;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) {
    th.emplace_back([&, t] {
      Table& tb = tabs[t];
      tb.lat_us.reserve(1 << 20);
      ready++;
      while (!go.load(std::memory_order_acquire)) {
      }
      const auto deadline = t_start + std::chrono::duration<double>(secs);
      Clock::time_point now = Clock::now();
      while (now < deadline) {
        const auto t0 = now;
        call(tb);
        now = Clock::now();
        tb.lat_us.push_back(std::chrono::duration<double, std::micro>(now - t0).count());
      }
      t_end_all[t] = now;
    });
  }
  while (ready.load() < T) {
  }
  t_start = Clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  Clock::time_point t_end = t_start;
  for (int t = 0; t < T; t++) t_end = std::max(t_end, t_end_all[t]);
  const double wall = std::chrono::duration<double>(t_end - t_start).count();

  std::vector<double> all;
  double bytes = 0;
  size_t min_calls = SIZE_MAX, max_calls = 0;
  bool good = true;
  for (auto& tb : tabs) {
    bytes += (double)tb.algo_bytes * tb.lat_us.size();
    all.insert(all.end(), tb.lat_us.begin(), tb.lat_us.end());
    min_calls = std::min(min_calls, tb.lat_us.size());
    max_calls = std::max(max_calls, tb.lat_us.size());
    if (verify) {
      uint32_t bad = 0;
      std::vector<uint8_t> ok(n);
      CK(hipMemcpy(&bad, tb.bad, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ok.data(), tb.ok, n, hipMemcpyDeviceToHost));
      good = good && bad == 0 && std::all_of(ok.begin(), ok.end(), [](uint8_t v) { return v == 1; });
    }
  }
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  uint64_t qb = 0, qr = 0, qmax = 0, er = 0, el = 0, ef = 0;
  int erun = 0;
  CKN(nova_sst_queue_stats(&qb, &qr, &qmax));
  CKN(nova_sst_engine_stats(&er, &el, &ef, &erun));
  uint64_t tn = 0;
  double ts[5] = {0, 0, 0, 0, 0};
  CKN(nova_sst_engine_trace_stats(&tn, ts));
  uint64_t dn = 0;
  double td[11] = {};
  CKN(nova_sst_engine_trace_detail(&dn, td));
  if (trace)
    printf("{\"trace_requests\": %llu, \"host_submit_to_done_us\": %.2f, \"gpu_dispatch_to_first_chunk_us\": %.2f, "
           "\"gpu_first_to_last_chunk_us\": %.2f, \"gpu_dispatch_to_last_us\": %.2f, \"host_max_us\": %.1f, "
           "\"detail_requests\": %llu, \"chunk0_us\": {\"seen\": %.2f, \"slot\": %.2f, \"body\": %.2f, "
           "\"drained\": %.2f, \"counted\": %.2f}, \"last_us\": {\"seen\": %.2f, \"slot\": %.2f, "
           "\"body\": %.2f, \"drained\": %.2f, \"counted\": %.2f, \"done\": %.2f}}\n",
           (unsigned long long)tn, ts[0], ts[1], ts[2], ts[3], ts[4], (unsigned long long)dn, td[2], td[0], td[3],
           td[4], td[5], td[6], td[7], td[8], td[9], td[10], td[1]);
  printf("{\"op\": \"%s\", \"path\": \"%s\", \"queue_batches\": %llu, \"queue_requests\": %llu, "
         "\"queue_max_tables\": %llu, \"engine_requests\": %llu, \"engine_launches\": %llu, "
         "\"engine_fallbacks\": %llu, \"threads\": %d, \"blocks_per_table\": %zu, \"table_bytes\": %llu, "
         "\"calls\": %zu, \"calls_per_thread_min\": %zu, \"calls_per_thread_max\": %zu, "
         "\"wall_s\": %.3f, \"aggregate_GBps\": %.1f, \"frac_of_8TBps\": %.4f, "
         "\"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, \"verified\": %s}\n",
         verify ? "verify" : "trailers", trace ? "engine_trace" : engine ? "engine" : queue ? "queue" : "direct",
         (unsigned long long)qb,
         (unsigned long long)qr, (unsigned long long)qmax, (unsigned long long)er, (unsigned long long)el,
         (unsigned long long)ef, T, n, (unsigned long long)tabs[0].algo_bytes, all.size(),
         min_calls, max_calls, wall, bytes / wall / 1e9, bytes / wall / 8e12, pct(0.50), pct(0.99),
         all.back(), good ? "true" : "false");
  for (auto& tb : tabs) {
    CKN(nova_stream_release(tb.stream));
    CK(hipStreamDestroy(tb.stream));
    CK(hipFree(tb.img));
    CK(hipFree(tb.offs));
    CK(hipFree(tb.lens));
    CK(hipFree(tb.ok));
    CK(hipFree(tb.bad));
  }
  return good ? 0 : 1;
}
