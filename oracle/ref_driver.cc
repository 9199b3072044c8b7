// TEST INFRASTRUCTURE ONLY -- C-ABI wrapper around the UNMODIFIED reference
// util/crc32c.cc, compiled from /root/reference where it lies (recipe:
// oracle/Makefile target `ref`, output oracle/_ref/libref_crc32c.so, which is
// git-ignored but travels to the GPU box).  Nothing in the product links it.
//
// Used (a) to generate tests/golden/ vectors (oracle/gen_golden.py) and (b) as
// the "reference" kind of bench.py's cpu_baseline: the reference's own
// leveldb::crc32c::Value timed on the host cores, one std::thread per core on
// contiguous shards (BASELINE.md CPU plan).
#include <cstddef>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "util/crc32c.h"  // /root/reference/util/crc32c.h:17-40

extern "C" {

uint32_t ref_extend(uint32_t init, const char* data, size_t n) {
  return leveldb::crc32c::Extend(init, data, n);  // util/crc32c.cc:487
}
uint32_t ref_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }
uint32_t ref_mask(uint32_t crc) { return leveldb::crc32c::Mask(crc); }
uint32_t ref_unmask(uint32_t m) { return leveldb::crc32c::Unmask(m); }

void ref_batch(const char* base, const uint64_t* offsets, const uint32_t* lengths,
               const uint32_t* init_or_null, uint32_t* out, size_t n) {
  for (size_t i = 0; i < n; i++)
    out[i] = leveldb::crc32c::Extend(init_or_null ? init_or_null[i] : 0u,
                                     base + offsets[i], lengths[i]);
}

int ref_batch_strided_mt(const char* base, uint64_t stride, uint32_t len, size_t n,
                         uint32_t* out, int threads, int reps) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    size_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
    pool.emplace_back([=] {
      for (int r = 0; r < reps; r++)
        for (size_t i = lo; i < hi; i++)
          out[i] = leveldb::crc32c::Value(base + i * stride, len);
    });
  }
  for (auto& th : pool) th.join();
  return threads;
}

// benchmarks/db_bench.cc:635-652 Crc32c(): the reference's own throughput
// method -- Value() over one 4 KiB string of 'x' until total_bytes, 1 thread.
uint32_t ref_dbbench_crc32c(int64_t total_bytes) {
  const std::string data(4096, 'x');
  uint32_t crc = 0;
  for (int64_t bytes = 0; bytes < total_bytes; bytes += 4096)
    crc = leveldb::crc32c::Value(data.data(), data.size());
  return crc;
}

}  // extern "C"
