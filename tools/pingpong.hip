// Host <-> GPU ping-pong latency probe (engine dispatch latency, round 5).
// One wave polls a flag word for the host's value k, then writes k back to a
// pinned host word; the host waits for the echo and sends k+1.  Flag word in
//   A: pinned host memory (the engine's ring until round 5), GPU polls over PCIe;
//   B: fine-grained device memory written by the host through the BAR (the
//      engine's ring since, crc32c_engine.hip EngIn).
// Build and run on the GPU box:
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/pingpong.hip -o tools/pingpong && ./tools/pingpong
// Every kernel spin is bounded (2 s of s_memrealtime), so the grid drains.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void pong(volatile uint64_t* flag, uint64_t* echo, uint32_t iters, uint32_t pipelined) {
  if (threadIdx.x != 0) return;
  const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 200000000ull;  // 2 s at 100 MHz
  for (uint32_t k = 1; k <= iters; k++) {
    for (;;) {
      const uint64_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v >= k) break;
      if (__builtin_amdgcn_s_memrealtime() > t_end) return;
    }
    __hip_atomic_store(echo, (uint64_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int run(const char* name, uint64_t* flag, uint64_t* echo, uint32_t iters) {
  volatile uint64_t* f = flag;
  volatile uint64_t* e = echo;
  *f = 0;
  *e = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, flag, echo, iters, 0u);
  CK(hipGetLastError());
  std::vector<double> us;
  us.reserve(iters);
  bool ok = true;
  for (uint32_t k = 1; k <= iters && ok; k++) {
    const auto t0 = std::chrono::steady_clock::now();
    *f = k;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    for (;;) {
      if (*e >= k) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        ok = false;
        break;
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipDeviceSynchronize());
  std::sort(us.begin() + 10, us.end());
  const size_t m = us.size() - 10;
  std::printf("{\"flag\": \"%s\", \"ok\": %s, \"iters\": %zu, \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f}\n",
              name, ok ? "true" : "false", m, us[10 + m / 2], us[10 + m / 10], us[10 + m * 9 / 10], us[10 + m * 99 / 100]);
  return ok ? 0 : 1;
}

int main() {
  const uint32_t iters = 20000;
  uint64_t *hflag = nullptr, *hecho = nullptr, *dflag = nullptr;
  CK(hipHostMalloc((void**)&hflag, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&hecho, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  int rc = run("pinned_host", hflag, hecho, iters);
  CK(hipExtMallocWithFlags((void**)&dflag, 4096, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, dflag));
  std::printf("{\"device_fine_grained\": \"%p\", \"host_ptr\": \"%p\"}\n", (void*)dflag, at.hostPointer);
  std::fflush(stdout);
  // the host stores through the BAR mapping (large BAR); a fault ends this process only
  rc |= run("device_fine_grained", dflag, hecho, iters);
  return rc;
}
