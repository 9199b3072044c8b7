// Log sort pre-pass probe (round 6): where do log_sort_kernel's ~31 us per
// launch go on a 2M-record log (U[1,4096] payloads, 256-record windows)?
// A standalone copy of the product kernel's structure (crc32c_device.hip
// log_sort_kernel, keymode 0) with one piece changed per variant:
//   0 the product's shape: 256 threads per window, one thread's serial prefix
//   1 64 threads per window (one wave takes four records per lane)
//   2 no prefix (bins left as counts: wrong order, timing only)
//   3 no LDS atomics (key computed, perm[i] = i: timing only)
//   4 key math in 32 bits with a shift for the power-of-two line (no 64-bit divide)
//   5 the prefix as a wave-parallel scan (wave 0, shuffles) instead of one thread
// Prints one JSON line per variant: best-of-10 kernel time from events.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/logsort_probe.hip -o tools/bin/logsort_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint32_t kWin = 1024, kBins = 288, kLogBlock = 32768;

__device__ __forceinline__ uint64_t block_end(uint64_t o, uint64_t len) {
  const uint64_t e = (o / kLogBlock + 1) * kLogBlock;
  return e < len ? e : len;
}

template <int V>
__global__ void __launch_bounds__(256) sort_kernel(uint64_t base, const uint64_t* __restrict__ offs, uint64_t n,
                                                   uint64_t buf_len, uint32_t line, uint32_t win,
                                                   uint32_t* __restrict__ perm) {
  __shared__ uint32_t cnt[kBins + 64];
  const uint32_t nt = blockDim.x;
  const uint64_t w0 = (uint64_t)blockIdx.x * win;
  for (uint32_t b = threadIdx.x; b < kBins; b += nt) cnt[b] = 0;
  __syncthreads();
  constexpr int kPer = kWin / 64;
  uint32_t key[kPer];
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint32_t j = threadIdx.x + nt * k;
    const uint64_t i = w0 + j;
    key[k] = 0;
    if (j < win && i < n) {
      const uint64_t o = offs[i];
      const uint64_t be = block_end(o, buf_len);
      uint64_t e = i + 1 < n ? offs[i + 1] : be;
      if (e > be || e < o) e = be;
      const uint64_t u0 = base + o + 6, u1 = base + (e > o + 7 ? e : o + 7);
      const uint64_t E = u1 & ~15ull;
      const uint64_t first = (u0 & ~15ull) & ~(uint64_t)(line - 1);
      const uint64_t Le = (E + line - 1) & ~(uint64_t)(line - 1);
      uint64_t S;
      if constexpr (V == 4) {
        const uint32_t sh = 31 - __builtin_clz(line);
        S = Le > first ? (uint32_t)((Le - first) >> sh) : 1;
      } else {
        S = Le > first ? (Le - first) / line : 1;
      }
      key[k] = S < kBins ? (uint32_t)S : kBins - 1;
      if constexpr (V != 3) atomicAdd(&cnt[key[k]], 1u);
    }
  }
  __syncthreads();
  if constexpr (V == 5) {
    // exclusive prefix in descending key order: reversed bin r = kBins-1-b;
    // lane l of wave 0 sums reversed bins [5l, 5l+5) (320 >= 288), one wave
    // scan of those sums, then writes its five bins' starts
    if (threadIdx.x < 64) {
      const uint32_t l = threadIdx.x;
      uint32_t c[5], sum = 0;
#pragma unroll
      for (int q = 0; q < 5; q++) {
        const int r = (int)(5 * l) + q;
        c[q] = r < (int)kBins ? cnt[kBins - 1 - r] : 0u;
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
        if (r < (int)kBins) cnt[kBins - 1 - r] = run;
        run += c[q];
      }
    }
  } else if constexpr (V != 2) {
    if (threadIdx.x == 0) {
      uint32_t run = 0;
      for (int b = kBins - 1; b >= 0; b--) {
        const uint32_t c = cnt[b];
        cnt[b] = run;
        run += c;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint32_t j = threadIdx.x + nt * k;
    const uint64_t i = w0 + j;
    if (j < win && i < n) {
      if constexpr (V == 3)
        perm[i] = (uint32_t)i;
      else
        perm[w0 + (atomicAdd(&cnt[key[k]], 1u) % win)] = (uint32_t)i;
    }
  }
}

int main() {
  // 2M records of 7 + U[1,4096] bytes, packed into 32 KiB log blocks
  const uint64_t n = 2u << 20;
  std::vector<uint64_t> offs(n);
  uint64_t pos = 0, x = 88172645463325252ull;
  for (uint64_t i = 0; i < n; i++) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const uint64_t len = 7 + 1 + x % 4096;
    const uint64_t left = kLogBlock - pos % kLogBlock;
    if (left < 7) pos += left;  // block trailer
    offs[i] = pos;
    pos += len;  // (a record runs on past its block: the key clamps, timing only)
  }
  const uint64_t total = pos;
  uint64_t* d_offs = nullptr;
  uint32_t* d_perm = nullptr;
  if (hipMalloc(&d_offs, n * 8) != hipSuccess || hipMalloc(&d_perm, n * 4) != hipSuccess) return 1;
  (void)hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const uint32_t win = 256, line = 128;
  const uint64_t wgs = (n + win - 1) / win;
  auto run = [&](auto kern, int v, uint32_t threads) {
    float best = 1e9f;
    for (int it = 0; it < 11; it++) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kern, dim3(wgs), dim3(threads), 0, 0, (uint64_t)0x7f0000000000ull, d_offs, n, total,
                         line, win, d_perm);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;
    }
    printf("{\"variant\": %d, \"threads\": %u, \"windows\": %llu, \"us\": %.2f}\n", v, threads,
           (unsigned long long)wgs, best * 1000.0);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; rep++) {
    run(sort_kernel<0>, 0, 256);
    run(sort_kernel<0>, 1, 64);
    run(sort_kernel<2>, 2, 256);
    run(sort_kernel<3>, 3, 256);
    run(sort_kernel<4>, 4, 256);
    run(sort_kernel<5>, 5, 256);
    run(sort_kernel<5>, 51, 64);
  }
  (void)hipFree(d_offs);
  (void)hipFree(d_perm);
  return 0;
}
