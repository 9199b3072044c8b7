// HBM read-ceiling probe (round 5): how fast can a kernel that only reads
// (and XOR-reduces) a 4 GiB device buffer go on one MI355X, by load shape?
//   U        16-B loads per lane in flight per iteration (4, 8, 16)
//   waves    per workgroup (4, 8, 12, 16); one workgroup per CU x occupancy
//   order    0: grid-stride over 1 KiB wave-lines, 1: each workgroup walks a
//            contiguous slab, 2: slabs assigned XCD-contiguously (workgroup
//            w on XCD w % 8 takes slab (w % 8) * (nwg / 8) + w / 8)
//   nt       non-temporal loads (1) or the default policy (0)
// Prints one JSON line per shape: best-of-10 time, GB/s, % of 8 TB/s.
// Build and run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/read_probe.hip -o tools/read_probe && ./tools/read_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u4;
typedef __attribute__((address_space(1))) const u4 gu4;

template <int U, bool NT>
__device__ __forceinline__ u4 ld(const u4* p) {
  if constexpr (NT) return __builtin_nontemporal_load((gu4*)p);
  return *(gu4*)p;
}

template <int U, bool NT>
__global__ void read_kernel(const u4* __restrict__ a, size_t n16, int order, unsigned* out) {
  const size_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const size_t nwg = gridDim.x;
  size_t wg = blockIdx.x;
  if (order == 2 && nwg % 8 == 0) wg = (blockIdx.x % 8) * (nwg / 8) + blockIdx.x / 8;
  u4 acc = {0, 0, 0, 0};
  if (order == 0) {
    const size_t lines = n16 / 64, total_waves = nwg * nw;
    size_t w = wg * nw + wave;
    for (; w + (size_t)(U - 1) * total_waves < lines; w += (size_t)U * total_waves) {
      u4 v[U];
#pragma unroll
      for (int k = 0; k < U; k++) v[k] = ld<U, NT>(a + (w + (size_t)k * total_waves) * 64 + lane);
#pragma unroll
      for (int k = 0; k < U; k++) acc ^= v[k];
    }
    for (; w < lines; w += total_waves) acc ^= ld<U, NT>(a + w * 64 + lane);
  } else {
    const size_t lines = n16 / 64, per = (lines + nwg - 1) / nwg;
    const size_t l0 = wg * per, l1 = std::min(lines, l0 + per);
    size_t l = l0 + wave;
    for (; l + (size_t)(U - 1) * nw < l1; l += (size_t)U * nw) {
      u4 v[U];
#pragma unroll
      for (int k = 0; k < U; k++) v[k] = ld<U, NT>(a + (l + (size_t)k * nw) * 64 + lane);
#pragma unroll
      for (int k = 0; k < U; k++) acc ^= v[k];
    }
    for (; l < l1; l += nw) acc ^= ld<U, NT>(a + l * 64 + lane);
  }
  const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) out[blockIdx.x] = x;  // (keeps the loads; practically never stores)
}

template <int U, bool NT>
float run(const u4* a, size_t n16, int waves, int wgs_per_cu, int order, unsigned* out, int cus) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 grid(cus * wgs_per_cu), block(64 * waves);
  float best = 1e30f;
  for (int r = 0; r < 12; r++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((read_kernel<U, NT>), grid, block, 0, 0, a, n16, order, out);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r >= 2) best = std::min(best, ms);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

int main() {
  const size_t bytes = 4ull << 30, n16 = bytes / 16;
  u4* a = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) {
    std::printf("{\"error\": \"alloc\"}\n");
    return 1;
  }
  (void)hipMemset(a, 0x5a, bytes);
  (void)hipDeviceSynchronize();
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  auto rep = [&](const char* name, int U, int nt, int waves, int wpc, int order, float ms) {
    const double gbs = (double)bytes / (ms * 1e-3) / 1e9;
    std::printf("{\"probe\": \"%s\", \"U\": %d, \"nt\": %d, \"waves\": %d, \"wgs_per_cu\": %d, \"order\": %d, "
                "\"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
                name, U, nt, waves, wpc, order, ms, gbs, gbs / 8000.0);
    std::fflush(stdout);
  };
  for (int order = 0; order < 3; order++)
    for (int waves : {8, 12, 16})
      for (int wpc : {1, 2}) {
        if (waves * wpc > 32) continue;
        rep("read", 4, 1, waves, wpc, order, run<4, true>(a, n16, waves, wpc, order, out, cus));
        rep("read", 8, 1, waves, wpc, order, run<8, true>(a, n16, waves, wpc, order, out, cus));
        rep("read", 16, 1, waves, wpc, order, run<16, true>(a, n16, waves, wpc, order, out, cus));
        rep("read", 8, 0, waves, wpc, order, run<8, false>(a, n16, waves, wpc, order, out, cus));
      }
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
