// Experiment (not product code): what does writing 1M 5-byte SSTable trailers
// cost, by store shape?  Image: 1M blocks of 4096+U[0,255] B, each followed by
// a 5-B trailer (the sst4k image of tools/bench_ops.py).  Variants of the
// second-pass scatter:
//   0  byte store + unaligned dword store (the product's trailer_scatter_kernel)
//   1  read the aligned 32-B sector(s) holding the trailer, patch, store whole
//      sectors (two dwordx4 stores per sector)
//   2  same with 64-B pieces
//   3  same with 128-B lines
//   4  five byte stores
// plus a plain nt read of the image (verify-like cost) and read + variant 0
// in the same launch order.  Times with hipEvents, median of 20.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/exp_scatter tools/exp_scatter.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void patch(uint8_t* lb, uint64_t base_a, uint64_t t, const uint8_t* tr) {
  for (int k = 0; k < 5; k++) {
    const uint64_t a = t + k;
    if (a >= base_a && a < base_a + 16) lb[a - base_a] = tr[k];
  }
}

template <int V>
__global__ void __launch_bounds__(256) scatter(uint8_t* base, const uint64_t* off, const uint32_t* sz,
                                              const uint32_t* crc, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t t = (uint64_t)base + off[i] + sz[i];
  const uint32_t m = crc[i];
  uint8_t tr[5] = {0, (uint8_t)m, (uint8_t)(m >> 8), (uint8_t)(m >> 16), (uint8_t)(m >> 24)};
  if constexpr (V == 0) {
    *(uint8_t*)t = 0;
    __builtin_memcpy((void*)(t + 1), &m, 4);
  } else if constexpr (V == 4) {
    for (int k = 0; k < 5; k++) ((uint8_t*)t)[k] = tr[k];
  } else if constexpr (V >= 10) {
    // write-only: whole aligned pieces of W bytes holding the trailer, no read
    // (garbage values: measures the store shape's HBM cost only)
    constexpr uint64_t W = V == 10 ? 16 : V == 11 ? 32 : 64;
    const uint64_t a0 = t & ~(W - 1), a1 = (t + 4) & ~(W - 1);
    const u32x4 v = {m, m, m, m};
    for (uint64_t a = a0; a <= a1; a += W)
#pragma unroll
      for (int k = 0; k < (int)(W / 16); k++) *(u32x4*)(a + 16 * k) = v;
  } else {
    constexpr uint64_t P = V == 1 ? 32 : V == 2 ? 64 : 128;
    const uint64_t a0 = t & ~(P - 1), a1 = (t + 4) & ~(P - 1);
    for (uint64_t a = a0; a <= a1; a += P) {
      // the 16-B pieces of the piece P that hold trailer bytes are patched;
      // all P bytes are rewritten
      u32x4 v[P / 16];
#pragma unroll
      for (int k = 0; k < (int)(P / 16); k++) v[k] = *(const u32x4*)(a + 16 * k);
#pragma unroll
      for (int k = 0; k < (int)(P / 16); k++) patch((uint8_t*)&v[k], a + 16 * k, t, tr);
#pragma unroll
      for (int k = 0; k < (int)(P / 16); k++) *(u32x4*)(a + 16 * k) = v[k];
    }
  }
}

__global__ void __launch_bounds__(256) readall(const uint8_t* base, uint64_t n16, uint32_t* sink) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += nth) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)(base + 16 * i));
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t n = 1 << 20;
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> sz(n), crc(n);
  uint64_t s = 88172645463325252ull, o = 0;
  for (uint64_t i = 0; i < n; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    sz[i] = 4096 + (uint32_t)(s & 255);
    off[i] = o;
    crc[i] = (uint32_t)(s >> 32);
    o += sz[i] + 5;
  }
  const uint64_t total = o + 256;
  uint8_t* d;
  uint64_t* doff;
  uint32_t *dsz, *dcrc, *sink;
  CK(hipMalloc(&d, total));
  CK(hipMemset(d, 0x5a, total));
  CK(hipMalloc(&doff, n * 8));
  CK(hipMalloc(&dsz, n * 4));
  CK(hipMalloc(&dcrc, n * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(doff, off.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsz, sz.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcrc, crc.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned g = (unsigned)((n + 255) / 256);
  auto run = [&](const char* name, auto launch) -> int {
    std::vector<float> ms;
    for (int it = 0; it < 40; it++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (it >= 20) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("{\"variant\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f}\n", name, ms[ms.size() / 2], ms[0]);
    return 0;
  };
  const uint64_t n16 = total / 16;
  run("read_image_nt", [&] { readall<<<2048, 256>>>(d, n16, sink); });
  run("scatter_byte_dword", [&] { scatter<0><<<g, 256>>>(d, doff, dsz, dcrc, n); });
  run("scatter_5bytes", [&] { scatter<4><<<g, 256>>>(d, doff, dsz, dcrc, n); });
  run("scatter_sector32", [&] { scatter<1><<<g, 256>>>(d, doff, dsz, dcrc, n); });
  run("scatter_piece64", [&] { scatter<2><<<g, 256>>>(d, doff, dsz, dcrc, n); });
  run("scatter_line128", [&] { scatter<3><<<g, 256>>>(d, doff, dsz, dcrc, n); });
  run("read+scatter_byte_dword", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<0><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+scatter_sector32", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<1><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+scatter_line128", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<3><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+write16_noread", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<10><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+write32_noread", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<11><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+write64_noread", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<12><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read+scatter_5bytes", [&] {
    readall<<<2048, 256>>>(d, n16, sink);
    scatter<4><<<g, 256>>>(d, doff, dsz, dcrc, n);
  });
  run("read_image_nt_again", [&] { readall<<<2048, 256>>>(d, n16, sink); });
  CK(hipDeviceSynchronize());
  return 0;
}
