// Lane-stream probe (round 6): can ONE LANE stream its own contiguous run of a
// log image fast enough?  A design for short log records that gives every lane
// a run of whole records (no rounds, no padding) reads 64 lanes' runs at once:
// each 16-B load instruction touches 64 different lines.  This probe measures
// that access shape on a 4 GiB buffer, with and without a CRC-like compute
// load per 16 B (16 v_perm + 16 ds_read_b32 from a 128 KiB LDS image + 8
// three-input xors: the rounds kernel's swath), against the coalesced shape.
//   run      bytes per lane (4-8 KiB): a G-lane stream's run is G times that
//   steps    16-B loads per lane per step (4: 64 B), two steps in flight
//   waves    per workgroup (8, 12); one workgroup per CU (LDS image)
//   nt       non-temporal loads (1) or the default policy (0)
//   compute  the swath's lookups on every 16 B (1) or none (0); with the
//            argument "depth": the lookups K times per piece and 1 or 2 steps
//            of loads in flight, printed as compute = K (one step in flight)
//            or 10 K + 2 (two steps): 1 / 12, 2 / 22, 3 / 32
// Prints one JSON line per shape: best-of-5 time, GB/s, % of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lanestream_probe.hip -o tools/bin/lanestream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u4;
typedef __attribute__((address_space(1))) const u4 gu4;

template <bool NT>
__device__ __forceinline__ u4 ld(const u4* p) {
  if constexpr (NT) return __builtin_nontemporal_load((gu4*)p);
  return *(gu4*)p;
}

__device__ __forceinline__ unsigned lds32(unsigned a) {
  return *reinterpret_cast<__attribute__((address_space(3))) const unsigned*>(a);
}

// one 16-B piece into 4 stream registers: 16 lookups (bank-replicated image)
__device__ __forceinline__ void swath(unsigned& c0, unsigned& c1, unsigned& c2, unsigned& c3, u4 d,
                                      unsigned lo) {
#define A4(c, p)                                                     \
  const unsigned p##0 = __builtin_amdgcn_perm(c, lo, 0x0c020400u);   \
  const unsigned p##1 = __builtin_amdgcn_perm(c, lo | 128u, 0x0c020500u); \
  const unsigned p##2 = __builtin_amdgcn_perm(c, lo | 0x10000u, 0x0c020600u); \
  const unsigned p##3 = __builtin_amdgcn_perm(c, lo | 0x10080u, 0x0c020700u);
  A4(c0, a) A4(c1, b) A4(c2, e) A4(c3, f)
#undef A4
  const unsigned ta0 = lds32(a0), ta1 = lds32(a1), ta2 = lds32(a2), ta3 = lds32(a3);
  const unsigned tb0 = lds32(b0), tb1 = lds32(b1), tb2 = lds32(b2), tb3 = lds32(b3);
  const unsigned te0 = lds32(e0), te1 = lds32(e1), te2 = lds32(e2), te3 = lds32(e3);
  const unsigned tf0 = lds32(f0), tf1 = lds32(f1), tf2 = lds32(f2), tf3 = lds32(f3);
  __builtin_amdgcn_sched_barrier(0);
  c0 = ta0 ^ ta1 ^ ta2 ^ ta3 ^ d.x;
  c1 = tb0 ^ tb1 ^ tb2 ^ tb3 ^ d.y;
  c2 = te0 ^ te1 ^ te2 ^ te3 ^ d.z;
  c3 = tf0 ^ tf1 ^ tf2 ^ tf3 ^ d.w;
}

// shape G (1, 2, 4, 8): 64 / G streams per wave, lane q of a G-lane group
// reading piece q of each 16G-byte swath of its group's run (the rounds
// kernel's shape at G lanes per record); shape 64: coalesced wave-lines
// (1 KiB per instruction, the stream kernel's shape).  K: the swath's lookups
// K times per piece (K = 3: about the rounds kernel's issue work per step at
// 2 lanes); DEPTH: steps of loads in flight while a step folds (1 or 2).
template <bool NT, bool COMPUTE, int K = 1, int DEPTH = 1>
__global__ void __launch_bounds__(768) probe_kernel(const u4* __restrict__ a, size_t n16, size_t run16,
                                                    int shape, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  for (unsigned i = threadIdx.x * 16; i < 131072; i += blockDim.x * 16)
    *reinterpret_cast<__attribute__((address_space(3))) u4*>(i) = u4{i, i * 3u, i * 5u, i * 7u};
  __syncthreads();
  const size_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const size_t gw = (size_t)blockIdx.x * nw + wave, tw = (size_t)gridDim.x * nw;
  const unsigned lo = (unsigned)(lane & 31) << 2;
  unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  u4 acc = {0, 0, 0, 0};
  // a wave's unit of work: 64 runs (lane streams) or 64 * run16 pieces as
  // wave-lines (coalesced); units are strided over the grid's waves
  const size_t unit16 = 64 * run16;
  const size_t units = n16 / unit16;
  auto fold = [&](u4 y0, u4 y1, u4 y2, u4 y3) {
    if constexpr (COMPUTE) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        swath(c0, c1, c2, c3, y0, lo);
        swath(c0, c1, c2, c3, y1, lo);
        swath(c0, c1, c2, c3, y2, lo);
        swath(c0, c1, c2, c3, y3, lo);
      }
    } else {
      acc ^= y0 ^ y1 ^ y2 ^ y3;
    }
  };
  for (size_t u = gw; u < units; u += tw) {
    const u4* base = a + u * unit16;
    const size_t G = (size_t)shape, grp = lane / G, q = lane % G;
    auto addr = [&](size_t k) -> const u4* {  // the lane's k-th piece (k < run16)
      return base + grp * (run16 * G) + k * G + q;
    };
    u4 x0 = ld<NT>(addr(0)), x1 = ld<NT>(addr(1)), x2 = ld<NT>(addr(2)), x3 = ld<NT>(addr(3));
    if constexpr (DEPTH == 1) {
      for (size_t k = 4; k <= run16; k += 4) {
        u4 y0 = x0, y1 = x1, y2 = x2, y3 = x3;
        if (k < run16) {
          x0 = ld<NT>(addr(k));
          x1 = ld<NT>(addr(k + 1));
          x2 = ld<NT>(addr(k + 2));
          x3 = ld<NT>(addr(k + 3));
        }
        fold(y0, y1, y2, y3);
      }
    } else {  // two steps in flight: fold step k-8 while k-4 and k are loading
      u4 z0 = ld<NT>(addr(4)), z1 = ld<NT>(addr(5)), z2 = ld<NT>(addr(6)), z3 = ld<NT>(addr(7));
      for (size_t k = 8; k <= run16 + 4; k += 4) {
        u4 y0 = x0, y1 = x1, y2 = x2, y3 = x3;
        x0 = z0, x1 = z1, x2 = z2, x3 = z3;
        if (k < run16) {
          z0 = ld<NT>(addr(k));
          z1 = ld<NT>(addr(k + 1));
          z2 = ld<NT>(addr(k + 2));
          z3 = ld<NT>(addr(k + 3));
        }
        fold(y0, y1, y2, y3);
      }
    }
  }
  const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w ^ c0 ^ c1 ^ c2 ^ c3;
  if (x == 0x9e3779b9u) out[blockIdx.x] = x;
}

// Span shape (round 6, session 2): each lane owns a CONTIGUOUS 64-B span of
// the wave's 4 KiB unit (lane-strided 16-B loads: each instruction touches the
// unit's 64 lines, the four together read them whole), the next unit's loads
// in flight while a unit computes.  The compute is the span design's for short
// log records: CHAINS sequential word chains per lane (16 / CHAINS dependent
// 4-lookup steps each, a reset/mask select per word), and, with SCAN, a
// 6-level cross-lane carry scan per unit (one 4-lookup operator and a
// shuffle per level) -- the cost of giving each record crossing a span its
// carry-in.  No CRC is checked: timing only.
__device__ __forceinline__ unsigned wstep(unsigned c, unsigned w, unsigned lo) {
  const unsigned x = c ^ w;
  const unsigned a0 = __builtin_amdgcn_perm(x, lo, 0x0c020400u);
  const unsigned a1 = __builtin_amdgcn_perm(x, lo | 128u, 0x0c020500u);
  const unsigned a2 = __builtin_amdgcn_perm(x, lo | 0x10000u, 0x0c020600u);
  const unsigned a3 = __builtin_amdgcn_perm(x, lo | 0x10080u, 0x0c020700u);
  return lds32(a0) ^ lds32(a1) ^ lds32(a2) ^ lds32(a3);
}
template <bool NT, int CHAINS, bool SCAN>
__global__ void __launch_bounds__(768) span_kernel(const u4* __restrict__ a, size_t n16, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  for (unsigned i = threadIdx.x * 16; i < 131072; i += blockDim.x * 16)
    *reinterpret_cast<__attribute__((address_space(3))) u4*>(i) = u4{i, i * 3u, i * 5u, i * 7u};
  __syncthreads();
  const size_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const size_t gw = (size_t)blockIdx.x * nw + wave, tw = (size_t)gridDim.x * nw;
  const unsigned lo = (unsigned)(lane & 31) << 2;
  const size_t units = n16 / 256;
  unsigned acc = 0, ev = (unsigned)lane * 0x9e3779b9u;
  size_t u = gw;
  if (u >= units) return;
  const u4* p = a + u * 256 + lane * 4;
  u4 x0 = ld<NT>(p), x1 = ld<NT>(p + 1), x2 = ld<NT>(p + 2), x3 = ld<NT>(p + 3);
  for (; u < units; u += tw) {
    const u4 y0 = x0, y1 = x1, y2 = x2, y3 = x3;
    if (u + tw < units) {
      const u4* q = a + (u + tw) * 256 + lane * 4;
      x0 = ld<NT>(q), x1 = ld<NT>(q + 1), x2 = ld<NT>(q + 2), x3 = ld<NT>(q + 3);
    }
    const unsigned w[16] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w,
                            y2.x, y2.y, y2.z, y2.w, y3.x, y3.y, y3.z, y3.w};
    unsigned c[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; k++) c[k] = 0;
    constexpr int L = 16 / CHAINS;
#pragma unroll
    for (int i = 0; i < L; i++) {
#pragma unroll
      for (int k = 0; k < CHAINS; k++) {
        // per-word events: a reset (record start) and a keep mask, as selects
        const unsigned bit = (ev >> ((k * L + i) & 31)) & 1u;
        const unsigned wm = bit ? (w[k * L + i] & 0xffff0000u) : w[k * L + i];
        const unsigned cin = bit ? 0xffffffffu : c[k];
        acc ^= bit ? c[k] : 0u;  // the ended record's state
        c[k] = wstep(cin, wm, lo);
      }
    }
    unsigned v = c[0];
#pragma unroll
    for (int k = 1; k < CHAINS; k++) v = wstep(v, c[k], lo);
    if constexpr (SCAN) {
#pragma unroll
      for (int lvl = 0; lvl < 6; lvl++) {
        const int d = 1 << lvl;
        const unsigned o = __shfl_up(v, d);
        const unsigned sh = wstep(o, 0u, lo);
        v = ((int)lane >= d && !(ev & (1u << lvl))) ? (v ^ sh) : v;
      }
    }
    acc ^= v;
    ev = ev * 1664525u + 1013904223u;
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = 4ull << 30, n16 = bytes / 16;
  u4* a = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
  (void)hipMemset(a, 0x5a, bytes);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](auto kern, int shape, size_t run_b, int waves, int nt, int comp) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    float best = 1e9f;
    for (int it = 0; it < 6; it++) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * waves), 131072, 0, a, n16, run_b / 16, shape, out);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;  // (first launch: warm-up)
    }
    const double gbs = (double)bytes / (best * 1e-3) / 1e9;
    printf("{\"lanes_per_stream\": %d, \"run_bytes_per_lane\": %zu, \"waves\": %d, \"nt\": %d, \"compute\": %d, "
           "\"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
           shape, run_b, waves, nt, comp, best, gbs, gbs / 8000.0);
    fflush(stdout);
  };
  auto run_span = [&](auto kern, int waves, int nt, int chains, int scan) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    float best = 1e9f;
    for (int it = 0; it < 6; it++) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * waves), 131072, 0, a, n16, out);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;
    }
    const double gbs = (double)bytes / (best * 1e-3) / 1e9;
    printf("{\"shape\": \"span64\", \"waves\": %d, \"nt\": %d, \"chains\": %d, \"scan\": %d, "
           "\"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", waves, nt, chains, scan, best, gbs, gbs / 8000.0);
    fflush(stdout);
  };
  if (argc > 1 && std::string(argv[1]) == "span") {
    for (int waves : {8, 12}) {
      run_span(span_kernel<false, 1, false>, waves, 0, 1, 0);
      run_span(span_kernel<true, 1, false>, waves, 1, 1, 0);
      run_span(span_kernel<false, 2, false>, waves, 0, 2, 0);
      run_span(span_kernel<false, 4, false>, waves, 0, 4, 0);
      run_span(span_kernel<false, 2, true>, waves, 0, 2, 1);
      run_span(span_kernel<false, 4, true>, waves, 0, 4, 1);
      run_span(span_kernel<true, 4, true>, waves, 1, 4, 1);
    }
    run(probe_kernel<true, false>, 64, 8192, 12, 1, 0);  // coalesced reference
  } else if (argc > 1 && std::string(argv[1]) == "depth") {
    // two lanes per stream, default policy, 8 KiB per lane: issue work per
    // step (K) against steps of loads in flight (DEPTH)
    for (int waves : {8, 12}) {
      run(probe_kernel<false, true, 1, 1>, 2, 8192, waves, 0, 1);
      run(probe_kernel<false, true, 1, 2>, 2, 8192, waves, 0, 12);
      run(probe_kernel<false, true, 2, 1>, 2, 8192, waves, 0, 2);
      run(probe_kernel<false, true, 2, 2>, 2, 8192, waves, 0, 22);
      run(probe_kernel<false, true, 3, 1>, 2, 8192, waves, 0, 3);
      run(probe_kernel<false, true, 3, 2>, 2, 8192, waves, 0, 32);
    }
  } else {
    for (int comp = 0; comp <= 1; comp++)
      for (int shape : {1, 2, 4, 8, 64})
        for (size_t rb : {4096ul, 8192ul})
          for (int waves : {8, 12})
            for (int nt = 0; nt <= 1; nt++) {
              if (shape == 64 && rb != 8192) continue;
              if (comp) {
                if (nt) run(probe_kernel<true, true>, shape, rb, waves, nt, comp);
                else run(probe_kernel<false, true>, shape, rb, waves, nt, comp);
              } else {
                if (nt) run(probe_kernel<true, false>, shape, rb, waves, nt, comp);
                else run(probe_kernel<false, false>, shape, rb, waves, nt, comp);
              }
            }
  }
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
