// Persistent per-SSTable engine.
//
// NovaLSM checksums one SSTable per call (~4K blocks, ~16.5 MiB) from many
// threads at once: the flush and compaction EnvBGThreads finishing tables
// (ltc/compaction_thread.h:77-107, StoCWritableFileClient::Format,
// ltc/stoc_file_client_impl.cpp:183-377) and readers verifying a fetched
// table (ReadAll, :843-882; table/table.cc:425-441).  One such table is
// ~2.6 us of HBM time, but a launch of any kernel over it pays a fixed
// ~25-29 us (launch, LDS table fill, ramp, tail: DESIGN.md 3.5d), so
// per-table launches -- direct, or coalesced by a host queue -- stay at
// 14-29 % of the HBM roofline.
//
// The engine pays the launch and the table fill once per burst of requests:
//   * one workgroup per CU (12 waves) stays resident with the M_256 tables in
//     LDS (G = 16 lanes per block);
//   * a submitting thread writes its request (image, descriptor arrays,
//     outputs, op, blocks per chunk) into a ring as tagged 8-byte words, and
//     bumps a tail word (the ring lives in device memory that the host writes
//     through the PCIe BAR; pinned host memory without a large BAR);
//   * wave 0 of workgroup 0 -- the dispatcher -- polls the next entry's words
//     and the tail in one round trip, copies new requests into device-memory
//     slots, maps their ticket pages to them and publishes their chunk
//     tickets by advancing one end word;
//   * one poller wave per CU reads the end word and shares it through LDS;
//     every other wave takes tickets from its group's head (eight heads, one
//     per XCD: group = workgroup index % 8, which is the XCD a workgroup runs
//     on under the round-robin dispatch; MI355X_MICROARCH.md "dequeue"),
//     finds the ticket's request (its cursor slot and the ticket's page, one
//     round trip), runs the chunk (engine_chunk: rounds of 4 blocks, a
//     block's loads in two passes), counts it on its group's counter line and
//     only then claims its next ticket (the claim's add is contended; before
//     the chunk, every load of the chunk would wait for it);
//   * the last chunk of a group writes that group's completion word of the
//     request in pinned host memory (the dispatcher writes those of groups
//     without tickets); the submitter spins until all 8 are set (a test for
//     >=: the words only grow).
//
// Sharing the GPU (round 5).  A resident instance holds ~153 KiB of every
// CU's LDS, so no other LDS-using kernel can start while it runs.  Every other
// launch of this library (engine_yield_begin / engine_yield_end around it)
// bumps a yield word in pinned memory and records an event on its stream.  The
// dispatcher, once it sees the word differ from its launch value, takes no
// new request, finishes the ones it took and exits; the next instance is
// launched behind every registered launch that has not finished
// (hipStreamWaitEvent), so it cannot take the CUs back from them.  An instance
// always takes the requests present when it starts (one batch) before it
// honours a yield: under steady plain traffic every instance still makes
// progress.
//
// Lifetime.  Once no request arrives for the idle time (default 1 ms) and
// every taken request is done, the dispatcher stops the workers and the kernel
// exits, recording the first request it did not take; a submitter that finds
// its request untaken relaunches the engine, which starts there.  Every spin
// is bounded: workers give up (error word) after 20 s without new tickets and
// no stop, the dispatcher after 20 s with a request unfinished and none new,
// submitters after NOVA_SST_ENGINE_TIMEOUT_MS.
//
// Taking a request back (round 5).  A submitter whose request
// fails (timeout, engine error, launch failure) runs the plain call only once
// the engine can no longer touch the request: it sets the request's cancel
// word, then
//   * the instance has not started (its `alive` word is not its generation):
//     it will read the cancel word when it reaches the request (the instance
//     stores `alive` and fences before its first ring read, the submitter
//     stores `cancel` and fences before it reads `alive`), and skips it;
//   * the instance exited without taking it: later instances skip it;
//   * otherwise the instance is stopped and the submitter waits for the
//     request's completion word or the kernel's end.
// If none of these comes within the hard limit the call returns an error
// WITHOUT the plain call (the engine may still write the outputs), and the
// engine is not used again by this process.  Otherwise the engine backs off
// (100 ms, doubling to 12.8 s, reset by the next success) and is retried.
//
// Memory visibility (cdna_hip_programming.md Guideline 16):
//   * host -> engine: requests and the tail word are read with system-scope
//     loads (fine-grained memory, no cache);
//   * dispatcher -> workers: slot fields and the end word are stored and
//     loaded with agent-scope atomics (write-through, L1-bypassing), drained
//     before the end word is advanced;
//   * caller memory: the chunk body loads descriptors, block bytes and stored
//     CRCs non-temporally, so no L1 line of a buffer rewritten since an earlier
//     request is used;
//   * results: stored write-through (agent-scope atomic stores) and drained
//     (s_waitcnt vmcnt(0)) before the chunk's done count is added -- no L2
//     write-back fence, which at one per chunk serialised the engine at
//     ~15 us per request; the last chunk's wave then stores the completion
//     word (system scope).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/prctl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "crc32c_kernels.hpp"

namespace {

using namespace nova_dev;

constexpr uint32_t kRing = 1024;  // requests in flight (host ring and device slots)
constexpr int kEngG = 16;         // lanes per block (units kernel: G = 16)
// Launch bound: 12 waves per CU, two passes of kEK12 swaths per 4 KiB block
// (157 VGPRs).  Round 4's 12-wave build kept the one-pass loads (kEK) and
// spilled; the 8-wave one-pass build (211 VGPRs) stays for
// NOVA_SST_ENGINE_WAVES <= 8.  Round 6 (profiles/r06_engine_waves.log, with
// the chunk rule retuned for it in engine_submit: r06_engine_cb12.log): verify
// at 16 callers 4.55-4.68 -> 5.27-5.36 TB/s, 8 callers 4.33-4.35 -> 4.91-5.04;
// trailers 4.35-4.43 -> 4.73-4.85 / 4.24 -> 4.78-4.83.
constexpr int kEngMaxWaves = 12;
constexpr int kEngWaves8 = 8;
constexpr int kEngWaves = 12;
constexpr uint32_t kCntGroups = kEngGroups;
constexpr uint32_t kTrWords = 16;
// Ticket pages: page[p] holds a copy of the request holding ticket kPage * p
// (its descriptor, tickets and seq, as 16 tagged 8-B words), so a wave finds
// its ticket's request in ONE round trip: its 16 lanes read the page, and a
// consistent copy (every tag the same seq) of a request of this instance
// whose tickets hold t is used as is.  Otherwise (a page whose first ticket
// belongs to an earlier request, one overwritten after a wrap, or one being
// rewritten) the copy's seq is a hint for the walk from the wave's cursor
// (an idle wave's cursor lags by every request it sat out).
constexpr uint32_t kPageShift = 4;
constexpr uint32_t kPages = 1u << 14;  // 256K tickets covered (wraps: hints only)
constexpr uint32_t kMaxIdleUs = 1000000;  // below the workers' 20 s give-up

// Exit reasons (EngCtl::why)
constexpr uint32_t kWhyIdle = 1, kWhyStop = 2, kWhyYield = 3, kWhyLost = 4, kWhySlice = 5;
constexpr uint32_t kWhyN = 6;

// A host ring entry (128 B), written by its submitter: 12 words, each
// (tag << 32) | a 32-bit half of a field, tag = low 32 bits of seq + 1.  The
// dispatcher polls the next entry's 12 words with one 8-B load per lane, in
// the same round trip as the tail, stop, yield and cancel words: an entry
// whose 12 tags are all its seq + 1 is complete (each word is one 8-B store
// and one 8-B load, so a half-written entry shows stale tags), and is taken
// without a second round trip over PCIe.
enum EngWord : uint32_t {
  kWBaseLo, kWBaseHi, kWOffsLo, kWOffsHi, kWSizesLo, kWSizesHi, kWOutLo, kWOutHi, kWBadLo, kWBadHi,
  kWN, kWPacked, kWords  // kWPacked: flags (bits 0-15) | mode << 16 | blocks per chunk << 20
};
struct EngHostReq {
  uint64_t w[16];
};
struct EngReq {  // an entry, decoded
  uint64_t base, offs, sizes, out, bad, n;
  uint32_t mode, flags, cb;
};
// Host -> engine words (round 5): fine-grained DEVICE memory that the host
// writes through the PCIe BAR (a large-BAR device; else pinned host memory).
// The dispatcher's poll then reads HBM instead of crossing PCIe: a host ->
// GPU -> host ping-pong measured 1.90 us against 2.65 us through pinned
// memory (tools/pingpong.hip, profiles/r05_pingpong.log).  The host
// only writes these words, with one exception: the take-back reads its
// cancel word back, which completes the posted write before it reads
// `alive` (a PCIe read does not pass an earlier posted write).
struct EngIn {
  uint64_t htail;   // requests [first_seq, htail) are in the ring
  uint32_t hstop;   // take no more requests, exit once the taken ones are done
  uint32_t pad0;
  uint64_t hyield;  // bumped by every non-engine launch of the library (yield)
  uint64_t pad1[13];
  EngHostReq ring[kRing];
  uint64_t cancel[kRing];  // cancel[seq % kRing] == seq + 1: its submitter took the request back
};
struct EngCtl {  // engine -> host words: pinned host memory (fine-grained)
  uint64_t pad1[16];
  uint64_t consumed;  // engine: the first seq it did not take (valid once exited)
  uint32_t exited;    // engine: this instance takes no more requests
  uint32_t error;     // engine: give-up code (1: a worker saw no new ticket for the give-up
                      // time, 2: a published ticket without a slot, 3: a request unfinished
                      // for the give-up time after the last arrival)
  uint64_t alive;     // engine: the instance's generation, stored before its first ring read
  uint32_t why;       // engine: exit reason (kWhy*)
  uint32_t pad2;
  uint64_t maxgap;    // engine: the dispatcher's longest gap between two polls (ticks), at exit
  uint64_t pad3[11];
};
struct EngSlot {  // a device slot (128 B), written by the dispatcher
  uint64_t seq1;          // request seq + 1 (0: never written)
  uint64_t cstart, cend;  // its chunk tickets [cstart, cend)
  uint64_t base, offs, sizes, out, bad, n;
  uint32_t mode, flags, cb, pad;
  uint64_t pad2[3];
};
// A ticket page: (tag << 32) | payload, tag = low 32 bits of the request's seq + 1.
enum EngPageWord : uint32_t {
  kPSeqHi, kPCsLo, kPCsHi, kPNch, kPBaseLo, kPBaseHi, kPOffsLo, kPOffsHi, kPSizesLo, kPSizesHi,
  kPOutLo, kPOutHi, kPBadLo, kPBadHi, kPN, kPPacked, kPWords  // kPPacked as kWPacked
};
struct EngPage {
  uint64_t w[kPWords];
};
// An instance's words in device memory.  Two of them, used by alternate
// instances (generation parity): each instance's dispatcher zeroes the OTHER
// one as its last act, so the next instance starts on a zeroed header without
// a memset packet ahead of its launch (a relaunch at every time slice; ~170 us
// of waiting callers with the memset: profiles/r05_engine_slowest.log).
struct EngHdr {
  uint64_t dend;  // chunk tickets published
  uint64_t p0[15];
  uint32_t dstop;
  uint32_t p1[31];
  uint64_t reqs_done;
  uint64_t p2[15];
  uint32_t head[kCntGroups][32];  // per-group ticket heads, one 128-B line each
};
constexpr uint32_t kHdrWords = sizeof(EngHdr) / 8;
struct EngDev {  // device memory: all zeroed once
  EngHdr hdr[2];
  // ---- below: slots and pages from an earlier instance hold seqs below the
  // new first_seq, which the lookup never takes.
  // Chunks finished, per slot: one counter per ticket group t % 8 (1/8 of the
  // request's adds per address).  Same-address atomics serialize in memory;
  // one counter for all of a 1024-chunk request put ~1024 of them on the
  // request's critical path.  The group whose count completes stores its own
  // completion word in host memory (hdone, 8 per request): a second-level
  // counter of the groups -- one more dependent device atomic on every
  // request's critical path -- is not needed.
  // Two banks per slot: request seq counts in bank (seq / kRing) & 1, and the
  // dispatcher, taking it, zeroes the OTHER bank -- the next occupant's
  // (seq + kRing, published only once seq is done, after the drain that
  // publishes seq).  So a request's counters were zeroed and drained one ring
  // turn before it was taken, and a worker that finds its page before the end
  // word moves never adds to a counter whose zeroing is still in flight; a
  // request left unfinished (an instance that gave up) dirties only a bank the
  // slot's next occupant zeroes.
  uint32_t cgrp[kRing][2][kCntGroups][32];  // 128-B line each
  EngSlot slot[kRing];
  // trace (s_memrealtime): 0 dispatched, 2 last chunk done; chunk 0's wave:
  // 3 ticket seen, 1 slot found, 4 body done, 5 drained, 6 counted; the last
  // chunk's wave: 7 ticket seen, 8 slot found, 9 body done, 10 drained, 11 counted
  uint64_t tr[kRing][kTrWords];
  EngPage page[kPages];      // ticket page -> a copy of the request holding its first ticket
};
struct EngParams {
  const EngIn* in;          // host -> engine words
  // hdone[(seq % kRing) * 8 + g] = seq + 1 once group g's results of the request
  // are in memory (groups without tickets: at publication); the request is
  // done when all 8 are
  uint64_t* hdone;
  EngCtl* ctl;
  EngDev* dev;
  EngHdr* hdr;             // this instance's header (zeroed)
  EngHdr* hdr_next;        // the next instance's: zeroed by this dispatcher at its exit
  uint64_t first_seq;
  uint64_t gen;            // this instance's generation (stored to ctl->alive)
  uint64_t yield_gen;      // in->hyield at launch: any other value is a yield
  uint64_t idle_ticks;     // s_memrealtime ticks (100 MHz) without a request before exiting
  uint64_t give_up_ticks;  // no new ticket (worker) / an unfinished request (dispatcher) this long: exit
  uint64_t slice_ticks;    // 0, or: take no request after running this long (then exit; the next instance follows)
  uint64_t* htrace;        // trace (or null): per request, the tr words copied to pinned memory
  uint32_t page_poll;      // waiting workers poll their ticket's page (NOVA_SST_ENGINE_PAGE_POLL, default 1)
  uint32_t drop_chunks;    // test hook: the workers run no chunk (nova_sst_engine_set_drop_chunks)
  CrcParams tab;           // tables and zero line for every chunk
};

typedef __attribute__((address_space(1))) uint32_t g32;
typedef __attribute__((address_space(1))) uint64_t g64;

template <typename T>
__device__ __forceinline__ T ld_agent(const T* a) {
  return __hip_atomic_load((const __attribute__((address_space(1))) T*)a, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* a, T v) {
  __hip_atomic_store((__attribute__((address_space(1))) T*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_sys(const T* a) {
  return __hip_atomic_load((const __attribute__((address_space(1))) T*)a, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void st_sys(T* a, T v) {
  __hip_atomic_store((__attribute__((address_space(1))) T*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS words at absolute byte addresses (the dynamic LDS region starts at 0).
__device__ __forceinline__ __attribute__((address_space(3))) uint64_t* lds64(uint32_t a) {
  return reinterpret_cast<__attribute__((address_space(3))) uint64_t*>(a);
}
__device__ __forceinline__ __attribute__((address_space(3))) uint32_t* lds32(uint32_t a) {
  return reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(a);
}
// Per workgroup: [the end word as last read][stop][poll lock], after the tables
// (main image, tree levels, byte table).  One waiting wave per CU at a time reads the
// device's end and stop words and copies them here; the others spin on
// these LDS words -- 256 pollers of the end word's line instead of ~2800.
template <int G>
constexpr uint32_t tree_levels() { return 2 + (G >= 2) + (G >= 4) + (G >= 8) + (G >= 16); }
template <int G>
constexpr uint32_t byte_tab_off() { return kMainBytes + tree_levels<G>() * kTreeBytes; }
template <int G>
constexpr uint32_t poll_off() { return byte_tab_off<G>() + 1024u; }

// Wave 0 of workgroup 0: host ring -> device slots, tickets published.
__device__ __forceinline__ void engine_dispatch(const EngParams& e) {
  const int lane = threadIdx.x & 63;
  EngDev* d = e.dev;
  // `alive` reaches host memory before any ring entry is read: a submitter
  // that cancelled a request and then read `alive` as not yet stored knows
  // this instance will read the cancel word (see the header comment)
  if (lane == 0) st_sys(&e.ctl->alive, e.gen);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
  uint64_t seen = e.first_seq, cend = 0;
  uint64_t last = now_ticks();
  const uint64_t born = last;
  uint64_t prev_poll = last, maxgap = 0;  // (a stalled or preempted dispatcher shows as a long gap)
  bool took = false;
  uint64_t auto_done = 0;  // group completions of groups without tickets (reqs_done counts the rest)
  for (;;) {
    {
      const uint64_t nowp = now_ticks();
      maxgap = nowp - prev_poll > maxgap ? nowp - prev_poll : maxgap;
      prev_poll = nowp;
    }
    // one round trip: lanes 0-11 the words of entry `seen`, lane 12 its cancel
    // word, 13 the tail, 14 the stop word, 15 the yield word
    uint64_t x = 0;
    {
      const uint64_t* a = nullptr;
      if (lane < (int)kWords) a = &e.in->ring[seen % kRing].w[lane];
      else if (lane == 12) a = &e.in->cancel[seen % kRing];
      else if (lane == 13) a = &e.in->htail;
      else if (lane == 14) a = reinterpret_cast<const uint64_t*>(&e.in->hstop);  // hstop | pad0 << 32
      else if (lane == 15) a = &e.in->hyield;
      if (lane < 16) x = ld_sys(a);
    }
    const uint32_t tag0 = (uint32_t)(seen + 1);
    const bool first_ready =
        (__builtin_amdgcn_ballot_w64(lane < (int)kWords && (uint32_t)(x >> 32) == tag0) & 0xfffull) == 0xfffull;
    auto lane64 = [&](int l) -> uint64_t {
      return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    };
    const uint64_t ht = lane64(13);
    const uint32_t stop = (uint32_t)lane64(14);
    const uint64_t yv = lane64(15);
    const bool avail = first_ready || ht > seen;
    // a yield stops the takes once this instance took its first batch (or
    // found none): some request moves per instance however often plain
    // launches arrive
    const bool yielded = yv != e.yield_gen;
    const bool sliced = e.slice_ticks && took && now_ticks() - born > e.slice_ticks;
    const bool drain = stop != 0 || sliced || (yielded && (took || !avail));
    if (!drain && avail) {
      // one request (the common case): decoded from the poll; more: every
      // lane reads its own entry (a second round trip), taken up to the
      // first that is not complete yet
      uint32_t m = 1;
      EngReq r{};
      uint64_t cancel = 0, nch = 0;
      bool mine = lane == 0;
      if (first_ready && ht <= seen + 1) {
        auto half = [&](uint32_t k) -> uint64_t { return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)k); };
        if (lane == 0) {
          r.base = half(kWBaseLo) | half(kWBaseHi) << 32;
          r.offs = half(kWOffsLo) | half(kWOffsHi) << 32;
          r.sizes = half(kWSizesLo) | half(kWSizesHi) << 32;
          r.out = half(kWOutLo) | half(kWOutHi) << 32;
          r.bad = half(kWBadLo) | half(kWBadHi) << 32;
          r.n = half(kWN);
          const uint32_t pk = (uint32_t)half(kWPacked);
          r.flags = pk & 0xffffu;
          r.mode = (pk >> 16) & 0xfu;
          r.cb = pk >> 20;
          cancel = lane64(12);
        }
      } else {
        const uint32_t want = (uint32_t)(ht - seen < 64 ? ht - seen : 64);
        bool ok = false;
        if ((uint32_t)lane < want) {
          const uint64_t seq = seen + lane;
          const EngHostReq* h = e.in->ring + seq % kRing;
          uint64_t w[kWords];
#pragma unroll
          for (uint32_t k = 0; k < kWords; k++) w[k] = ld_sys(&h->w[k]);
          cancel = ld_sys(&e.in->cancel[seq % kRing]);
          ok = true;
#pragma unroll
          for (uint32_t k = 0; k < kWords; k++) ok = ok && (uint32_t)(w[k] >> 32) == (uint32_t)(seq + 1);
          r.base = (uint32_t)w[kWBaseLo] | (uint64_t)(uint32_t)w[kWBaseHi] << 32;
          r.offs = (uint32_t)w[kWOffsLo] | (uint64_t)(uint32_t)w[kWOffsHi] << 32;
          r.sizes = (uint32_t)w[kWSizesLo] | (uint64_t)(uint32_t)w[kWSizesHi] << 32;
          r.out = (uint32_t)w[kWOutLo] | (uint64_t)(uint32_t)w[kWOutHi] << 32;
          r.bad = (uint32_t)w[kWBadLo] | (uint64_t)(uint32_t)w[kWBadHi] << 32;
          r.n = (uint32_t)w[kWN];
          const uint32_t pk = (uint32_t)w[kWPacked];
          r.flags = pk & 0xffffu;
          r.mode = (pk >> 16) & 0xfu;
          r.cb = pk >> 20;
        }
        // the complete entries from `seen` on (lane 0's is, by the tail)
        const uint64_t notok = ~__builtin_amdgcn_ballot_w64(ok);
        m = notok ? (uint32_t)__builtin_ctzll(notok) : 64u;
        if (m > want) m = want;
        if (m == 0) {  // (the tail ran ahead of a word's visibility: poll again)
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        mine = (uint32_t)lane < m;
      }
      if (mine) {
        if (cancel == seen + lane + 1) r.n = 0;  // taken back by its submitter: no tickets, done at once
        if (r.cb == 0 || r.cb > 16) r.cb = 16;
        nch = (r.n + r.cb - 1) / r.cb;
      }
      // inclusive prefix of the chunk counts over the lanes
      uint64_t inc = nch;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint64_t o = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(inc >> 32), s) << 32) |
                           (uint32_t)__shfl_up((int)(uint32_t)inc, s);
        if (lane >= s) inc += o;
      }
      if ((uint32_t)lane < m) {
        const uint64_t seq = seen + lane;
        // the slot's previous request (seq - kRing) is done: the bank it
        // counted in is the next occupant's (see EngDev::cgrp)
        const uint32_t other = (uint32_t)((seq / kRing) & 1u) ^ 1u;
        for (uint32_t x = 0; x < kCntGroups; x++) st_agent(&d->cgrp[seq % kRing][other][x][0], 0u);
        if (e.htrace) {
          st_agent(&d->tr[seq % kRing][0], now_ticks());
          for (uint32_t k = 1; k < 12; k++) st_agent(&d->tr[seq % kRing][k], (uint64_t)0);
        }
      }
      // trace: the stamps are zero before a worker that finds its page early
      // stores its own
      if (e.htrace) drain_vm();
      if ((uint32_t)lane < m) {
        const uint64_t seq = seen + lane;
        EngSlot* S = &d->slot[seq % kRing];
        st_agent(&S->cstart, cend + inc - nch);
        st_agent(&S->cend, cend + inc);
        st_agent(&S->base, r.base);
        st_agent(&S->offs, r.offs);
        st_agent(&S->sizes, r.sizes);
        st_agent(&S->out, r.out);
        st_agent(&S->bad, r.bad);
        st_agent(&S->n, r.n);
        st_agent(&S->mode, r.mode);
        st_agent(&S->flags, r.flags);
        st_agent(&S->cb, r.cb);
        st_agent(&S->seq1, seq + 1);
      }
      const uint64_t total = uni64(((uint64_t)(uint32_t)__shfl((int)(uint32_t)(inc >> 32), 63) << 32) |
                                   (uint32_t)__shfl((int)(uint32_t)inc, 63));
      // ticket pages: every page whose first ticket a request holds gets a
      // copy of it (the wave's 64 lanes write one request's pages at a time)
      for (uint32_t k = 0; k < m; k++) {
        auto rl = [&](uint64_t v) -> uint64_t {  // lane k's 64-bit value
          return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
        };
        const uint64_t cs = cend + rl(inc - nch), ce = cend + rl(inc);
        const uint64_t p0 = (cs + (1u << kPageShift) - 1) >> kPageShift, p1 = (ce + (1u << kPageShift) - 1) >> kPageShift;
        const uint64_t np = p1 - p0 < kPages ? p1 - p0 : kPages;
        if (np == 0) continue;  // (scalar)
        const uint64_t seq1 = seen + k + 1;
        const uint64_t tag = (uint64_t)(uint32_t)seq1 << 32;
        const uint64_t rb = rl(r.base), ro = rl(r.offs), rs = rl(r.sizes), rq = rl(r.out), rd = rl(r.bad);
        const uint32_t rn = (uint32_t)rl(r.n);
        const uint32_t rp = (uint32_t)__builtin_amdgcn_readlane((int)((r.flags & 0xffffu) | (r.mode << 16) | (r.cb << 20)), (int)k);
        // 16 lanes per page, one word each: every store instruction writes 4
        // whole 128-B pages (coalesced) instead of one word of 64 pages
        const uint32_t wi = (uint32_t)lane & (kPWords - 1);
        uint32_t pv = 0;
        switch (wi) {
          case kPSeqHi: pv = (uint32_t)(seq1 >> 32); break;
          case kPCsLo: pv = (uint32_t)cs; break;
          case kPCsHi: pv = (uint32_t)(cs >> 32); break;
          case kPNch: pv = (uint32_t)(ce - cs); break;
          case kPBaseLo: pv = (uint32_t)rb; break;
          case kPBaseHi: pv = (uint32_t)(rb >> 32); break;
          case kPOffsLo: pv = (uint32_t)ro; break;
          case kPOffsHi: pv = (uint32_t)(ro >> 32); break;
          case kPSizesLo: pv = (uint32_t)rs; break;
          case kPSizesHi: pv = (uint32_t)(rs >> 32); break;
          case kPOutLo: pv = (uint32_t)rq; break;
          case kPOutHi: pv = (uint32_t)(rq >> 32); break;
          case kPBadLo: pv = (uint32_t)rd; break;
          case kPBadHi: pv = (uint32_t)(rd >> 32); break;
          case kPN: pv = rn; break;
          default: pv = rp; break;
        }
        for (uint64_t j = (uint32_t)lane / kPWords; j < np; j += 64 / kPWords)
          st_agent(&d->page[(p0 + j) & (kPages - 1)].w[wi], tag | pv);
      }
      drain_vm();  // every lane's slot and page stores are written through before the end moves
      cend += total;
      if (lane == 0) st_agent(&e.hdr->dend, cend);
      // groups without tickets in a request (all 8 for one taken back) are
      // done now; they count toward the dispatcher's expected completions
      uint32_t idle_groups = 0;
      if ((uint32_t)lane < m) {
        const uint64_t seq = seen + lane;
        const uint64_t cs = cend - total + inc - nch, ce = cend - total + inc;
        for (uint32_t g = 0; g < kCntGroups; g++)
          if (engine_group_share(cs, ce, g) == 0) {
            st_sys(&e.hdone[(seq % kRing) * kCntGroups + g], seq + 1);
            idle_groups++;
          }
      }
      for (int s = 32; s >= 1; s >>= 1) idle_groups += (uint32_t)__shfl_xor((int)idle_groups, s);
      auto_done += uni32(idle_groups);
      seen += m;
      took = true;
      last = now_ticks();
      continue;
    }
    const uint64_t quiet = now_ticks() - last;
    if (drain || quiet > e.idle_ticks) {
      uint64_t done = 0;
      if (lane == 0) done = ld_agent(&e.hdr->reqs_done);
      // every request taken is finished: all 8 groups of each
      const bool all_done = uni64(done) + auto_done == kCntGroups * (seen - e.first_seq);
      // a request unfinished long after the last arrival cannot finish: give up
      const bool lost = !all_done && quiet > e.give_up_ticks;
      if (all_done || lost) {
        // the next instance's header, zeroed and drained before `exited`
        // (every worker of this instance uses e.hdr only)
        {
          uint64_t* z = reinterpret_cast<uint64_t*>(e.hdr_next);
          for (uint32_t k = (uint32_t)lane; k < kHdrWords; k += 64) st_agent(&z[k], (uint64_t)0);
          drain_vm();
        }
        if (lane == 0) {
          if (lost) st_sys(&e.ctl->error, 3u);
          st_sys(&e.ctl->why, lost ? kWhyLost : stop ? kWhyStop : yielded ? kWhyYield : sliced ? kWhySlice : kWhyIdle);
          st_sys(&e.ctl->maxgap, maxgap);
          st_agent(&e.hdr->dstop, 1u);
          st_sys(&e.ctl->consumed, seen);
          __hip_atomic_store((__attribute__((address_space(1))) uint32_t*)&e.ctl->exited, 1u,
                             __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
      }
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// One chunk of a request: blocks [c * cb, (c + 1) * cb) of it, in rounds of
// kGroups = 4 blocks, one per 16-lane group -- the burst kernel's shape
// (crc32c_burst_kernel) on the rounds kernel's bank-replicated
// M_256 tables:
//   * a group issues ALL of its block's loads at once (up to kEK swaths of
//     256 B: a 4 KiB SSTable block in one pass; longer blocks take more
//     passes) with the tail line(s) -- the bytes [E, u1) and, for verify, the
//     stored CRC -- so a round is one memory round trip, not one per step;
//   * the wave's groups run the wave's largest swath count, each block's
//     region end-aligned (shorter blocks start on zero pieces);
//   * in-lane M4/M8 and cross-lane M16..M128 fold, then finish_block (tail
//     bytes from LDS, the n < 4 init fix, the mode's epilogue);
//   * the next round's descriptors are loaded before this round folds.
// Every load of caller memory is non-temporal and every result store is
// write-through (the engine outlives the caller's writes and reads).
constexpr int kEK = 18;  // swaths per pass: 4.5 KiB (4096 + 255 + 5 B blocks: one pass)
constexpr int kEK12 = 9;  // the 12-wave build: 2 passes per 4 KiB block (157 VGPRs)

// A trailer [type][LE32 masked crc] written through (sc1, as st_through's
// agent-scope stores compile): the type byte, then the CRC as one unaligned
// dword store (the hardware splits one that crosses a line) -- two partial
// writes at the memory instead of five byte stores.  The dword store is
// inline asm (an atomic store must be aligned); the chunk's vmcnt(0) drain
// before its count covers it like every other result store.
__device__ __forceinline__ void engine_store_trailer(uint8_t* d, uint32_t type, uint32_t m, bool quirk) {
  const uint32_t w = quirk ? ((m & 0x00ffffffu) | ((uint32_t)'!' << 24)) : m;
  st_through(d, (uint8_t)type);
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(d + 1), "v"(w) : "memory");
}

template <int MODE, int EK>
__device__ __forceinline__ void engine_chunk(const uint8_t* lds, const CrcParams& p, uint64_t c) {
  constexpr int G = kEngG;
  constexpr uint64_t kS = 16ull * G;
  constexpr uint32_t kGroups = 64 / G;
  constexpr bool kTail2 = MODE == kVerify;
  const int lane = threadIdx.x & 63;
  const int q = lane & (G - 1);
  const int grp = lane / G;
  const uint32_t rep = (uint32_t)(lane & 31) << 2;
  const uint32_t lo0 = rep, lo1 = rep | 128u, lo2 = rep | 0x10000u, lo3 = rep | 0x10080u;
  const uint8_t* tree = lds + kMainBytes;  // level l: M_{4 * 2^l}
  const bool raw = (p.flags & NOVA_CRC32C_RAW) != 0;
  const uint32_t extra = MODE == kVerify ? 1u : 0u;  // verify covers block + type byte
  const uint64_t zl = (uint64_t)p.zline;
  const uint64_t base = (uint64_t)p.base;
  const uint64_t b_lo = c * p.chunk;
  const uint64_t b_hi = b_lo + p.chunk < p.n_blocks ? b_lo + p.chunk : p.n_blocks;
  uint32_t nbad = 0;
  // this round's descriptors (and, loaded during its fold, the next round's)
  auto desc = [&](uint64_t b0, uint64_t& o, uint32_t& ln) {
    const uint64_t b = b0 + grp;
    const uint64_t bb = b < b_hi ? b : b_lo;  // clamped: valid memory, result unused
    o = ld_nt<true>(p.offsets + bb);
    ln = ld_nt<true>(p.lengths + bb);
  };
  uint64_t o_cur = 0, o_nxt = 0;
  uint32_t l_cur = 0, l_nxt = 0;
  desc(b_lo, o_cur, l_cur);
  for (uint64_t b0 = b_lo; b0 < b_hi; b0 += kGroups) {
    const uint64_t b = b0 + grp;
    const bool valid = b < b_hi;
    const uint64_t u0 = base + o_cur;
    const uint32_t n = l_cur + extra;
    const uint64_t u1 = u0 + n;
    const uint64_t E = u1 & ~15ull;
    const uint64_t A0 = u0 & ~15ull;
    const uint32_t K = valid && E > A0 ? (uint32_t)((E - A0 + kS - 1) / kS) : 0u;
    const uint32_t Kw = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max(K));
    uint64_t first = E - (uint64_t)Kw * kS + 16ull * q;
    FlatSet Y;
    Y.u0 = u0;
    Y.u1 = u1;
    Y.rec = b;
    Y.ninit = (raw || n < 4) ? 0u : ~0u;  // init 0 (table/format.cc, table_builder.cc)
    Y.st = 0;
    Y.valid = valid;
    // tail line(s): [E, E+16) holds the tail bytes (verify: the start of the
    // stored CRC), [E+16, E+32) the rest of a stored CRC
    Y.t = gload16((valid && (kTail2 || (u1 & 15) != 0)) ? E : zl);
    if constexpr (kTail2) Y.t2 = gload16(valid && u1 + 4 > E + 16 ? E + 16 : zl);
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    // positions relative to the lane's first piece: the block's first byte
    // (head masking) and its first line (pieces before it read zeros); 64-bit,
    // since a round may pair a block over 1 GiB with short ones whose start
    // then lies more than 2^30 bytes after the round's first piece
    int64_t urel = (int64_t)(u0 - first), arel = (int64_t)(A0 - first);
    for (uint32_t k0 = 0; k0 < Kw; k0 += EK) {
      uint4 d[EK];
#pragma unroll
      for (int i = 0; i < EK; i++) {
        const bool in = valid && k0 + i < Kw && (int64_t)(kS * i) >= arel;
        d[i] = gload16(in ? first + (uint64_t)i * kS : zl);
      }
      if (k0 == 0 && b0 + kGroups < b_hi) desc(b0 + kGroups, o_nxt, l_nxt);  // under the data loads
#pragma unroll
      for (int i = 0; i < EK; i++) {
        if (k0 + i < Kw) {  // wave-uniform
          const int64_t hr = urel - (int64_t)(kS * i);
          const int32_t h = hr < -4 ? -4 : (hr > 32 ? 32 : (int32_t)hr);
          const uint4 w = is_head(h) ? head_piece(d[i], h, Y.ninit) : d[i];
          swath4<0>(lds, c0, c1, c2, c3, w, lo0, lo1, lo2, lo3);
        }
      }
      first += (uint64_t)EK * kS;  // the next pass
      urel -= (int64_t)(EK * kS);
      arel -= (int64_t)(EK * kS);
    }
    // fold the group's stream words: in-lane M4/M8, then M16 .. M128 across the group
    uint32_t v = lapply(tree + kTreeBytes, lapply(tree, c0) ^ c1) ^ (lapply(tree, c2) ^ c3);
    auto level = [&](int k, uint32_t o) {  // o: v of lane q ^ 2^k
      const bool right = (q >> k) & 1;
      v = lapply(tree + (2 + k) * kTreeBytes, right ? o : v) ^ (right ? v : o);
    };
    level(0, lane_xor<1>(v));
    level(1, lane_xor<2>(v));
    level(2, lane_xor<4>(v));
    level(3, lane_xor<8>(v));
    uint64_t wb_a = 0;
    uint32_t wb_v = 0;
    finish_block<MODE, kMainBytes>(lds, byte_tab_off<G>(), p, raw, v, Y, wb_a, wb_v);
    if (q == 0 && valid) {
      if constexpr (MODE == kVerify) {
        st_through((uint8_t*)wb_a, (uint8_t)wb_v);
        nbad += wb_v ? 0u : 1u;
      } else if constexpr (MODE == kTrailer) {
        engine_store_trailer((uint8_t*)wb_a, (p.flags >> 8) & 0xffu, wb_v, (p.flags & NOVA_TRAILER_TB_QUIRK) != 0);
      } else {
        st_through((uint32_t*)wb_a, wb_v);
      }
    }
    o_cur = o_nxt;
    l_cur = l_nxt;
  }
  if constexpr (MODE == kVerify) {  // one add per chunk, performed in memory (system scope)
    const uint32_t nb = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(__builtin_popcountll(__builtin_amdgcn_ballot_w64(nbad & 1)) +
              2 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((nbad >> 1) & 1)) +
              4 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((nbad >> 2) & 1)) +
              8 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((nbad >> 3) & 1)) +
              16 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((nbad >> 4) & 1))));
    if (lane == 0 && nb && p.n_bad)
      __hip_atomic_fetch_add((g32*)p.n_bad, nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Every other wave: tickets -> chunks (engine_chunk).
template <int G, int EK>
__device__ __forceinline__ void engine_work(const EngParams& e, const uint8_t* lds) {
  // (test hook: no worker runs a chunk, so the dispatcher's "lost" exit leaves
  // the requests it took unfinished whatever the timing)
  if (e.drop_chunks) return;
  const int lane = threadIdx.x & 63;
  EngDev* d = e.dev;
  // Tickets t with t % 8 == x go to the waves of group x, each taking the
  // next from its group's head (dynamic: a request's chunks go to whichever
  // waves are free; one queue per CU instead made every request wait for the
  // slowest of 256 queues -- 35 % less at 16 callers).  The group is the
  // workgroup index mod 8: every group has workgroups whatever the device's
  // XCD count or partition mode (the hardware XCC id may miss values, which
  // left tickets unclaimed: ADVICE r04), and under the round-robin dispatch
  // of a full MI355X it is the workgroup's XCD, so each head's line stays in
  // one XCD's L2.
  const uint32_t xcc = engine_group_of_wg(blockIdx.x);
  auto claim = [&]() -> uint64_t {
    uint32_t k = 0;
    if (lane == 0)
      k = __hip_atomic_fetch_add((g32*)&e.hdr->head[xcc][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return xcc + (uint64_t)kCntGroups * uni32(k);
  };
  uint64_t r = e.first_seq;  // request cursor (the wave's tickets only grow)
  uint64_t dend = 0;
  uint64_t t = claim();
  // t's ticket page: lanes 0-15 read its 16 words (one round trip); `found`
  // if it holds a consistent copy of a request of this instance whose
  // tickets hold t (tickets are unique within an instance; seqs of earlier
  // instances are below first_seq)
  uint64_t pw = 0, pseq1 = 0, pcs = 0;
  bool found = false;
  auto read_page = [&]() {
    pw = 0;
    if (lane < (int)kPWords) pw = ld_agent(&d->page[(t >> kPageShift) & (kPages - 1)].w[lane]);
    const uint32_t ptag = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pw >> 32), 0);
    const bool pcons = ptag != 0 &&
        (__builtin_amdgcn_ballot_w64(lane < (int)kPWords && (uint32_t)(pw >> 32) == ptag) & 0xffffull) == 0xffffull;
    auto pl = [&](uint32_t k) -> uint64_t { return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pw, (int)k); };
    pseq1 = pcons ? (pl(kPSeqHi) << 32 | ptag) : 0;
    pcs = pl(kPCsLo) | pl(kPCsHi) << 32;
    found = pcons && pseq1 > e.first_seq && t >= pcs && t < pcs + pl(kPNch);
  };
  for (;;) {
    found = false;
    if (t >= dend) {  // wait for the ticket to be published, or for the stop
      constexpr uint32_t kPoll = poll_off<G>();
      uint64_t t0 = now_ticks();
      for (uint32_t spin = 0;; spin++) {
        // t's page, read directly: the dispatcher writes a request's pages
        // before it moves the end word (its counters were zeroed a ring turn
        // earlier: EngDev::cgrp), so a found page starts the chunk one
        // end-word hop earlier
        // (profiles/r05_engine_page_poll_ab.log); a page that does not hold
        // t's request (t's request began mid-page) waits for the end word
        if (e.page_poll) {
          read_page();
          if (found) break;
        }
        // the workgroup's copy first; then, if no other wave of this CU is
        // reading them, the device's words (published into the copy)
        // (atomic loads: other waves write these words; a plain load could be hoisted)
        uint64_t x = __hip_atomic_load(lds64(kPoll), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint32_t stop = __hip_atomic_load(lds32(kPoll + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint32_t got = 0;
        if (t >= x && !stop && lane == 0) {
          uint32_t expect = 0;
          got = __hip_atomic_compare_exchange_strong(lds32(kPoll + 12), &expect, 1u, __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                    ? 1u : 0u;
        }
        if (uni32(got)) {
          uint64_t g = 0;
          uint32_t gs = 0;
          if (lane == 0) {
            g = ld_agent(&e.hdr->dend);
            gs = ld_agent(&e.hdr->dstop);
            // only the lock holder writes them, so a plain compare is enough
            if (g > __hip_atomic_load(lds64(kPoll), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
              __hip_atomic_store(lds64(kPoll), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (gs) __hip_atomic_store(lds32(kPoll + 8), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(lds32(kPoll + 12), 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          x = uni64(g);
          stop = uni32(gs);
        } else {
          x = uni64(x);
          stop = uni32(stop);
        }
        if (t < x) {
          dend = x;
          break;
        }
        if (stop) return;
        if (x != dend) {  // progress: restart the give-up clock
          dend = x;
          t0 = now_ticks();
        } else if (now_ticks() - t0 > e.give_up_ticks) {
          if (lane == 0) st_sys(&e.ctl->error, 1u);
          return;
        }
        if (spin < 64)
          __builtin_amdgcn_s_sleep(1);
        else
          __builtin_amdgcn_s_sleep(6);
      }
    }
    const uint64_t ts_seen = e.htrace ? now_ticks() : 0;
    // The request holding ticket t.  Slot r % kRing is reused for seq
    // r + kRing only after request r is done, and a live request's seq is
    // above (newest written seq) - kRing, so a slot found holding a newer
    // seq s1 - 1 moves the cursor to s1 - kRing (still at or below it).
    // First t's ticket page (one round trip); a consistent copy of a request
    // of this instance that holds t is t's request (tickets are unique within
    // an instance).  Otherwise its seq is a hint for the walk: the cursor's
    // slot is read whole (one round trip), the hinted request is tried next,
    // then slots are walked forward one at a time.  After a wrap a hint may
    // name a later request, or one the dispatcher is still writing (ADVICE
    // r04) -- any inconsistency met after following it restarts the walk from
    // the cursor, which is never past t's request and whose slots were all
    // written before t was published.
    uint64_t cstart = 0, cend = 0, base = 0, offs = 0, sizes = 0, out = 0, bad = 0, n = 0;
    uint32_t mode = 0, flags = 0, cb = 0;
    if (!found) read_page();  // (published: t < dend)
    auto pl = [&](uint32_t k) -> uint64_t { return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pw, (int)k); };
    if (found) {  // the page's copy is t's request
      r = pseq1 - 1;
      cstart = pcs;
      cend = pcs + pl(kPNch);
      base = pl(kPBaseLo) | pl(kPBaseHi) << 32;
      offs = pl(kPOffsLo) | pl(kPOffsHi) << 32;
      sizes = pl(kPSizesLo) | pl(kPSizesHi) << 32;
      out = pl(kPOutLo) | pl(kPOutHi) << 32;
      bad = pl(kPBadLo) | pl(kPBadHi) << 32;
      n = pl(kPN);
      const uint32_t pk = (uint32_t)pl(kPPacked);
      flags = pk & 0xffffu;
      mode = (pk >> 16) & 0xfu;
      cb = pk >> 20;
    }
    bool hinted = false, via_hint = false;
    const uint64_t r0 = r;
    while (!found) {
      const EngSlot* S = &d->slot[r % kRing];
      uint64_t s1 = 0;
      if (lane == 0) {
        s1 = ld_agent(&S->seq1);
        cstart = ld_agent(&S->cstart);
        cend = ld_agent(&S->cend);
        base = ld_agent(&S->base);
        offs = ld_agent(&S->offs);
        sizes = ld_agent(&S->sizes);
        out = ld_agent(&S->out);
        bad = ld_agent(&S->bad);
        n = ld_agent(&S->n);
        mode = ld_agent(&S->mode);
        flags = ld_agent(&S->flags);
        cb = ld_agent(&S->cb);
      }
      s1 = uni64(s1);
      const uint64_t ce = uni64(cend);
      if (!hinted) {
        // the page's seq is a hint: t's request or an earlier one (checked
        // below like the cursor)
        hinted = true;
        if (!(s1 == r + 1 && t >= uni64(cstart) && t < ce) && pseq1 > r + 1) {
          r = pseq1 - 1;
          via_hint = true;
          continue;
        }
      }
      if (s1 > r + 1) {
        r = s1 - kRing > r + 1 ? s1 - kRing : r + 1;
        continue;
      }
      if (s1 == r + 1 && t >= ce) {
        r++;
        continue;
      }
      if (s1 == r + 1 && t < uni64(cstart)) {  // a stale (wrapped) hint overshot: walk from the cursor
        r = r0;
        via_hint = false;
        continue;
      }
      if (s1 == r + 1) break;
      if (via_hint) {  // the hinted slot is not written (yet): walk from the cursor
        r = r0;
        via_hint = false;
        continue;
      }
      if (lane == 0) st_sys(&e.ctl->error, 2u);  // published tickets with no slot: cannot happen
      return;
    }
    cstart = uni64(cstart);
    cend = uni64(cend);
    CrcParams p = e.tab;
    p.base = (const uint8_t*)uni64(base);
    p.offsets = (const uint64_t*)uni64(offs);
    p.lengths = (const uint32_t*)uni64(sizes);
    p.n_blocks = uni64(n);
    p.flags = uni32(flags);
    p.chunk = uni32(cb);
    mode = uni32(mode);
    const uint64_t c = t - cstart;
    const uint64_t ts_slot = e.htrace ? now_ticks() : 0;
    if (mode == kVerify) {
      p.ok_out = (uint8_t*)uni64(out);
      p.n_bad = (uint32_t*)uni64(bad);
      engine_chunk<kVerify, EK>(lds, p, c);
    } else if (mode == kTrailer) {
      engine_chunk<kTrailer, EK>(lds, p, c);
    } else {
      p.out = (uint32_t*)uni64(out);
      engine_chunk<kStore, EK>(lds, p, c);
    }
    // publish the chunk: its results were stored write-through (st_through);
    // once drained they are in memory, so the count needs no release fence
    const uint64_t ts_body = e.htrace ? now_ticks() : 0;
    drain_vm();
    const uint64_t ts_drain = e.htrace ? now_ticks() : 0;
    if (lane == 0) {
      // the request's tickets are counted per group (t % 8), one line each;
      // this group's share: t' in [cstart, cend), t' % 8 == grp
      const uint32_t grp = xcc;
      const uint64_t mine = engine_group_share(cstart, cend, grp);
      const uint32_t prev = __hip_atomic_fetch_add((g32*)&d->cgrp[r % kRing][(r / kRing) & 1u][grp][0], 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t ts_count = e.htrace ? now_ticks() : 0;
      if (e.htrace && c == 0) {
        uint64_t* w = d->tr[r % kRing];
        st_agent(&w[3], ts_seen);
        st_agent(&w[1], ts_slot);
        st_agent(&w[4], ts_body);
        st_agent(&w[5], ts_drain);
        st_agent(&w[6], ts_count);
      }
      if ((uint64_t)prev + 1 == mine) {
        // the group's last chunk of the request: every other chunk of the
        // group drained its results before its add, this one before its own
        if (e.htrace && grp == (uint32_t)((cend - 1) % kCntGroups)) {
          // (trace: the group of the request's last ticket stands for "last")
          uint64_t* w = d->tr[r % kRing];
          st_agent(&w[2], now_ticks());
          st_agent(&w[7], ts_seen);
          st_agent(&w[8], ts_slot);
          st_agent(&w[9], ts_body);
          st_agent(&w[10], ts_drain);
          st_agent(&w[11], ts_count);
          drain_vm();
          for (uint32_t k = 0; k < 12; k++) st_sys(&e.htrace[(r % kRing) * kTrWords + k], ld_agent(&w[k]));
          drain_vm();
        }
        st_sys(&e.hdone[(r % kRing) * kCntGroups + grp], r + 1);
        __hip_atomic_fetch_add((g64*)&e.hdr->reqs_done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // the next ticket: claimed after this chunk is counted (the claim's add
    // is contended; issued before the chunk, every load of the chunk waited
    // for it: in-order vmcnt; issued under the chunk's last loads instead, it
    // measured the same: profiles/r06_engine_waves.log)
    t = claim();
  }
}

template <int G, int W, int EK>
__global__ void __launch_bounds__(W * 64) crc32c_engine_kernel(EngParams e) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  lds_fill_tables(lds, e.tab.tab_main, e.tab.tab_tree, tree_levels<G>() * kTreeBytes / 16, e.tab.tab_byte, 64);
  if (threadIdx.x == 0) {  // the workgroup's copy of the end / stop words, and the poll lock
    *lds64(poll_off<G>()) = 0;
    *lds32(poll_off<G>() + 8) = 0;
    *lds32(poll_off<G>() + 12) = 0;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  if (blockIdx.x == 0 && wave == 0) {
    engine_dispatch(e);
    return;
  }
  engine_work<G, EK>(e, lds);
}

// The instantiation a launch of `waves` waves per CU uses: 9-12 waves the
// two-pass build (kEK12 swaths per pass, 157 VGPRs: 3 waves per SIMD), up to
// 8 the one-pass build (kEK, 211 VGPRs).
inline const void* engine_fn(uint32_t waves) {
  return waves > (uint32_t)kEngWaves8 ? reinterpret_cast<const void*>(&crc32c_engine_kernel<kEngG, kEngMaxWaves, kEK12>)
                                      : reinterpret_cast<const void*>(&crc32c_engine_kernel<kEngG, kEngWaves8, kEK>);
}

template <int G>
constexpr size_t engine_lds(int waves) {
  (void)waves;  // the poll words sit after the largest launch's wave scratch
  return poll_off<G>() + 16;
}

// ---- host side --------------------------------------------------------------
uint64_t env_u64(const char* name, uint64_t def) {
  const char* v = getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  const unsigned long long x = strtoull(v, &end, 10);
  return end && *end == 0 ? (uint64_t)x : def;
}

using Clock = std::chrono::steady_clock;

// CPUs this process may keep busy: its affinity mask, capped by a cgroup v2
// CPU quota (cpu.max); spinning waiters get all but two of them
// (NOVA_SST_ENGINE_SPINNERS overrides).
int spinner_budget() {
  const uint64_t env = env_u64("NOVA_SST_ENGINE_SPINNERS", 0);
  if (env) return (int)std::min<uint64_t>(env, 1024);
  int cpus = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
  if (cpus <= 0) cpus = 1;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    unsigned long long period = 0;
    if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
      const double quota = strtod(q, nullptr) / (double)period;
      if (quota > 0 && quota < cpus) cpus = (int)std::ceil(quota);
    }
    fclose(f);
  }
  return std::max(1, cpus - 2);
}

// engine_submit's result when the request could not be taken back: the
// caller must NOT run the plain call (the engine may still write the outputs)
constexpr int kEngineUnsafe = -1000;
constexpr int kEngineDeclined = -1001;  // a yield storm: the plain call, nothing was published
constexpr uint64_t kStormExitsPerS = 5000;  // plain calls back to back: ~7900 yield exits / s; one per 200 us: ~2600
constexpr int64_t kStormWindowNs = 2000000, kStormHoldNs = 20000000;
// ring-full wait before the request goes to the plain call (nothing published yet)
constexpr uint64_t kRingWaitMs = 1000;

thread_local uint32_t tl_wait_delay_us = 0;  // test hook: nova_sst_engine_set_wait_delay_us
// This thread's last engine request (nova_sst_engine_last_call): where its
// time went on the host -- waiting for the engine's lock, holding it
// (ring writes, a relaunch), waiting for the completion words -- how many
// of the waits slept, and whether the wait relaunched the engine.
struct LastCall {
  uint64_t lock_ns = 0, held_ns = 0, wait_ns = 0, sleeps = 0, relaunched = 0, seq = 0, cb = 0, spun = 0;
};
thread_local LastCall tl_last;

uint64_t stream_key(hipStream_t s) {
  if (s == hipStreamPerThread)  // one alias per thread: key by the thread
    return (std::hash<std::thread::id>{}(std::this_thread::get_id()) << 1) | 1u;
  return (uint64_t)(uintptr_t)s;
}

// The engine's host lock: held for ~1 us per request (ring words), ~70 us for
// a relaunch.  Waiters spin (then yield) instead of sleeping on a futex: at
// 16 callers a woken waiter waited 0.3-8 ms for a CPU
// (profiles/r05_engine_slowest.log: lock waits of the slowest calls).
struct SpinMutex {
  std::atomic<bool> f{false};
  void lock() {
    for (uint32_t i = 0; f.exchange(true, std::memory_order_acquire); i++)
      while (f.load(std::memory_order_relaxed)) {
        if (++i < 4096) __builtin_ia32_pause();
        else std::this_thread::yield();
      }
  }
  bool try_lock() { return !f.load(std::memory_order_relaxed) && !f.exchange(true, std::memory_order_acquire); }
  void unlock() { f.store(false, std::memory_order_release); }
};

struct Engine {
  SpinMutex mu;
  bool ready = false, broken = false, running = false;
  int dev = 0;
  int cus = 0;
  hipStream_t stream = nullptr;
  EngIn* in = nullptr;         // host -> engine words (device memory through the BAR, or pinned)
  bool in_dev = false;         // `in` is device memory
  uint64_t* hdone = nullptr;   // pinned
  EngCtl* ctl = nullptr;       // pinned
  EngDev* ddev = nullptr;
  uint64_t next_seq = 0;     // the next request's seq
  uint64_t inst_first = 0;   // the running instance's first seq
  uint64_t gen = 0;          // instances launched (the running one's generation)
  std::atomic<uint64_t> inflight{0};         // requests submitted and not yet returned
  std::atomic<uint64_t> inflight_blocks{0};  // their blocks
  uint64_t requests = 0, relaunches = 0, fallbacks = 0;
  uint64_t exits[kWhyN] = {};  // instance exits by reason (kWhy*), counted at relaunch / stop
  int queue_mode = 0;          // NOVA_SST_ENGINE_QUEUE (see init_locked)
  uint32_t slice_us = 0;       // NOVA_SST_ENGINE_SLICE_US / nova_sst_engine_set_slice_us
  bool slice_set = false;      // set through the API
  uint64_t timeouts = 0, errors = 0, taken_back = 0, unsafe = 0, yield_waits = 0;
  uint64_t launch_ns_max = 0, launch_slow = 0;  // host time in launch_locked: the largest (not the first), launches over 1 ms
  uint64_t gap_ticks_max = 0;                   // the dispatchers' longest gap between two polls
  uint32_t idle_us = 0, waves = 0;
  uint32_t give_up_us = 0;                    // 0: 20 s (nova_sst_engine_set_give_up_us, a test hook)
  uint32_t drop_chunks = 0;                   // nova_sst_engine_set_drop_chunks (a test hook)
  // Take-backs waiting (with mu released) for an instance to end: no instance
  // is launched meanwhile, so the stream's last work stays the one waited for.
  int tb_active = 0;
  uint64_t host_done = 0;                     // requests whose completion words the host wrote (take_back_locked)
  std::atomic<uint32_t> timeout_ms{0};        // 0: NOVA_SST_ENGINE_TIMEOUT_MS (default 10000)
  // Waiting (round 5): at most max_spinners waiters spin; the others poll in
  // short sleeps.  16 waiters spinning on a 16-CPU cgroup quota exhausted it
  // every 100-200 ms and every thread of the process was stopped for 2-7 ms
  // (cpu.stat nr_throttled; the 2.1-2.4 ms tails at 16 threads).
  int max_spinners = 1;
  std::atomic<int> spinners{0};
  uint64_t sleep_waits = 0;  // requests whose waiter slept (approximate: not under mu)
  std::atomic<uint32_t> failures{0};          // consecutive failed requests (backoff)
  std::atomic<int64_t> avoid_until_ns{0};     // steady clock: requests go plain until then
  // Yield registry: the launches this engine must not take the CUs from.
  // `live` once the pinned control block exists; then every non-engine launch
  // of the library bumps ygen (stored to in->hyield) and records an event on
  // its stream (the stream's last one is kept).  ymu orders bumps, records and
  // the relaunch's snapshot (mu, when both are held, is taken first).
  std::atomic<bool> live{false};
  std::mutex ymu;
  uint64_t ygen = 0;
  // Yield storms: plain launches of the library arriving back to back make
  // every instance exit after a few requests (1.19 TB/s for 8 engine callers
  // against ~2.4 for the same callers' direct calls: profiles/r06_engine_mixed_gaps.log).
  // Over windows of at least 2 ms, more than kStormExitsPerS instance exits
  // for yields a second route the requests of the next 20 ms to the plain
  // path (declined, not failed).  Instance exits, not plain launches, are
  // counted: plain calls while no instance runs cost the engine nothing.
  int64_t storm_t0_ns = 0, storm_until_ns = 0;  // under mu
  uint64_t storm_x0 = 0, storm_declined = 0;     // under mu
  std::unordered_map<uint64_t, hipEvent_t> yev;
  // trace (nova_sst_engine_set_trace): per-request spans, summed under tmu
  uint64_t* htrace = nullptr;  // pinned, kRing x kTrWords
  bool trace = false;
  std::mutex tmu;
  uint64_t tr_n = 0;
  double tr_host_us = 0, tr_wait_us = 0, tr_run_us = 0, tr_gpu_us = 0, tr_host_max = 0;
  uint64_t tr_dn = 0;
  double tr_detail[11] = {};  // words 1..11 - word 0, summed (us)

  int init_locked(int d) {
    if (ready) return 0;
    dev = d;
    int err = 0;
    DevTables* t = tables(&err);
    if (!t) return err;
    cus = t->cus;
    {
      // NOVA_SST_ENGINE_CUS: run on fewer CUs (one workgroup each, whose LDS
      // tables keep any other kernel off that CU while the engine is
      // resident); workgroups go round-robin over the XCDs, so every XCD
      // still gets its share.  Rounded down to a multiple of 8.
      const uint64_t want = env_u64("NOVA_SST_ENGINE_CUS", 0);
      if (want >= 8 && want < (uint64_t)cus) cus = (int)(want & ~7ull);
    }
    // NOVA_SST_ENGINE_QUEUE: how the instance reaches the device.  HIP maps
    // streams onto GPU_MAX_HW_QUEUES shared hardware queues (4 by default),
    // whose packets run in order: work of any stream that shares the
    // engine's queue waits behind the resident kernel -- for as long as
    // requests keep arriving (tools/queue_probe.py: a torch op on such a
    // stream waited 1.6 s).  1 (default): the instance is launched as a
    // cooperative kernel, which the runtime sends to a queue of its own,
    // and the stream stays non-blocking (the probe: 16 streams and the null
    // stream unaffected); 0: a plain launch on a non-blocking stream (shared
    // queue: a stream behind the instance waits up to one time slice, below);
    // 2: a stream with a CU mask of every CU (a queue of its own, but a
    // blocking stream: the null stream waits for the engine -- measured, not
    // used).  A cooperative launch that fails falls back to 0.
    queue_mode = (int)env_u64("NOVA_SST_ENGINE_QUEUE", 1);
    // NOVA_SST_ENGINE_SLICE_US (default 20000): an instance takes no request
    // after running this long; it finishes the ones it took and exits, and the
    // next request's waiter launches the next instance.  A device-wide sync
    // (hipDeviceSynchronize, torch.cuda.synchronize) waits for the work each
    // stream had when it was called -- the running instance, not its
    // successors -- and a kernel of another library waiting for CUs gets them
    // at the instance boundary: both wait about one slice at most under
    // steady traffic, instead of until the traffic stops.  0: no slice.
    if (!slice_set)
      slice_us = (uint32_t)std::min<uint64_t>(kMaxIdleUs, env_u64("NOVA_SST_ENGINE_SLICE_US", 20000));
    hipError_t e = hipSuccess;
    if (queue_mode == 2) {
      int phys = 0;
      (void)hipDeviceGetAttribute(&phys, hipDeviceAttributeMultiprocessorCount, d);
      std::vector<uint32_t> mask((uint32_t)std::max(phys, 1) / 32 + 1, 0u);
      for (int c = 0; c < phys; c++) mask[c / 32] |= 1u << (c % 32);
      e = hipExtStreamCreateWithCUMask(&stream, (uint32_t)mask.size(), mask.data());
    } else {
      e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    }
    if (e == hipSuccess) e = alloc_in(d);
    if (e == hipSuccess)
      e = hipHostMalloc((void**)&hdone, sizeof(uint64_t) * kRing * kCntGroups, hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess)
      e = hipHostMalloc((void**)&ctl, sizeof(EngCtl), hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess)
      e = hipHostMalloc((void**)&htrace, sizeof(uint64_t) * kTrWords * kRing, hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) e = hipMalloc((void**)&ddev, sizeof(EngDev));
    if (e == hipSuccess) e = hipMemset(ddev, 0, sizeof(EngDev));  // slots: seq1 = 0 (never written)
    if (e == hipSuccess)
      for (const uint32_t wv : {(uint32_t)kEngWaves8, (uint32_t)kEngMaxWaves})
        if (e == hipSuccess)
          e = hipFuncSetAttribute(engine_fn(wv), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)engine_lds<kEngG>((int)wv));

    if (e != hipSuccess) {
      (void)hipGetLastError();
      broken = true;
      return (int)e;
    }
    memset(hdone, 0, sizeof(uint64_t) * kRing * kCntGroups);
    memset(ctl, 0, sizeof(EngCtl));
    if (!idle_us) idle_us = (uint32_t)std::min<uint64_t>(kMaxIdleUs, env_u64("NOVA_SST_ENGINE_IDLE_US", 1000));
    max_spinners = spinner_budget();
    waves = (uint32_t)env_u64("NOVA_SST_ENGINE_WAVES", kEngWaves);
    if (waves < 2 || waves > (uint32_t)kEngMaxWaves) waves = kEngWaves;
    // From here on every non-engine launch registers itself.  A launch made
    // before it saw `live` was enqueued before this store; the device-wide
    // sync below waits for it, so the first instance cannot take the CUs from it.
    live.store(true);
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
      (void)hipGetLastError();
      broken = true;
      return (int)e;
    }
    ready = true;
    return 0;
  }

  // The host -> engine words: fine-grained device memory on a large-BAR device
  // (the host's stores go through the BAR), checked by a store and a read
  // back; else, or with NOVA_SST_ENGINE_RING=host (env value 0), pinned host memory.
  hipError_t alloc_in(int d) {
    int large_bar = 0;
    (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, d);
    (void)hipGetLastError();
    const char* ev = getenv("NOVA_SST_ENGINE_RING");
    const bool want_dev = large_bar && !(ev && (!strcmp(ev, "host") || !strcmp(ev, "0")));
    if (want_dev && hipExtMallocWithFlags((void**)&in, sizeof(EngIn), hipDeviceMallocFinegrained) == hipSuccess) {
      if (hipMemset(in, 0, sizeof(EngIn)) == hipSuccess && hipDeviceSynchronize() == hipSuccess) {
        volatile EngIn* vi = in;
        vi->pad1[0] = 0x6e6f7661u;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        if (vi->pad1[0] == 0x6e6f7661u) {
          vi->pad1[0] = 0;
          in_dev = true;
          return hipSuccess;
        }
      }
      (void)hipFree(in);
      in = nullptr;
    }
    (void)hipGetLastError();
    in_dev = false;
    const hipError_t e = hipHostMalloc((void**)&in, sizeof(EngIn), hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) memset(in, 0, sizeof(EngIn));
    return e;
  }

  // Registered launches not yet finished: the engine's stream waits for them
  // (under ymu), and the instance's yield value is read in the same section,
  // so a launch registered later changes in->hyield for it.
  uint64_t wait_for_yielded_locked() {
    std::lock_guard<std::mutex> lk(ymu);
    for (auto it = yev.begin(); it != yev.end();) {
      const hipError_t q = hipEventQuery(it->second);
      if (q == hipErrorNotReady) {
        if (hipStreamWaitEvent(stream, it->second, 0) == hipSuccess) yield_waits++;
        ++it;
      } else if (yev.size() > 256) {  // finished: drop it (bounded map)
        (void)hipEventDestroy(it->second);
        it = yev.erase(it);
      } else {
        ++it;
      }
    }
    (void)hipGetLastError();
    return ygen;
  }

  // A fresh instance over requests [first, ...): the previous one has exited.
  int launch_locked(uint64_t first) {
    const auto tl0 = Clock::now();
    const int rc = launch_locked_(first);
    const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - tl0).count();
    if (gen > 1) {  // (the first launch loads the code object)
      launch_ns_max = std::max(launch_ns_max, ns);
      launch_slow += ns > 1000000 ? 1 : 0;
    }
    return rc;
  }
  int launch_locked_(uint64_t first) {
    // No host wait for the previous instance: its dispatcher has exited (it
    // took no more requests and finished the ones it took), its workers only
    // see the stop and end, and the new instance follows it in stream order.
    // (A stream sync here cost every relaunch -- every time slice, every
    // yield -- a host round trip.)  Its header was zeroed by the previous
    // instance's dispatcher (EngHdr), or at init.
    hipError_t e = hipSuccess;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    volatile EngCtl* c = ctl;
    c->exited = 0;
    c->consumed = 0;
    reinterpret_cast<volatile EngIn*>(in)->hstop = 0;
    c->error = 0;
    c->why = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    int err = 0;
    DevTables* t = tables(&err);
    if (!t) {
      running = false;
      return err;
    }
    EngParams p{};
    p.in = in;
    p.hdone = hdone;
    p.ctl = ctl;
    p.dev = ddev;
    p.hdr = &ddev->hdr[(gen + 1) & 1];
    p.hdr_next = &ddev->hdr[gen & 1];
    p.first_seq = first;
    p.gen = gen + 1;
    p.yield_gen = wait_for_yielded_locked();
    p.idle_ticks = (uint64_t)idle_us * 100;  // s_memrealtime: 100 MHz
    // 20 s (every spin of the engine is bounded); shorter only through the test hook
    p.give_up_ticks = give_up_us ? (uint64_t)give_up_us * 100 : 20ull * 100000000ull;
    p.drop_chunks = drop_chunks;
    p.slice_ticks = (uint64_t)slice_us * 100;
    p.htrace = trace ? htrace : nullptr;
    static const uint32_t page_poll = (uint32_t)env_u64("NOVA_SST_ENGINE_PAGE_POLL", 1);
    p.page_poll = page_poll;
    p.tab.tab_main = t->main[gindex(kEngG)];
    p.tab.tab_tree = t->tree;
    p.tab.tab_ft = t->ft;
    p.tab.tab_sh16 = t->sh16;
    p.tab.tab_byte = t->byte8;  // M_1 byte table (tail bytes)
    p.tab.zline = reinterpret_cast<const uint8_t*>(t->zero_word);
    if (queue_mode == 1) {
      void* args[] = {&p};
      e = hipLaunchCooperativeKernel(engine_fn(waves), dim3((uint32_t)cus), dim3(64 * waves), args,
                                     (unsigned)engine_lds<kEngG>((int)waves), stream);
      if (e != hipSuccess) {  // not available: plain launches (time-sliced like the others)
        (void)hipGetLastError();
        queue_mode = 0;
      }
    }
    if (queue_mode != 1) {
      void* args[] = {&p};
      e = hipLaunchKernel(engine_fn(waves), dim3((uint32_t)cus), dim3(64 * waves), args,
                          engine_lds<kEngG>((int)waves), stream);
    }
    if (e != hipSuccess) {
      running = false;
      return (int)e;
    }
    inst_first = first;
    running = true;
    gen++;
    return 0;
  }

  // The running instance took no more requests (idle exit, yield or stop): a
  // fresh one starts at the first request it did not take.
  int relaunch_if_exited_locked() {
    volatile EngCtl* c = ctl;
    if (running && !c->exited) return 0;
    // a take-back is waiting for the instance to end (mu released): the
    // waiters' polls relaunch once it is through
    if (tb_active) return 0;
    uint64_t first = inst_first;
    if (running) {
      first = c->consumed;
      const uint32_t why = c->why;
      exits[why < kWhyN ? why : 0]++;
      const uint64_t mg = c->maxgap;
      gap_ticks_max = mg > gap_ticks_max ? mg : gap_ticks_max;
    }
    running = false;
    relaunches++;
    return launch_locked(first);
  }

  // Request seq's 8 group completion words all hold seq + 1 or more (each
  // only grows: seq + 1, then a later occupant's seq + 1 + k * kRing).
  bool done(uint64_t seq) const {
    const volatile uint64_t* h = hdone + (seq % kRing) * kCntGroups;
    bool all = true;
    for (uint32_t g = 0; g < kCntGroups; g++) all = all && h[g] >= seq + 1;
    return all;
  }
  bool ring_slot_free(uint64_t seq) const { return seq < kRing || done(seq - kRing); }

  uint32_t timeout() const {
    static const uint32_t env = (uint32_t)env_u64("NOVA_SST_ENGINE_TIMEOUT_MS", 10000);
    const uint32_t t = timeout_ms.load();
    return t ? t : env;
  }

  // Request seq's completion words, written by the host for a request that an
  // ended instance took and left unfinished (a "lost" exit, a worker error):
  // no later instance revisits it (they start at `consumed`, past it), so
  // without them its ring slot would never free and every request reaching
  // that slot would wait kRingWaitMs and fall back.  The words
  // only grow; an ended instance writes no more of them.
  void host_mark_done(uint64_t seq) {
    volatile uint64_t* h = hdone + (seq % kRing) * kCntGroups;
    for (uint32_t g = 0; g < kCntGroups; g++)
      if (h[g] < seq + 1) h[g] = seq + 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    host_done++;
  }

  // The instance whose end a take-back waited for has ended (its stream is
  // idle) with request seq not done.  It took the request (consumed > seq):
  // mark it done from the host.  It did not record its exit (an aborted
  // kernel): the engine is not used again.
  void after_instance_end(uint64_t seq) {
    volatile EngCtl* c = ctl;
    if (done(seq)) return;
    if (c->exited) {
      if (c->consumed > seq) host_mark_done(seq);  // (<= seq: a later instance skips it)
    } else {
      broken = true;
    }
  }

  // Take request seq back (its submitter failed to get a result): returns 0
  // once the engine can no longer touch it (the plain call may run), or
  // kEngineUnsafe.  Called with lk (on mu) held; while it waits for the
  // instance to end it releases lk in 50-us steps (other
  // submitters and waiters are not held off for up to 30 s), and tb_active
  // keeps any instance from being launched meanwhile.
  int take_back_locked(uint64_t seq, std::unique_lock<SpinMutex>& lk) {
    volatile EngCtl* c = ctl;
    taken_back++;
    volatile EngIn* vi = in;
    vi->cancel[seq % kRing] = seq + 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    // device memory: reading the word back completes the posted write before
    // `alive` is read (the Dekker pair above)
    if (in_dev && vi->cancel[seq % kRing] != seq + 1) {
      unsafe++;
      broken = true;
      return kEngineUnsafe;
    }
    if (done(seq)) return 0;                // done or skipped: never touched again
    if (!running) return 0;                 // no instance: the next one skips it
    if (c->alive != gen) return 0;          // not started: it will read the cancel word
    if (c->exited && c->consumed <= seq) return 0;  // exited without taking it
    // The running instance took it or may: stop it, then wait for the request
    // (run or skipped) or for the kernel's end.
    vi->hstop = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const auto t0 = Clock::now();
    const auto limit = std::chrono::milliseconds(std::max<uint32_t>(timeout(), 30000));
    tb_active++;
    int rc = 0;
    for (;;) {
      if (done(seq)) break;
      const hipError_t q = hipStreamQuery(stream);
      if (q == hipSuccess) {  // the instance (the stream's last work) has ended
        after_instance_end(seq);
        break;
      }
      (void)hipGetLastError();
      if (Clock::now() - t0 > limit) {
        unsafe++;
        broken = true;  // an engine that neither finishes nor ends: not used again
        rc = kEngineUnsafe;
        break;
      }
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      lk.lock();
    }
    tb_active--;
    return rc;
  }

  // After a failed request: back off (100 ms, doubling to 12.8 s; reset by a success).
  void back_off() {
    const uint32_t f = failures.fetch_add(1) + 1;
    const int64_t ms = 100ll << std::min<uint32_t>(f - 1, 7);
    const int64_t until = std::chrono::duration_cast<std::chrono::nanoseconds>(
                              (Clock::now() + std::chrono::milliseconds(ms)).time_since_epoch()).count();
    avoid_until_ns.store(until);
  }
  bool backing_off() const {
    const int64_t u = avoid_until_ns.load(std::memory_order_relaxed);
    return u && std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count() < u;
  }
};

constexpr int kMaxDev = 16;
Engine g_eng[kMaxDev];

void stop_all_at_exit();

Engine* engine_for_device(int* err) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    *err = NOVA_E_NODEV;
    return nullptr;
  }
  static std::once_flag once;
  std::call_once(once, [] { atexit(stop_all_at_exit); });
  *err = 0;
  return &g_eng[dev];
}

int engine_stop(Engine& g) {
  std::lock_guard<SpinMutex> lk(g.mu);
  if (!g.ready || !g.running) return 0;
  volatile EngCtl* c = g.ctl;
  reinterpret_cast<volatile EngIn*>(g.in)->hstop = 1;
  const auto t0 = Clock::now();
  while (!c->exited) {
    if (Clock::now() - t0 > std::chrono::seconds(10)) return NOVA_E_NODEV;  // still running; retried later
    std::this_thread::yield();
  }
  const hipError_t e = hipStreamSynchronize(g.stream);
  g.inst_first = c->consumed;
  const uint32_t why = c->why;
  g.exits[why < kWhyN ? why : 0]++;
  g.running = false;
  reinterpret_cast<volatile EngIn*>(g.in)->hstop = 0;
  return e == hipSuccess ? 0 : (int)e;
}

void stop_all_at_exit() {
  for (Engine& g : g_eng)
    if (g.ready && g.running) (void)engine_stop(g);
}

Engine* engine_if_live() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
    (void)hipGetLastError();
    return nullptr;
  }
  Engine* g = &g_eng[dev];
  return g->live.load() ? g : nullptr;
}

void bump_yield_locked(Engine& g) {
  g.ygen++;
  reinterpret_cast<volatile EngIn*>(g.in)->hyield = g.ygen;
}

}  // namespace

namespace nova_dev {

void engine_yield_begin() {
  Engine* g = engine_if_live();
  if (!g) return;
  std::lock_guard<std::mutex> lk(g->ymu);
  bump_yield_locked(*g);
}

void engine_yield_end(hipStream_t s) {
  Engine* g = engine_if_live();
  if (!g) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();  // being captured into a graph: nothing to record now
    return;
  }
  std::lock_guard<std::mutex> lk(g->ymu);
  hipEvent_t& ev = g->yev[stream_key(s)];
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    ev = nullptr;
    g->yev.erase(stream_key(s));
    bump_yield_locked(*g);
    return;
  }
  if (hipEventRecord(ev, s) != hipSuccess) (void)hipGetLastError();
  bump_yield_locked(*g);
}

void engine_forget_stream(hipStream_t s) {
  Engine* g = engine_if_live();
  if (!g) return;
  std::lock_guard<std::mutex> lk(g->ymu);
  auto it = g->yev.find(stream_key(s));
  if (it == g->yev.end()) return;
  // (the caller synchronised the stream; a stream wait that captured the
  // event keeps its own reference)
  (void)hipEventDestroy(it->second);
  (void)hipGetLastError();
  g->yev.erase(it);
}

// Runs one request on the engine and waits for it.  Returns 0; nonzero when
// the engine did not run it and cannot touch it any more (the caller then
// makes the plain call); kEngineUnsafe when it could not be taken back (no
// plain call: an error for the caller).
int engine_submit(int mode, const uint8_t* base, const uint64_t* offs, const uint32_t* sizes, uint64_t n,
                  uint32_t flags, void* out, uint32_t* bad) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  Engine& g = *gp;
  // blocks per chunk fixed at 1..16 (0: adaptive, below)
  static const uint32_t cb_fixed = (uint32_t)std::min<uint64_t>(16, env_u64("NOVA_SST_ENGINE_CB", 0));
  if (g.backing_off()) return NOVA_E_NODEV;
  uint64_t seq = 0;
  bool failed = false;
  LastCall lc;
  const auto t_lock = Clock::now();
  {
    std::unique_lock<SpinMutex> lk(g.mu);
    const auto t_held = Clock::now();
    lc.lock_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_held - t_lock).count();
    if (g.broken) return NOVA_E_NODEV;
    {  // yield storm: decline (the caller runs the plain call) until it is over
      const int64_t now = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                              Clock::now().time_since_epoch()).count();
      if (now - g.storm_t0_ns >= kStormWindowNs) {
        const uint64_t x = g.exits[kWhyYield];
        if (g.storm_t0_ns && (x - g.storm_x0) * 1000000000ull > kStormExitsPerS * (uint64_t)(now - g.storm_t0_ns))
          g.storm_until_ns = now + kStormHoldNs;
        g.storm_t0_ns = now;
        g.storm_x0 = x;
      }
      if (now < g.storm_until_ns) {
        g.storm_declined++;
        return kEngineDeclined;
      }
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    if ((err = g.init_locked(dev))) return err;
    seq = g.next_seq;
    const auto tw = Clock::now();
    while (!g.ring_slot_free(seq)) {  // kRing requests in flight: wait for the oldest
      // (a taken-back request's slot frees once an instance skips it)
      if ((err = g.relaunch_if_exited_locked()) || Clock::now() - tw > std::chrono::milliseconds(kRingWaitMs))
        return err ? err : NOVA_E_NODEV;  // nothing published: the plain call is safe
      lk.unlock();
      std::this_thread::yield();
      lk.lock();
      seq = g.next_seq;
    }
    g.next_seq = seq + 1;
    g.inflight.fetch_add(1);
    const uint64_t blocks = g.inflight_blocks.fetch_add(n) + n;
    // blocks per chunk, a multiple of 4 (one round of the chunk body): short
    // chunks (latency) when the engine is quiet, longer ones (fewer tickets per
    // block) when it is busy.  12 waves (1.5x the workers): 4 per 20K blocks in
    // flight, rounded down -- for 4K-block tables 4 up to 9 callers, 8 at 10-14,
    // 12 at 15-19 (each the best of 4 / 8 / 12 / 16 in the sweeps,
    // profiles/r06_engine_cb12.log); 8 waves: 4 per 16K, rounded up
    // (tools/concurrent_sst.py sweeps, round 4).
    const uint64_t cb_auto = g.waves > (uint32_t)kEngWaves8 ? 4 * std::max<uint64_t>(1, blocks / 20480)
                                                            : 4 * ((blocks + 16383) / 16384);
    const uint32_t cb = cb_fixed ? cb_fixed : (uint32_t)std::min<uint64_t>(16, cb_auto);
    const uint32_t half[kWords] = {
        (uint32_t)(uint64_t)base, (uint32_t)((uint64_t)base >> 32), (uint32_t)(uint64_t)offs,
        (uint32_t)((uint64_t)offs >> 32), (uint32_t)(uint64_t)sizes, (uint32_t)((uint64_t)sizes >> 32),
        (uint32_t)(uint64_t)out, (uint32_t)((uint64_t)out >> 32), (uint32_t)(uint64_t)bad,
        (uint32_t)((uint64_t)bad >> 32), (uint32_t)n, (flags & 0xffffu) | ((uint32_t)mode << 16) | (cb << 20)};
    const uint64_t tag = (uint64_t)(uint32_t)(seq + 1) << 32;
    volatile uint64_t* w = reinterpret_cast<volatile EngIn*>(g.in)->ring[seq % kRing].w;
    for (uint32_t k = 0; k < kWords; k++) w[k] = tag | half[k];  // one 8-B store each
    std::atomic_thread_fence(std::memory_order_seq_cst);
    reinterpret_cast<volatile EngIn*>(g.in)->htail = seq + 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    g.requests++;
    if (g.relaunch_if_exited_locked()) {
      g.errors++;
      failed = true;
    }
    lc.seq = seq;
    lc.cb = cb;
    lc.held_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t_held).count();
  }
  if (tl_wait_delay_us)  // test hook: this waiter starts late (past a ring turn)
    std::this_thread::sleep_for(std::chrono::microseconds(tl_wait_delay_us));
  // wait for the completion word; relaunch if the instance exited without
  // taking this request
  const auto t_submit = Clock::now();
  const volatile EngCtl* c = g.ctl;
  const auto t0 = Clock::now();
  const uint32_t timeout_ms = g.timeout();
  // The words only grow (seq + 1, then seq + 1 + kRing once this request is
  // done and its ring slot reused), so a waiter descheduled past a full ring
  // turn still sees its request done.
  bool spinning = g.spinners.fetch_add(1) < g.max_spinners;
  if (!spinning) g.spinners.fetch_sub(1);
  int slack = -1;  // the thread's timer slack before its first sleep (restored after)
  for (uint64_t spin = 0; !failed; spin++) {
    if (g.done(seq)) break;
    if (!spinning || (spin & 255) == 255) {
      if (c->error) {
        std::lock_guard<SpinMutex> lk(g.mu);
        g.errors++;
        failed = true;
        break;
      }
      if (c->exited) {
        std::lock_guard<SpinMutex> lk(g.mu);
        lc.relaunched++;
        if (!g.done(seq) && g.relaunch_if_exited_locked()) {
          g.errors++;
          failed = true;
          break;
        }
      }
      if (Clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
        std::lock_guard<SpinMutex> lk(g.mu);
        g.timeouts++;
        failed = true;
        break;
      }
      if (spinning && spin > (1u << 16)) std::this_thread::yield();
    }
    if (spinning) {
      __builtin_ia32_pause();
      continue;
    }
    // more waiters than CPUs to spin on: poll every ~10 us, asleep
    if (slack < 0) {
      slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
      (void)prctl(PR_SET_TIMERSLACK, 1000ul, 0, 0, 0);  // 1 us: the sleeps end on time
      g.sleep_waits++;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(8));
    lc.sleeps++;
    if (g.spinners.load(std::memory_order_relaxed) < g.max_spinners) {  // a spinner left: take its place
      if (g.spinners.fetch_add(1) < g.max_spinners) spinning = true;
      else g.spinners.fetch_sub(1);
    }
  }
  if (spinning) g.spinners.fetch_sub(1);
  lc.spun = spinning ? 1 : 0;
  lc.wait_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
  tl_last = lc;
  if (slack >= 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
  if (failed) {
    int rc = 0;
    {
      std::unique_lock<SpinMutex> lk(g.mu);
      rc = g.take_back_locked(seq, lk);
    }
    g.back_off();
    g.inflight.fetch_sub(1);
    g.inflight_blocks.fetch_sub(n);
    return rc ? rc : NOVA_E_NODEV;
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  g.inflight.fetch_sub(1);
  g.inflight_blocks.fetch_sub(n);
  if (g.failures.load(std::memory_order_relaxed)) g.failures.store(0);
  if (g.trace) {  // this request's spans (the stamps were stored before its completion word)
    const double host_us = std::chrono::duration<double, std::micro>(Clock::now() - t_submit).count();
    const volatile uint64_t* tr = g.htrace + (seq % kRing) * kTrWords;
    const uint64_t t0 = tr[0], t1 = tr[1], t2 = tr[2];
    uint64_t w[12];
    bool all = true;
    for (int k = 0; k < 12; k++) {
      w[k] = tr[k];
      all = all && w[k] >= t0 && w[k] - t0 < 100000000ull;  // stamped, within a second
    }
    std::lock_guard<std::mutex> lk(g.tmu);
    g.tr_n++;
    g.tr_host_us += host_us;
    g.tr_host_max = host_us > g.tr_host_max ? host_us : g.tr_host_max;
    if (t1 >= t0 && t2 >= t1) {  // s_memrealtime: 100 MHz
      g.tr_wait_us += (double)(t1 - t0) / 100.0;
      g.tr_run_us += (double)(t2 - t1) / 100.0;
      g.tr_gpu_us += (double)(t2 - t0) / 100.0;
    }
    if (all) {
      g.tr_dn++;
      for (int k = 1; k < 12; k++) g.tr_detail[k - 1] += (double)(w[k] - t0) / 100.0;
    }
  }
  return 0;
}

bool engine_unsafe(int rc) { return rc == kEngineUnsafe; }
bool engine_declined(int rc) { return rc == kEngineDeclined; }

std::atomic<int> g_engine_override{-1};  // nova_sst_engine_set_enabled (-1: NOVA_SST_ENGINE)

bool engine_enabled() {
  static const bool env_on = env_u64("NOVA_SST_ENGINE", 1) != 0;
  const int o = g_engine_override.load();
  return o < 0 ? env_on : o != 0;
}

void engine_count_fallback() {
  int err = 0;
  Engine* g = engine_for_device(&err);
  if (!g) return;
  std::lock_guard<SpinMutex> lk(g->mu);
  g->fallbacks++;
}

}  // namespace nova_dev

extern "C" {

int nova_sst_engine_start(void) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  if (gp->broken) return NOVA_E_NODEV;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if ((err = gp->init_locked(dev))) return err;
  return gp->relaunch_if_exited_locked();
}

int nova_sst_engine_stop(void) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  return engine_stop(*gp);
}

int nova_sst_engine_stats(uint64_t* requests, uint64_t* launches, uint64_t* fallbacks, int* running) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  if (requests) *requests = gp->requests;
  if (launches) *launches = gp->gen;
  if (fallbacks) *fallbacks = gp->fallbacks;
  if (running) *running = gp->running && gp->ctl && !((volatile EngCtl*)gp->ctl)->exited ? 1 : 0;
  return 0;
}

int nova_sst_engine_counters(uint64_t* out, size_t n) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  if (!out) return NOVA_E_INVAL;
  std::lock_guard<SpinMutex> lk(gp->mu);
  const uint64_t v[NOVA_ENGINE_COUNTERS] = {
      gp->requests, gp->gen, gp->fallbacks,
      (uint64_t)(gp->running && gp->ctl && !((volatile EngCtl*)gp->ctl)->exited ? 1 : 0),
      gp->exits[kWhyIdle], gp->exits[kWhyYield], gp->exits[kWhyStop], gp->exits[kWhyLost],
      gp->timeouts, gp->errors, gp->taken_back, gp->unsafe, gp->yield_waits, gp->ygen,
      (uint64_t)gp->broken, (uint64_t)gp->backing_off(), gp->exits[kWhySlice], gp->launch_ns_max / 1000,
      gp->launch_slow, gp->gap_ticks_max / 100, gp->sleep_waits, (uint64_t)gp->max_spinners,
      (uint64_t)gp->in_dev, gp->host_done, (uint64_t)gp->waves, gp->storm_declined};
  for (size_t i = 0; i < n && i < NOVA_ENGINE_COUNTERS; i++) out[i] = v[i];
  return 0;
}

int nova_sst_engine_set_trace(int on) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  gp->trace = on != 0;  // from the next instance
  std::lock_guard<std::mutex> lt(gp->tmu);
  gp->tr_n = 0;
  gp->tr_host_us = gp->tr_wait_us = gp->tr_run_us = gp->tr_gpu_us = gp->tr_host_max = 0;
  gp->tr_dn = 0;
  for (double& x : gp->tr_detail) x = 0;
  return 0;
}

int nova_sst_engine_trace_detail(uint64_t* n, double* out11) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<std::mutex> lt(gp->tmu);
  const double k = gp->tr_dn ? 1.0 / (double)gp->tr_dn : 0.0;
  if (n) *n = gp->tr_dn;
  if (out11)
    for (int i = 0; i < 11; i++) out11[i] = gp->tr_detail[i] * k;
  return 0;
}

int nova_sst_engine_trace_stats(uint64_t* n, double* out5) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<std::mutex> lt(gp->tmu);
  const double k = gp->tr_n ? 1.0 / (double)gp->tr_n : 0.0;
  if (n) *n = gp->tr_n;
  if (out5) {
    out5[0] = gp->tr_host_us * k;  // submit -> completion seen, host clock
    out5[1] = gp->tr_wait_us * k;  // dispatched -> first chunk started, GPU clock
    out5[2] = gp->tr_run_us * k;   // first chunk started -> last chunk done
    out5[3] = gp->tr_gpu_us * k;   // dispatched -> last chunk done
    out5[4] = gp->tr_host_max;
  }
  return 0;
}

int nova_sst_engine_set_enabled(int on) {
  if (on < -1 || on > 1) return NOVA_E_INVAL;
  g_engine_override.store(on);
  return 0;
}

int nova_sst_engine_set_idle_us(uint32_t us) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  // the next instance; at most 1 s, below the workers' 20 s give-up
  gp->idle_us = us ? std::min<uint32_t>(us, kMaxIdleUs) : 1000;
  return 0;
}

int nova_sst_engine_set_slice_us(uint32_t us) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  // from the next instance; ~0u: no slice; 0: back to NOVA_SST_ENGINE_SLICE_US
  if (us == 0) {
    gp->slice_set = false;
    gp->slice_us = (uint32_t)std::min<uint64_t>(kMaxIdleUs, env_u64("NOVA_SST_ENGINE_SLICE_US", 20000));
  } else {
    gp->slice_set = true;
    gp->slice_us = us == ~0u ? 0u : std::min<uint32_t>(us, kMaxIdleUs);
  }
  return 0;
}

int nova_sst_engine_set_timeout_ms(uint32_t ms) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  gp->timeout_ms.store(ms);
  return 0;
}

void nova_sst_engine_set_wait_delay_us(uint32_t us) { tl_wait_delay_us = us; }

int nova_sst_engine_set_give_up_us(uint32_t us) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  gp->give_up_us = us;  // from the next instance
  return 0;
}

int nova_sst_engine_set_drop_chunks(uint32_t on) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  gp->drop_chunks = on ? 1u : 0u;  // from the next instance
  return 0;
}

int nova_sst_engine_last_call(uint64_t* out, size_t n) {
  if (!out) return NOVA_E_INVAL;
  const uint64_t v[8] = {tl_last.lock_ns, tl_last.held_ns, tl_last.wait_ns, tl_last.sleeps,
                         tl_last.relaunched, tl_last.seq, tl_last.cb, tl_last.spun};
  for (size_t i = 0; i < n && i < 8; i++) out[i] = v[i];
  return 0;
}

int nova_sst_engine_yield(void* stream) {
  nova_dev::engine_yield_begin();
  nova_dev::engine_yield_end((hipStream_t)stream);
  return 0;
}

int nova_sst_engine_reset(void) {
  int err = 0;
  Engine* gp = engine_for_device(&err);
  if (!gp) return err;
  std::lock_guard<SpinMutex> lk(gp->mu);
  gp->failures.store(0);
  gp->avoid_until_ns.store(0);
  return 0;
}

}  // extern "C"
