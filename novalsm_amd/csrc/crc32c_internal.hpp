// Declarations shared by the two translation units of the engine:
//   crc32c_device.hip  the product: kernels instantiated for production,
//                      per-device tables, dispatch and the C-ABI
//                      (libnova_crc32c.so);
//   crc32c_diag.hip    diagnostics only: experiment kernels, timing-ablation
//                      instantiations and the nova_diag_* knobs, linked with
//                      the product object into libnova_crc32c_diag.so.
// The product calls into the diagnostics TU only through the hook table
// g_diag, which only crc32c_diag.hip fills (null in libnova_crc32c.so).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <unordered_map>

#include "../../include/nova_crc32c.h"

namespace nova_dev {


constexpr int kWaves = 16;                 // waves per workgroup
constexpr int kThreads = kWaves * 64;
constexpr uint32_t kMainBytes = 131072;    // 4 tables x 256 x 32 replicas x 4 B
constexpr int kTreeLevels = 8;             // M4, M8, M16, ..., M512 (M256/M512: burst kernel)
constexpr uint32_t kTreeBytes = 4096;      // per level
constexpr uint32_t kWaveScratch = 512;     // per wave: 2x16 prefixes (+pad) + accumulators
constexpr int kNumG = 5;                   // G = 1, 2, 4, 8, 16

// kLogWrite / kLogVerify: offsets[i] points at a log record header
// [LE32 masked crc][LE16 length][type] (db/log_format.h:27-30); the CRC covers
// type byte + payload (db/log_writer.cc:112-114, db/log_reader.cc:251-262).
enum Mode { kStore = 0, kTrailer = 1, kVerify = 2, kLogWrite = 3, kLogVerify = 4 };

struct CrcParams {
  const uint8_t* base;
  const uint64_t* offsets;   // null: strided
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t len;
  uint32_t flags;
  const uint32_t* init;      // may be null (units kernel); stream kernel: never null
  uint32_t init_stride;      // 1, or 0 with init -> a zero word (stream kernel)
  uint32_t* out;             // kStore
  uint8_t* ok_out;           // kVerify
  uint32_t* n_bad;           // kVerify, may be null
  uint64_t n_blocks;
  uint32_t seg;              // segment bytes (multiple of 16); 0 = one unit per block
  uint32_t chunk;            // blocks per wave chunk (<= 16)
  uint64_t n_chunks;
  const uint32_t* tab_main;  // replicated LDS image, 32768 u32
  const uint32_t* tab_tree;  // kTreeLevels x 1024 u32
  const uint32_t* tab_ft;    // 16 x 1024 u32
  const uint32_t* tab_sh16;  // 32 x 1024 u32
  uint64_t* stamps;          // diagnostics: per-wave {tables loaded, done} (or null)
  uint32_t* sched;           // stream kernel: per-workgroup claim counters, 64 B apart
  uint32_t steal_limit;      // stream kernel: max other workgroups probed when out of work
  uint32_t bpg;              // stream kernel: consecutive blocks per lane group per round
  const uint32_t* tab_byte;  // flat kernel: one-byte step table M_1 (256 u32)
  const uint8_t* zline;      // 1 KiB of zeros (target of masked-off loads)
  // flat kernel: descriptor arrays are always loaded (no branch), absent ones
  // read word 0 of zline through a zero mask; offset = offsets[i & omask] +
  // i * stride, length = lengths[i & lmask] + len, init = init[i & imask].
  uint64_t omask, lmask, imask;
  const uint32_t* perm;      // rounds kernel: block index per sorted position (or null)
  uint32_t sort_local;       // rounds kernel: sort each chunk's blocks by step count
  uint64_t buf_len;          // log modes: bytes of the log image at base (bounds of every record)
  // log-stream kernel (crc32c_logstream_kernel) and its gated fallback
  const uint32_t* first;     // first record of each 32 KiB log block (n_lblocks + 1 entries)
  uint64_t n_lblocks;        // log blocks in the image
  uint32_t* ls_flag;         // bit 0: offsets unsorted (pre-pass), bit 1: records overlap
  uint32_t* ls_bad;          // log-stream mismatch count (added to n_bad unless it falls back)
  uint32_t* ls_left;         // records the log-stream kernel leaves to the rounds follow-up
  const uint32_t* gate;      // rounds kernel: run only if *gate != 0 (else fold ls_bad in)
  // trailer writer (rounds kernel): *tr_flag == 0 (trailer_layout_kernel found
  // the blocks ascending and disjoint) lets each block with init[i] != 0 (the
  // pre-pass's eligibility array) rewrite the whole 64-B pieces holding its
  // trailer; null or nonzero: byte stores
  const uint32_t* tr_flag;
  // trailer writer, two-pass form: 1 at blocks whose whole-piece window must not
  // be used (the first and last block of each table of a coalesced batch); may be null
  const uint8_t* tr_last;
  uint32_t out_pos;  // host: launch the kVarOutPos instantiation (log records in p.perm's order)
  uint32_t wvar;  // diagnostics (timing, kVarDiag): 1 = whole-piece stores non-temporal,
                  // 2 = no result writes, 3 = no per-block epilogue and no writes;
                  // log records: 4 / 5 / 6 = the decode stage reads no tail line /
                  // no header / neither (WRONG results, written); 7 = the
                  // XCD-contiguous chunk order with a permutation too; 8 / 9 =
                  // no head masking / no group fold at a round's end (WRONG
                  // results, written); 4-6, 8, 9 count no mismatches
};

// Kernel variants (diagnostics / tuning; 0 = production).
constexpr int kVarNoLookup = 1;  // ablation: stream step without table lookups
constexpr int kVarCached = 2;    // default-policy data loads (production uses nt)
constexpr int kVarStamps = 4;    // record per-wave s_memrealtime stamps (diagnostics)
constexpr int kVarStaticClaims = 8;  // stream kernel: claims without atomics (diagnostics)
constexpr int kVarNarrow = 16;  // flat/rounds/units: one word's lookups in flight (fold4, A/B)
constexpr int kVarWide = 32;    // stream kernel: a swath's 16 lookups in flight (fold4w, A/B)
constexpr int kVarLsFast = 64;  // log-stream kernel: every swath on the fast path (ablation: WRONG CRCs)
constexpr int kVarInit = 128;   // rounds kernel, store mode: per-block init values (general head masking)
constexpr int kVarNoTail = 256;  // rounds kernel ablation: no tail-line loads (WRONG CRCs)
// Diagnostics instantiation of the rounds kernel (crc32c_diag.hip only): the
// log-stream follow-up gate, the whole-piece store forms and the store/epilogue
// timing ablations (CrcParams::gate, tr_flag, wvar) are compiled in.  The
// product's instantiations (VAR 0, kVarInit) carry none of it.
constexpr int kVarDiag = 512;
// Rounds kernel, log modes: results indexed by the record's position in
// CrcParams::perm's order (dense per chunk) instead of its index; log write
// stores Mask(crc) to out[pos] and the record's status to ok_out[pos] and
// leaves the image alone.  log_unperm_kernel finishes the call.
constexpr int kVarOutPos = 1024;
// Rounds kernel: the per-block epilogue (tail bytes, mask, store / compare)
// once per round for the round's groups (rounds 1-2 form; the diagnostics
// store forms need it) instead of once per chunk for all 64 blocks lane-parallel.
constexpr int kVarRoundEpi = 2048;
// Units chunk body inside the persistent SSTable engine (crc32c_engine.hip):
// every load of caller memory is non-temporal (no stale L1 lines of a buffer
// rewritten between requests) and verify loads each stored CRC with its
// descriptor.
constexpr int kVarEngine = 4096;
// Rounds kernel (diagnostics A/B): 16 waves per workgroup
// (launch bound 1024 threads: 128 VGPRs) instead of 12 (168 VGPRs).
constexpr int kVarW16 = 8192;
// Rounds kernel (diagnostics A/B): fold the empty steps a wave issues while
// its next chunk's descriptors load, as rounds 1-4 did (the product skips them).
constexpr int kVarFoldEmpty = 16384;
// Data-load cache policy A/Bs (diagnostics): system scope (a volatile 16-B
// load: sc0 sc1) and device scope (two 8-B agent-scope atomic loads: sc1, L1
// bypassed, L2 allocated as usual), against nt (product at 8+ lanes) and the
// default policy (kVarCached, product for log records at 2-4 lanes).
constexpr int kVarLdSys = 32768;
constexpr int kVarLdDev = 65536;

constexpr size_t kLdsMax = 160 * 1024;  // per CU on MI355X
constexpr int kMaxDevices = 64;
constexpr int kSchedWords = 256 * 16;  // per stream: up to 256 workgroups x 64 B

// ---- per-device tables ------------------------------------------------------
struct DevTables {
  uint32_t* main[kNumG] = {};
  uint32_t* tree = nullptr;
  uint32_t* ft = nullptr;
  uint32_t* sh16 = nullptr;
  uint32_t* zero_word = nullptr;  // 1 KiB of zeros: the NULL-init stand-in and the zero line
                                  // (the rounds kernel reads up to 48G + 16 bytes past it)
  uint32_t* byte8 = nullptr;      // M_1 byte table (flat kernel tail steps)
  uint32_t* byte8lm = nullptr;    // the same + 17 x 16-B prefix masks (rounds kernel head steps)
  uint32_t* op1024 = nullptr;     // M_1024 byte tables (burst kernel stream step)
  uint32_t* op1024r = nullptr;    // diagnostics: the same, 16-way bank-replicated
  uint32_t* ls_tabs = nullptr;    // diagnostics: log-stream kernel LDS tail (M4, M16, prefix masks)
  int cus = 0;
  int err = 0;
  // Stream-ordered scratch pool (StreamScratch): keeps up to 512 MiB mapped
  // between calls.  With the default pool's release threshold (0) every sync
  // handed the scratch back to the driver and the next call mapped it again:
  // a trailer writer waited on per table paid ~20-200 us for it
  // (profiles/r04_trailer_forms_sizes*.log).  Null: hipMallocAsync.
  hipMemPool_t pool = nullptr;
  // Claim counters, one 16 KiB slot per HIP stream (256 workgroups x 64 B).
  // Launches on one stream run in order, so no two running launches share a
  // slot; each launch leaves its slot zeroed (sched_release).  A slot lives
  // until nova_stream_release(stream) (or process exit); the library's own
  // streams (port hook, host-streamed path) come from a pool and are reused.
  // The lock covers only the map: nothing waits on the GPU while holding it.
  std::mutex sched_mu;
  std::unordered_map<uint64_t, uint32_t*> sched_by_stream;
};

DevTables* tables(int* err);
uint32_t* sched_slot(DevTables* t, hipStream_t stream);
// The product dispatch (crc32c_device.hip run()) for a variable-length batch
// described by p (base may be 0 with absolute offsets): crc32c_queue.hip.
int dispatch(int mode, CrcParams& p, hipStream_t stream);
int gindex(int G);
int upload_u32(uint32_t** dst, const uint32_t* src, size_t n);  // hipMalloc + copy

// ---- tuning knobs (thread-local; 0 / -1 = the product's defaults) ----------
// nova_crc32c_set_tuning sets g_tune_g / g_tune_seg; the others are set only
// by the diagnostics library's nova_diag_* entry points.
extern thread_local std::atomic<int> g_tune_g;
extern thread_local std::atomic<uint32_t> g_tune_seg;
extern thread_local std::atomic<int> g_tune_static_pct;  // steal probe limit (-1 = default)
extern thread_local std::atomic<int> g_tune_var;         // kernel variant (ablations)
extern thread_local std::atomic<int> g_tune_bpg;
extern thread_local std::atomic<int> g_tune_chunk;
extern thread_local std::atomic<int> g_tune_waves;       // waves per workgroup (0 = per-kernel default)
extern thread_local std::atomic<int> g_tune_parity;      // XOR parity kernel variant (0 = default)
extern thread_local std::atomic<int> g_tune_kernel;      // VarKernel (0 = auto)
// rounds kernel order: 0 blocks in order, 1 whole-batch sort (diagnostics),
// 2 each chunk sorted + large logs in windows (log_sort_kernel), results by
// position (default); diagnostics A/B for large logs: 3 windows only, by
// position; 4 windows + chunks, results in place; 5 windows only, in place
extern thread_local std::atomic<int> g_tune_sort;
// log sort window in records (0 = 512); negative: -window, and log write sorts too
extern thread_local std::atomic<int> g_tune_logwin;
extern thread_local std::atomic<int> g_tune_logkey;
extern thread_local std::atomic<int> g_tune_trailer_1pass;  // trailer / log-write store forms
extern thread_local std::atomic<int> g_tune_burst;       // 0 auto, 16/64/65 force, -1 off
extern thread_local std::atomic<int> g_tune_split;       // 0 auto, 1 force, -1 off
extern thread_local std::atomic<uint64_t*> g_diag_stamps;

int waves_per_wg(int def);
uint64_t flat_waves();

// ---- dispatch -----------------------------------------------------------------
enum VarKernel { kAuto = 0, kUnitsK = 1, kFlatK = 2, kRoundsK = 3, kLogStreamK = 4 };
struct Plan {
  int kernel;
  int G;
  uint32_t seg;
  uint32_t chunk;  // rounds kernel: blocks per claimed chunk (0: the kernel's default)
};
Plan plan(uint64_t n_blocks, uint64_t bytes_per_block, bool uniform, int mode, bool large,
          uint32_t cus = 256);

// Scratch that lives between launches of ONE call is allocated and freed in
// stream order (hipMallocAsync / hipFreeAsync from the device's default
// pool): every call owns its own array, so calls from several host threads
// on one stream cannot see each other's scratch, and nothing is freed while
// a kernel still reads it.
struct StreamScratch {
  void* p = nullptr;
  hipStream_t s = nullptr;
  int alloc(size_t bytes, hipStream_t stream) {
    s = stream;
    int err = 0;
    DevTables* t = tables(&err);
    if (t && t->pool && hipMallocFromPoolAsync(&p, bytes, t->pool, stream) == hipSuccess) return 0;
    (void)hipGetLastError();
    if (hipMallocAsync(&p, bytes, stream) == hipSuccess) return 0;
    p = nullptr;
    (void)hipGetLastError();  // not sticky for the caller's next launch check
    return NOVA_E_NOMEM;
  }
  ~StreamScratch() {
    if (p) (void)hipFreeAsync(p, s);
  }
};

// The kernels' launchers are host templates in crc32c_kernels.hpp
// (launch_rounds_v<MODE, VAR> and friends): each TU instantiates the variants
// it launches, the product only VAR 0 (and kVarInit).

// Trailer writer for rounds-kernel batches (crc32c_device.hip): the CRC pass
// into a stream-ordered array, then the trailers patched into whole 64-B
// pieces.  trailer_layout: the pieces' eligibility pre-pass
// (zeroes *flag first); both return 0 or an error.
int trailer_two_pass(CrcParams& p, int G, uint32_t chunk, DevTables* t, hipStream_t stream);

// The persistent per-SSTable engine (crc32c_engine.hip):
// engine_submit runs one request (kStore: out = uint32_t* CRCs; kTrailer: out
// unused; kVerify: out = uint8_t* ok flags, bad = mismatch counter) and waits
// for it; nonzero = the engine could not run it (the caller makes the plain
// call).  NOVA_SST_ENGINE=0 turns it off (engine_enabled).
int engine_submit(int mode, const uint8_t* base, const uint64_t* offs, const uint32_t* sizes, uint64_t n,
                  uint32_t flags, void* out, uint32_t* bad);
bool engine_enabled();
void engine_count_fallback();
// Engine ticket groups (crc32c_engine.hip): ticket t goes to group t % 8,
// taken by the waves of the workgroups w with w % 8 == group (every group has
// workgroups whenever the grid has at least 8); a request's chunk tickets
// [cstart, cend) hold group_share(cstart, cend, g) tickets of group g, counted
// on g's completion line, and the request is done when groups_used(...) lines
// are full.  Host-callable for the CPU test (nova_diag_engine_groups).
constexpr uint32_t kEngGroups = 8;
__host__ __device__ inline uint32_t engine_group_of_wg(uint32_t wg) { return wg & (kEngGroups - 1); }
__host__ __device__ inline uint64_t engine_group_below(uint64_t n, uint32_t g) {
  return n > g ? (n - g + kEngGroups - 1) / kEngGroups : 0;  // tickets t < n with t % 8 == g
}
__host__ __device__ inline uint64_t engine_group_share(uint64_t cstart, uint64_t cend, uint32_t g) {
  return engine_group_below(cend, g) - engine_group_below(cstart, g);
}
__host__ __device__ inline uint64_t engine_groups_used(uint64_t cstart, uint64_t cend) {
  return cend - cstart < kEngGroups ? cend - cstart : kEngGroups;
}
// engine_submit's code for a request the engine could not be made to let go
// of: the caller returns an error and must not run the plain call.
bool engine_unsafe(int rc);
// Sharing the GPU with the engine: every launch of the library that is not the
// engine's is bracketed by engine_yield_begin (the resident engine starts to
// drain and exit) and engine_yield_end(stream) once it is enqueued (the next
// engine instance waits for it).  Both do nothing until the engine of the
// current device has been started once.  engine_forget_stream drops a
// released stream's event.
void engine_yield_begin();
void engine_yield_end(hipStream_t s);
void engine_forget_stream(hipStream_t s);
struct EngineYield {
  hipStream_t s;
  explicit EngineYield(hipStream_t st) : s(st) { engine_yield_begin(); }
  ~EngineYield() { engine_yield_end(s); }
  EngineYield(const EngineYield&) = delete;
  EngineYield& operator=(const EngineYield&) = delete;
};
int trailer_layout(const CrcParams& p, DevTables* t, hipStream_t stream, uint32_t* elig, uint32_t* flag);

// ---- diagnostics hooks (crc32c_diag.hip fills g_diag; null in the product) --
// Each returns true when it took over the launch, with its result in *rc.
struct DiagHooks {
  int (*init_device)(DevTables* t);  // diagnostics tables and kernel attributes
  // run(): before the streaming-kernel choice (log-stream experiment)
  bool (*run_early)(int mode, CrcParams& p, DevTables* t, hipStream_t s, int* rc);
  // run(): once planned (store forms, flat kernel)
  bool (*run_planned)(int mode, CrcParams& p, const Plan& pl, DevTables* t, hipStream_t s, int* rc);
  // kernel variants in place of the product launch (knobs: g_tune_var,
  // g_tune_sort, g_tune_trailer_1pass, stamps)
  bool (*rounds)(int mode, int G, CrcParams& p, DevTables* t, hipStream_t s, uint32_t chunk, int* rc);
  bool (*units)(int mode, int G, CrcParams& p, DevTables* t, hipStream_t s, int* rc);
  bool (*stream)(int G, CrcParams& p, DevTables* t, hipStream_t s, int* rc);
  bool (*burst)(int V, int mode, CrcParams& p, DevTables* t, hipStream_t s, int* rc);
  // nova_crc32c_describe of a flat-kernel plan
  int (*describe_flat)(int G, int mode, char* buf, size_t buflen);
  // nova_xor_parity: a variant (u chunks per lane, fu fragments per load) the
  // product does not instantiate (rejected A/B forms, e.g. 16 x 1, which spills)
  bool (*parity)(int u, int fu, const uint8_t* base, const uint64_t* frag_offsets, uint32_t n_frags,
                 uint64_t parity_len, uint8_t* out, uint64_t wgs, hipStream_t s, int* rc);
};
extern DiagHooks* g_diag;

}  // namespace nova_dev
