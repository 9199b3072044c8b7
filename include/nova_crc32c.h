/*
 * nova_crc32c.h -- C-ABI of the MI355X-native batched CRC32C block-checksum
 * engine (drop-in for NovaLSM's per-SSTable-block checksum path).
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures; a
 * stream is passed as `void*` holding a hipStream_t, NULL = default stream).
 * Every entry point below names the reference interface it replaces.
 *
 * Conventions
 *   - Device-batch entry points take DEVICE pointers (hipMalloc'd, or any
 *     address the GPU can load from) for data, descriptors and outputs, enqueue
 *     work on `stream` and return without synchronising.  Return 0 on success,
 *     a hipError_t value (> 0) or a NOVA_E_* code (< 0) on failure.  They never
 *     fall back to the CPU: with no usable GPU they return an error.
 *   - Results are bit-identical to looping leveldb::crc32c::Extend
 *     (util/crc32c.cc:487-588) over the blocks, for any byte alignment of
 *     starts and lengths.
 *   - All entry points are reentrant; tables are built once per device
 *     (thread-safe), and launches keep no mutable global state, so many host
 *     threads may call concurrently on their own streams
 *     (the reference's contract, SURVEY.md 8(b) "Threading").
 */
#ifndef NOVA_CRC32C_H_
#define NOVA_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- flags ------------------------------------------------------------- */
/* Extend each block's CRC by one trailing type byte, NOVA_CRC32C_TYPE(t):
 * table/table_builder.cc:202-203 `crc = Extend(Value(block, n), &type, 1)`. */
#define NOVA_CRC32C_APPEND_TYPE 0x1u
/* Store Mask(crc) (util/crc32c.h:28-31) instead of the raw CRC. */
#define NOVA_CRC32C_MASK_OUTPUT 0x2u
/* Trailer writer only: TableBuilder ordering -- trailer[4] = '!' AFTER the
 * masked CRC was encoded (table/table_builder.cc:204-206).  Without this flag
 * the StoCWritableFileClient ordering is used ('!' first, then the encode
 * overwrites it: ltc/stoc_file_client_impl.cpp:717-719). */
#define NOVA_TRAILER_TB_QUIRK 0x4u
/* Output the linear ("raw") CRC: zero initial register and no final
 * complement, i.e. Extend(c, D) == ~(M_|D|(~c) ^ raw(D)).  Used to combine
 * partial CRCs (nova_crc32c_combine).  Ignores init_or_null. */
#define NOVA_CRC32C_RAW 0x8u
/* Scheduling hint for variable-length batches (results are identical either
 * way): most blocks are >= 16 KiB (e.g. a LevelDB block_size of 16-64 KiB).
 * Long blocks are then cut into 32 KiB segments whose CRCs are combined
 * (crc32c_units_kernel); without it blocks are checksummed whole in lockstep
 * rounds of similar-length blocks (crc32c_rounds_kernel), the faster choice
 * for NovaLSM's ~4 KiB data blocks.  Accepted by nova_crc32c_batch and
 * nova_sstable_write_trailers.  A hinted batch of at most 1024 blocks (and a
 * fixed-stride batch of at most 8192 blocks over 64 KiB) is cut into pieces
 * spread over the whole device and recombined (split-and-combine path): a few
 * large blocks would otherwise run on a few waves.  Unhinted variable batches
 * holding multi-MiB blocks should pass the hint. */
#define NOVA_CRC32C_HINT_LARGE_BLOCKS 0x10u
#define NOVA_CRC32C_TYPE(t) (((uint32_t)(uint8_t)(t)) << 8)

/* ---- error codes (negative; positive values are hipError_t) ------------ */
#define NOVA_E_INVAL (-1)    /* bad argument */
#define NOVA_E_NODEV (-2)    /* no usable gfx950 device / HIP runtime */
#define NOVA_E_NOMEM (-3)    /* device or pinned allocation failed */

/* ---- scalar API: util/crc32c.h:17-40 ------------------------------------
 * Single-block calls stay on the host: one 4 KiB block costs ~1.4 us on a
 * CPU core versus ~5+ us to launch a kernel.  The GPU is
 * reached through the batch entry points below. */
/* replaces leveldb::crc32c::Extend, util/crc32c.h:17 / util/crc32c.cc:487 */
uint32_t nova_crc32c_extend(uint32_t init_crc, const char* data, size_t n);
/* replaces leveldb::crc32c::Value, util/crc32c.h:20-22 */
uint32_t nova_crc32c_value(const char* data, size_t n);
/* replaces leveldb::crc32c::Mask, util/crc32c.h:28-31 */
uint32_t nova_crc32c_mask(uint32_t crc);
/* replaces leveldb::crc32c::Unmask, util/crc32c.h:34-37 */
uint32_t nova_crc32c_unmask(uint32_t masked_crc);
/* crc32_combine: CRC of A||B from crc(A), crc(B), |B| (host, O(log |B|)).
 * The GF(2) shift the reference's stride tables encode (util/crc32c.cc:107-453). */
uint32_t nova_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* ---- plug-in hook: port::AcceleratedCRC32C, port/port_stdcxx.h:179-189 ---
 * Same contract: returns Extend(crc, buf, size).  Passes the reference's
 * self-test ("TestCRCBuffer" -> 0xdcbc59fa, util/crc32c.cc:477-485), after
 * which the reference sends EVERY Extend() here (util/crc32c.cc:487-491), so
 * the hook never returns a wrong CRC:
 *   - buffers below NOVA_HOOK_MIN_BYTES (env, default 8 MiB) run on the host
 *     (the library's SSE4.2 Extend, three interleaved crc32 chains: ~30-35
 *     GiB/s on one EPYC core; the measured crossover with the device path,
 *     copy included, lies between 4 and 16 MiB: tools/hook_crossover.py);
 *   - larger ones are copied to the GPU (one pooled stream and staging buffer
 *     per calling thread), checksummed by the HIP kernels and folded on the
 *     host; ANY device failure (no device, allocation beyond
 *     NOVA_HOOK_MAX_STAGING, a HIP error) falls back to the host Extend.
 * `buf` is HOST memory.  nova_port_stats counts the three outcomes.
 * Per-thread device footprint: a thread keeps its staging (the call's size
 * plus 1 B per KiB) between calls only while it is at most
 * NOVA_HOOK_KEEP_STAGING (env, default 64 MiB); a larger call frees it when it
 * returns.  nova_host_staging_release() frees the calling thread's staging. */
uint32_t nova_port_accelerated_crc32c(uint32_t crc, const char* buf, size_t size);
void nova_port_stats(uint64_t* host_calls, uint64_t* device_calls, uint64_t* fallback_calls);

/* ---- device batches ------------------------------------------------------
 * Variable-length: block i is base[offsets[i] .. offsets[i]+lengths[i]).
 * init_or_null[i] is block i's Extend() init (NULL: all 0, i.e. Value()).
 * Replaces a caller loop of crc32c::Value/Extend over the blocks of one
 * SSTable: table/table_builder.cc:202, ltc/stoc_file_client_impl.cpp:713-716,
 * table/table.cc:436. */
int nova_crc32c_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                      const uint32_t* init_or_null, uint32_t* out_crc, size_t n_blocks,
                      uint32_t flags, void* stream);

/* Fixed-stride: block i is base[i*stride .. i*stride+len). */
int nova_crc32c_batch_strided(const void* base, uint64_t stride, uint32_t len,
                              size_t n_blocks, const uint32_t* init_or_null,
                              uint32_t* out_crc, uint32_t flags, void* stream);

/* ---- SSTable composites -----------------------
 * Trailer writer: for each block (offsets[i], sizes[i]) of an SSTable image in
 * device memory, write the 5-byte trailer at buf+offsets[i]+sizes[i]:
 * [type][LE32 Mask(Extend(Value(block), type))], type = (flags >> 8) & 0xff,
 * with NOVA_TRAILER_TB_QUIRK reproducing TableBuilder's trailer[4]='!'.
 * Replaces TableBuilder::WriteRawBlock's checksum part
 * (table/table_builder.cc:192-212) and StoCWritableFileClient::WriteRawBlock
 * (ltc/stoc_file_client_impl.cpp:704-723). */
int nova_sstable_write_trailers(void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                size_t n_blocks, uint32_t flags, void* stream);

/* Read-verify: block i occupies sizes[i]+5 bytes at buf+offsets[i]
 * (block, type byte, LE32 masked CRC).  ok_out[i] = 1 iff
 * Unmask(DecodeFixed32(data+n+1)) == Value(data, n+1); *n_bad_out (device
 * u32, must be zeroed by the caller, may be NULL) is incremented per mismatch.
 * Replaces Table::ReadBlock's verify_checksums branch (table/table.cc:434-440,
 * "block checksum mismatch"). */
int nova_sstable_verify_blocks(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                               size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out,
                               void* stream);
/* The same with flags: only NOVA_CRC32C_HINT_LARGE_BLOCKS is read (a table of
 * >= 16 KiB blocks: 32 KiB segments, or pieces over the whole device for at
 * most 1024 blocks); results are identical. */
int nova_sstable_verify_blocks_ex(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                  size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out,
                                  uint32_t flags, void* stream);

/* ---- per-SSTable calls from many threads: the persistent engine ----------
 * The same operations as nova_sstable_write_trailers / _verify_blocks (same
 * arguments, same results), host-synchronous: the call returns when the
 * trailers / ok flags / n_bad are in device memory.  NovaLSM's compaction and
 * reader threads each checksum one SSTable per call
 * (ltc/stoc_file_client_impl.cpp:274-289, :843-882, table/table.cc:425-441):
 * too little work for a launch of its own.  These calls run on a persistent
 * kernel (crc32c_engine.hip) that stays resident while
 * requests arrive -- one workgroup per CU, tables loaded once -- and exits
 * after NOVA_SST_ENGINE_IDLE_US (default 1000, at most 1 s) without one; the
 * next call starts it again.
 * Sharing the GPU: while resident the engine holds every CU's LDS.  Every
 * other launch of this library (plain batches, composites, log, parity,
 * host-streamed paths, the hook) makes it yield: it takes no new request,
 * finishes the ones it took and exits, and its next instance starts only
 * after those launches have finished; so a plain call waits at most for the
 * requests already taken.  Kernels of OTHER libraries are
 * not seen: call nova_sst_engine_yield(stream) after enqueuing them on
 * `stream` (or keep the engine off with nova_sst_engine_set_enabled(0)).
 * Other streams' work is never queued behind the resident kernel: it is
 * launched cooperatively, which HIP runs on a hardware queue of its own
 * (NOVA_SST_ENGINE_QUEUE).  A device-wide sync
 * (hipDeviceSynchronize) waits for the running instance, which exits after
 * at most one time slice (nova_sst_engine_set_slice_us, default 20 ms).
 * Work queued on `stream` before the call (the image, its descriptors)
 * completes first: the call synchronises `stream` when it is busy.  A table
 * of more than 2^20 blocks runs as the plain call on `stream`, and so does a
 * request the engine did not run: no device memory, an engine error, or
 * NOVA_SST_ENGINE_TIMEOUT_MS (default 10000; nova_sst_engine_set_timeout_ms)
 * without a result.  The plain call runs only once the engine can no longer
 * touch the request (it is taken back: never started, skipped, or the
 * instance stopped and ended); the engine then backs off (100 ms, doubling to
 * 12.8 s, reset by a success) and is tried again.  If it cannot be taken back
 * within max(timeout, 30 s) the call returns NOVA_E_NODEV WITHOUT the plain
 * call -- the outputs may still be written -- and the engine is not used
 * again by this process.  A verify counter is zeroed before the plain call
 * recomputes it.  NOVA_SST_ENGINE=0: the round-3 coalescing queue instead
 * (concurrent calls grouped into shared launches, NOVA_SST_QUEUE_SLOTS 1..4
 * batches in flight, nova_sst_queue_set_slots). */
int nova_sst_queue_write_trailers(void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                  size_t n_blocks, uint32_t flags, void* stream);
int nova_sst_queue_verify_blocks(const void* buf, const uint64_t* offsets, const uint32_t* sizes,
                                 size_t n_blocks, uint8_t* ok_out, uint32_t* n_bad_out,
                                 void* stream);
int nova_sst_queue_set_slots(int slots);
/* Coalescing queue (NOVA_SST_ENGINE=0): batches launched, requests served,
 * most tables in one batch (this device). */
int nova_sst_queue_stats(uint64_t* batches, uint64_t* requests, uint64_t* max_tables_per_batch);
/* Test hook for the coalescing queue (NOVA_SST_ENGINE=0 or
 * nova_sst_engine_set_enabled(0)): hold = 1 keeps every queued request from
 * leading a batch (callers queue up), 0 releases them (the front one leads and
 * takes the compatible ones behind it), -1 changes nothing; *queued (may be
 * NULL) gets the number of requests waiting in the queue. */
int nova_sst_queue_hold(int hold, uint64_t* queued);

/* The engine of this device: start it now (it also starts on the first
 * queued call), stop it (waits for requests in flight; the next call starts
 * it again), its counters (requests run, instances launched, requests that
 * fell back to the plain call, whether an instance is resident), and the idle
 * time before an instance exits (from the next instance; 0: 1000 us). */
int nova_sst_engine_start(void);
int nova_sst_engine_stop(void);
int nova_sst_engine_stats(uint64_t* requests, uint64_t* launches, uint64_t* fallbacks, int* running);
int nova_sst_engine_set_idle_us(uint32_t us);
/* Counters of this device's engine, out[0..n) (n <= NOVA_ENGINE_COUNTERS):
 * requests, instances launched, plain-call fallbacks, resident now; instance
 * exits after the idle time, for a yield, for a stop, giving up on a request;
 * requests timed out, engine errors, requests taken back, requests that could
 * not be taken back; relaunches that waited for a yielded launch, yield bumps;
 * disabled for good, backing off now; instance exits at the end of a time
 * slice (NOVA_SST_ENGINE_SLICE_US); the longest host time of a relaunch (us)
 * and the relaunches that took over 1 ms; the longest gap between two polls
 * of a dispatcher (us, a stalled or preempted instance); requests whose
 * waiter slept instead of spinning, and the most waiters that spin at once
 * (this process's CPUs, capped by its cgroup quota, minus 2;
 * NOVA_SST_ENGINE_SPINNERS); 1 if the request ring is in device memory
 * (written by the host through the PCIe BAR; NOVA_SST_ENGINE_RING=host keeps
 * it in pinned host memory); requests whose completion words the host wrote
 * after the instance that took them ended without finishing them (a "lost"
 * exit or a worker error; their ring slots would never free otherwise); the
 * waves per CU its instances launch with (NOVA_SST_ENGINE_WAVES, default 12;
 * 0 before the engine's first use); requests declined during a yield storm
 * (instances exiting for other launches of the library over 5000 times a
 * second: the plain call ran, not counted as fallbacks). */
#define NOVA_ENGINE_COUNTERS 26
int nova_sst_engine_counters(uint64_t* out, size_t n);
/* Time slice of an engine instance in us, from the next instance (0: back to
 * NOVA_SST_ENGINE_SLICE_US, default 20000; 0xFFFFFFFF: none).  An instance
 * takes no request after running this long, finishes the ones it took and
 * exits; the next one follows at once.  Bounds what a device-wide sync and
 * another library's kernels wait under steady traffic. */
int nova_sst_engine_set_slice_us(uint32_t us);
/* Host timeout for one engine request (0: NOVA_SST_ENGINE_TIMEOUT_MS). */
int nova_sst_engine_set_timeout_ms(uint32_t ms);
/* Make the resident engine yield to work the caller enqueued on `stream`
 * (its next instance waits for that work); for kernels of other libraries. */
int nova_sst_engine_yield(void* stream);
/* End a backoff now (the next request tries the engine). */
int nova_sst_engine_reset(void);
/* Test hook, calling thread only: wait `us` after submitting a request before
 * waiting for it (a waiter descheduled past a whole ring turn). */
void nova_sst_engine_set_wait_delay_us(uint32_t us);
/* Test hook: the engine's give-up time in us, from the next instance (0: the
 * default 20 s).  A dispatcher with a request unfinished this long after the
 * last arrival exits "lost" and its workers stop: a way to make an instance end
 * with a request it took unfinished (its submitter takes it back, DESIGN.md
 * 3.5g). */
int nova_sst_engine_set_give_up_us(uint32_t us);
/* Test hook: from the next instance, on != 0 makes the engine's workers run no
 * chunk (the dispatcher still takes requests), so with a short give-up time the
 * instance ends "lost" with every request it took unfinished, deterministically.
 * Not for production use. */
int nova_sst_engine_set_drop_chunks(uint32_t on);
/* The calling thread's last engine request, out[0..n) (n <= 8): host ns
 * waiting for the engine's lock, ns holding it (ring writes, a relaunch), ns
 * waiting for the completion words; sleeps during that wait, relaunches
 * it made; the request's seq and blocks per chunk; 1 if it ended spinning. */
int nova_sst_engine_last_call(uint64_t* out, size_t n);
/* Route the nova_sst_queue_* calls of this process: 1 the engine, 0 the
 * coalescing queue, -1 back to NOVA_SST_ENGINE (default: the engine). */
int nova_sst_engine_set_enabled(int on);
/* Engine tracing (from the next instance; resets the sums): per request, the
 * dispatcher's, first chunk's and last chunk's s_memrealtime stamps.
 * nova_sst_engine_trace_stats: requests traced and averages in us of
 * [submit -> completion seen (host clock), dispatched -> first chunk started,
 * first chunk started -> last chunk done, dispatched -> last chunk done (GPU
 * clock)], then the largest host span. */
int nova_sst_engine_set_trace(int on);
int nova_sst_engine_trace_stats(uint64_t* n, double* out5);
/* Where a traced request's GPU time goes: requests with every stamp, and the
 * average us after its dispatch at which chunk 0's wave saw its ticket, found
 * the slot, finished the blocks, drained the stores, counted the chunk; then
 * when the last chunk was done; then the same five for the last chunk's wave
 * (out11 = [slot0, last_done, seen0, body0, drain0, count0, seenL, slotL,
 * bodyL, drainL, countL]). */
int nova_sst_engine_trace_detail(uint64_t* n, double* out11);

/* ---- MANIFEST / write-ahead log records ----------
 * buf holds buf_len bytes of a log file image starting at a 32 KiB log-block
 * boundary (db/log_format.h:27, kBlockSize).  record_offsets[i] (relative to
 * buf) points at a physical record header [LE32 masked crc][LE16 length][type]
 * (db/log_format.h:27-30) followed by `length` payload bytes.
 * Bounds, as log::Reader::ReadPhysicalRecord checks them (db/log_reader.cc:
 * 196-247): a record whose header or payload runs past its 32 KiB block (or
 * past buf_len) is never read.  A header that does not fit (fewer than 7
 * bytes left) is the block's trailer, skipped silently (:198-203), or, in the
 * file's last partial block or at/past buf_len, the end of the file (:204-211);
 * only a PAYLOAD past a full block is a "bad record length" (:230-235).
 * Write: header crc = Mask(Extend(type_crc[type], payload, length)) --
 * db/log_writer.cc:99-114 (type_crc[t] = Value(&t, 1), :16-21), computed as
 * Value(header+6, 1+length).  Out-of-bounds records are skipped (nothing is
 * written for them).
 * Verify: status_out[i] is one of NOVA_LOG_*; *n_bad_out (device u32, zeroed
 * by the caller, may be NULL) counts the records the reader reports as
 * corruption (CHECKSUM_MISMATCH, BAD_LENGTH).
 * Performance only: the dispatch sizes its groups and sort windows from the
 * mean record span buf_len / n_records, so pass the log's length, not a larger
 * allocation (results are identical either way). */
#define NOVA_LOG_CHECKSUM_MISMATCH 0 /* :251-262 "checksum mismatch" */
#define NOVA_LOG_OK 1                /* Unmask(stored) == Value(header+6, 1+length) */
#define NOVA_LOG_BAD_LENGTH 2        /* :228-235 "bad record length": payload past a full block (not read) */
#define NOVA_LOG_ZERO_RECORD 3       /* :241-247 type 0, length 0: skipped, not reported */
#define NOVA_LOG_TRUNCATED 4         /* :204-211, :236-239 cut by the end of the file: EOF, not reported */
#define NOVA_LOG_BLOCK_TRAILER 5     /* :198-203 < 7 bytes left in a full block: a trailer, skipped, not reported */
int nova_log_write_crcs(void* buf, size_t buf_len, const uint64_t* record_offsets,
                        size_t n_records, void* stream);
int nova_log_verify_records(const void* buf, size_t buf_len, const uint64_t* record_offsets,
                            size_t n_records, uint8_t* status_out, uint32_t* n_bad_out,
                            void* stream);

/* ---- XOR parity block ------------------------------
 * out[i] = XOR over fragments f of base[frag_offsets[f] + i], i < parity_len
 * (device pointers).  Replaces the byte-at-a-time host loop of
 * StoCWritableFileClient::Format, ltc/stoc_file_client_impl.cpp:334-349,
 * including its reading of parity_len bytes from every fragment start. */
int nova_xor_parity(const void* base, const uint64_t* frag_offsets, size_t n_frags,
                    size_t parity_len, void* out, void* stream);

/* ---- host-resident streamed paths ---------------------------------------
 * Blocks live in HOST memory (pinned or pageable; the analogue of NovaLSM's
 * RDMA-registered backing_mem_, ltc/stoc_file_client_impl.cpp:43-45).  The
 * batch is cut into chunks that flow H2D -> kernel -> D2H over n_streams
 * pooled HIP streams (1..8); descriptors and outputs are HOST arrays.
 * Synchronous.  Pageable memory is registered (hipHostRegister) for the
 * duration of the call.
 *
 * BASELINE config 5, fixed stride: chunks of chunk_blocks blocks.  Its
 * copies run in order on one copy stream and its kernels on another, chunk
 * by chunk through events, with n_streams (at least 2) device buffers in
 * rotation (NOVA_STREAM_HOST_PIPE=0: the round-4 form, each of n_streams
 * streams copying, checksumming and copying back its own chunks). */
int nova_crc32c_stream_host(const void* host_base, uint64_t stride, uint32_t len,
                            size_t n_blocks, uint32_t* host_out, uint32_t flags,
                            size_t chunk_blocks, int n_streams);
/* Variable-length, any order: a chunk is a run of consecutive descriptors
 * whose blocks span <= chunk_bytes (0: 64 MiB; a larger block gets its own
 * chunk), and copies that span -- so descriptors in address order (an
 * SSTable's blocks) copy each byte once.  Same results as nova_crc32c_batch. */
int nova_crc32c_batch_host(const void* host_base, const uint64_t* offsets, const uint32_t* lengths,
                           const uint32_t* init_or_null, uint32_t* out_crc, size_t n_blocks,
                           uint32_t flags, size_t chunk_bytes, int n_streams);
/* Trailers into a host SSTable image (StoCWritableFileClient::Format over
 * backing_mem_, ltc/stoc_file_client_impl.cpp:183-377): the GPU computes
 * Mask(Extend(Value(block), type)), the host stores the 5 bytes.  Same bytes as
 * nova_sstable_write_trailers. */
int nova_sstable_write_trailers_host(void* host_buf, const uint64_t* offsets, const uint32_t* sizes,
                                     size_t n_blocks, uint32_t flags, size_t chunk_bytes,
                                     int n_streams);
/* Read-verify of a host SSTable image (the ReadAll slab,
 * ltc/stoc_file_client_impl.cpp:843-882): ok_out[i] and *n_bad_out are HOST
 * outputs with nova_sstable_verify_blocks' meaning. */
int nova_sstable_verify_blocks_host(const void* host_buf, const uint64_t* offsets,
                                    const uint32_t* sizes, size_t n_blocks, uint8_t* ok_out,
                                    uint32_t* n_bad_out, size_t chunk_bytes, int n_streams);
/* The three calls above keep the calling thread's device staging (n_streams x
 * the largest chunk) and pinned result buffer between calls; this frees them,
 * and the port hook's staging of the calling thread.
 * chunk_bytes 0 sizes chunks to the image (about two per stream, 4-64 MiB). */
void nova_host_staging_release(void);

/* ---- utilities ----------------------------------------------------------- */
/* Fill nbytes of device memory with the splitmix64 counter stream
 * (novalsm_amd/synth.py): synthetic blocks without host initialisation. */
int nova_fill_splitmix64(void* dev, size_t nbytes, uint64_t seed, uint64_t first_word,
                         void* stream);
/* Build + upload the tables for the current device (optional: done lazily). */
int nova_device_init(void);
/* A caller stream's claim-counter slot (16 KiB of device memory, created on the
 * stream's first batch launch) lives until the stream is released: call this
 * before hipStreamDestroy on a stream that ran batches.  It waits for the
 * stream's work.  nova_stream_slots() counts live slots (diagnostics). */
int nova_stream_release(void* stream);
size_t nova_stream_slots(void);
/* Lanes per block ("G") and segment bytes the dispatcher would pick for an
 * aligned fixed-stride batch; returns 1 for the streaming kernel, 0 for the
 * units kernel, 2 for the flat kernel, 3 for the rounds kernel, 4 for the
 * burst (one-SSTable latency) kernel, 5 for the split-and-combine path (a few
 * large blocks cut into pieces over the whole device).  nova_crc32c_describe writes a JSON object naming the kernel
 * and its launch parameters (for reports and profiles); variable: 0 fixed-stride,
 * 1 variable-length, 2 variable-length with NOVA_CRC32C_HINT_LARGE_BLOCKS. */
int nova_crc32c_plan(size_t n_blocks, uint64_t bytes_per_block, int* lanes_per_unit,
                     uint32_t* seg_bytes);
int nova_crc32c_describe(size_t n_blocks, uint64_t len, uint64_t stride, int variable, char* buf,
                         size_t buflen); /* variable 3: a batch of log records */
const char* nova_crc32c_kernel_name(int lanes_per_unit);
/* Overrides for tuning/tests: lanes per unit (0 = auto) and segment size
 * (0 = auto).  Per calling thread: other threads keep the automatic plan. */
void nova_crc32c_set_tuning(int lanes_per_unit, uint32_t seg_bytes);
const char* nova_error_string(int err);
/* ABI version: bump on any signature or result-meaning change (2: log entry
 * points take buf_len; 3: log verify status NOVA_LOG_BLOCK_TRAILER (5), not
 * counted in n_bad, and the nova_sst_engine_* entry points; 4: the engine
 * yields to other launches, takes failed requests back, and the counters,
 * timeout, yield, reset and wait-delay entry points). */
int nova_crc32c_abi_version(void);

/* ---- diagnostics: libnova_crc32c_diag.so ONLY ---------------------------
 * The product library does not export anything below.  The diagnostics
 * library is the product's objects linked with one more translation unit
 * (crc32c_diag.hip: its own kernels and diagnostics instantiations of the
 * product templates, reached through a hook table; no preprocessor switch) and
 * adds timing ablations, alternative schedules and read-ceiling probes for
 * tools/ and the tuning tests.  All knobs are per calling thread.
 * variant: 0 production, 1 ablation (no table lookups -- WRONG CRCs, timing
 * only), 2 default-policy (cached) data loads instead of nt. */
void nova_diag_set_variant(int variant);
/* variant 4: the streaming kernel writes {begin, end, XCC id} per wave
 * (s_memrealtime ticks, 100 MHz) to dev_stamps[3*wave ...]. */
void nova_diag_set_stamps(uint64_t* dev_stamps);
/* Streaming kernel: how many other workgroups' claim counters a wave probes
 * for work once its own are exhausted (default 8 = one per XCD; -1 default). */
void nova_diag_set_static_pct(int steal_probes);
/* Streaming kernel: consecutive blocks per lane group per round (default 1). */
void nova_diag_set_blocks_per_group(int bpg);
/* Read-ceiling probe: variant = loads in flight per lane (2,4,8,16)
 * | 0x100 nt policy | 0x200 1024-thread workgroups (else 256).  out_dev holds
 * one u32 per launched thread. */
int nova_diag_read_ceiling(const void* base, size_t bytes, uint32_t* out_dev, int wgs,
                           int variant, void* stream);
/* Waves per workgroup for the batch kernels (1..16, flat kernel <= 12; 0 =
 * per-kernel default). */
void nova_diag_set_stream_waves(int waves);
/* Kernel for variable-length / unaligned batches: 0 auto, 1 units, 2 flat
 * (per-group block streams), 3 rounds (sorted batch, lockstep rounds).
 * Process-wide. */
void nova_diag_set_variable_kernel(int kernel);
/* Rounds kernel: take the batch in order (0), sort it by block step count
 * first (1, a pre-pass), or sort each claimed chunk of 64 blocks (2, default). */
void nova_diag_set_rounds_sort(int on);
/* Store form of large trailer-writer and log-write batches:
 * 0 = the product's (trailer bytes / CRC fields stored by the CRC kernel),
 * 2 = trailers in two passes (CRC array + scatter), 3 = whole 64-B pieces
 * where the layout allows, 4 = the same non-temporal; timing ablations that
 * write NO results: 5 = whole-piece form, 6 = product form (any mode). */
void nova_diag_set_trailer_single_pass(int on);
/* Burst (one-SSTable) kernel: 0 automatic, 16 or 64 lanes per block forced for
 * any batch size of store / trailer / verify, -1 never. */
void nova_diag_set_burst_lanes(int lanes);
/* Split-and-combine path for few large blocks: 0 automatic, 1 forced for any
 * store / trailer / verify batch, -1 never. */
void nova_diag_set_split(int on);
/* XOR parity kernel variant: chunks per thread (bits 0-3), fragments loaded
 * together (bits 4-7), workgroups per CU (bits 8-15); 0 fields = default. */
void nova_diag_set_parity_variant(int variant);
/* Units kernel: blocks per claimed wave chunk (1..16, default 8; 0 = default). */
void nova_diag_set_chunk_blocks(int blocks);
/* Plain coalesced streaming read of `bytes` (multiple of 16) with `wgs`
 * 256-thread workgroups; out_dev receives wgs*256 words.  The chip's read
 * ceiling for the roofline discussion. */
int nova_diag_read_stream(const void* base, size_t bytes, uint32_t* out_dev, int wgs,
                          void* stream);
/* Occupy every CU (one workgroup with all 160 KiB of LDS each) for `us`
 * microseconds (<= 5 s): a foreign kernel holding the resident engine off the
 * device, for the engine's take-back tests. */
int nova_diag_hold_cus(uint32_t us, void* stream);
/* The engine's ticket-group arithmetic on the host (CPU test): out[0..8)
 * workgroups per group for a grid of `wgs`, out[8..16) a request's tickets
 * [cstart, cend) per group, out[16] the groups that complete it. */
int nova_diag_engine_groups(uint32_t wgs, uint64_t cstart, uint64_t cend, uint64_t* out);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* NOVA_CRC32C_H_ */
