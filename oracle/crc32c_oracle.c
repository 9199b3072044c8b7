/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the batched CRC32C path.
 *
 * This file is the checker, never the product: only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load the library built from
 * it (oracle/liboracle_crc32c.so).  The product path (novalsm_amd/, the HIP
 * kernels behind include/nova_crc32c.h) never links or calls it.
 *
 * It is a from-scratch plain-C restatement of NovaLSM's portable CRC-32C
 * (util/crc32c.cc) -- no reference source is copied.  The five 256-entry tables
 * the reference ships as literals (util/crc32c.cc:20-453) are *generated* here
 * from the Castagnoli polynomial:
 *   - byte table      == kByteExtensionTable      (util/crc32c.cc:20-105)
 *   - stride tables   == kStrideExtensionTable0..3 (util/crc32c.cc:107-453):
 *     byte b placed at byte position k of the register, advanced through 16
 *     zero bytes (the 16-byte crc32_combine shift operator).
 * The loop structure follows util/crc32c.cc:487-588 step by step (see the
 * comments on oracle_extend), so its per-core speed is a like-for-like CPU
 * baseline ("port" kind in bench.py).
 *
 * Pinned by: util/crc32c_test.cc:14-61 known answers, the self-test constant
 * util/crc32c.cc:479-481, and golden vectors produced by the reference
 * util/crc32c.cc compiled unmodified into oracle/_ref/ (oracle/gen_golden.py,
 * tests/golden/crc32c_golden.json).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#define POLY 0x82F63B78u  /* reflected Castagnoli polynomial 0x1EDC6F41 */

static uint32_t byte_tab[256];      /* == kByteExtensionTable */
static uint32_t stride_tab[4][256]; /* stride_tab[k] == kStrideExtensionTable(3-k) */
static int tabs_ready = 0;
static pthread_once_t tabs_once = PTHREAD_ONCE_INIT;

/* one zero byte through the register (the STEP1 recurrence with data 0) */
static uint32_t zero_byte(uint32_t l) { return byte_tab[l & 0xff] ^ (l >> 8); }

static void build_tables(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (POLY & (0u - (c & 1u)));
    byte_tab[i] = c;
  }
  /* util/crc32c.cc:505-511 STEP4(s): crc_s = LE32(p+4s) ^ T3[crc_s&0xff] ^
   * T2[(crc_s>>8)&0xff] ^ T1[(crc_s>>16)&0xff] ^ T0[crc_s>>24]; the stride
   * table for byte position k is "byte at position k, then 16 zero bytes". */
  for (int k = 0; k < 4; k++) {
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t l = b << (8 * k);
      for (int z = 0; z < 16; z++) l = zero_byte(l);
      stride_tab[k][b] = l;
    }
  }
  tabs_ready = 1;
}

static void ensure_tables(void) {
  if (!tabs_ready) pthread_once(&tabs_once, build_tables);
}

static inline uint32_t read_le32(const uint8_t *p) {
  /* util/crc32c.cc:459-461 -> util/coding.h:122-130 DecodeFixed32 */
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

/* Restatement of leveldb::crc32c::Extend, util/crc32c.cc:487-588 (portable
 * branch; the accelerated branch is dead because HAVE_CRC32C=0,
 * include/port/port_config.h:23-26). */
uint32_t oracle_extend(uint32_t crc, const uint8_t *p, size_t n) {
  ensure_tables();
  const uint8_t *e = p + n;
  uint32_t l = crc ^ 0xffffffffu; /* :495, kCRC32Xor :456 */
#define O_STEP1()                              \
  do {                                         \
    uint32_t c_ = (l & 0xff) ^ *p++;           \
    l = byte_tab[c_] ^ (l >> 8);               \
  } while (0)
#define O_STEP4(s)                                                          \
  do {                                                                      \
    c##s = read_le32(p + (s) * 4) ^ stride_tab[0][c##s & 0xff] ^            \
           stride_tab[1][(c##s >> 8) & 0xff] ^                              \
           stride_tab[2][(c##s >> 16) & 0xff] ^ stride_tab[3][c##s >> 24];  \
  } while (0)
#define O_STEP4W(w)                                               \
  do {                                                            \
    w ^= l;                                                       \
    for (int i_ = 0; i_ < 4; i_++) w = (w >> 8) ^ byte_tab[w & 0xff]; \
    l = w;                                                        \
  } while (0)

  /* :535-541 byte steps until p is 4-aligned (only if that is within range) */
  const uint8_t *x = (const uint8_t *)(((uintptr_t)p + 3) & ~(uintptr_t)3);
  if (x <= e) {
    while (p != x) O_STEP1();
  }
  if ((e - p) >= 16) {
    /* :543-549 load one 16-byte swath into four stride partials */
    uint32_t c0 = read_le32(p + 0) ^ l;
    uint32_t c1 = read_le32(p + 4);
    uint32_t c2 = read_le32(p + 8);
    uint32_t c3 = read_le32(p + 12);
    p += 16;
    /* :556-558 STEP16 loop */
    while ((e - p) >= 16) {
      O_STEP4(0);
      O_STEP4(1);
      O_STEP4(2);
      O_STEP4(3);
      p += 16;
    }
    /* :561-569 one word at a time, rotating the partials */
    while ((e - p) >= 4) {
      O_STEP4(0);
      uint32_t tmp = c0;
      c0 = c1;
      c1 = c2;
      c2 = c3;
      c3 = tmp;
      p += 4;
    }
    /* :572-576 fold the four partials */
    l = 0;
    O_STEP4W(c0);
    O_STEP4W(c1);
    O_STEP4W(c2);
    O_STEP4W(c3);
  }
  /* :580-582 byte tail */
  while (p != e) O_STEP1();
#undef O_STEP1
#undef O_STEP4
#undef O_STEP4W
  return l ^ 0xffffffffu;
}

/* util/crc32c.h:20-22 */
uint32_t oracle_value(const uint8_t *p, size_t n) { return oracle_extend(0, p, n); }
/* util/crc32c.h:24-40 */
uint32_t oracle_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t oracle_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* Flags shared with include/nova_crc32c.h (values must match). */
#define O_APPEND_TYPE 0x1u
#define O_MASK_OUTPUT 0x2u

static uint32_t finish(uint32_t crc, uint32_t flags) {
  if (flags & O_APPEND_TYPE) {
    uint8_t t = (uint8_t)((flags >> 8) & 0xff);
    crc = oracle_extend(crc, &t, 1); /* table/table_builder.cc:203 */
  }
  if (flags & O_MASK_OUTPUT) crc = oracle_mask(crc);
  return crc;
}

/* Reference-semantics batch: one Extend per block, exactly what a caller looping
 * over util/crc32c.cc would produce. */
void oracle_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                  const uint32_t *init_or_null, uint32_t *out, size_t n_blocks,
                  uint32_t flags) {
  for (size_t i = 0; i < n_blocks; i++) {
    uint32_t init = init_or_null ? init_or_null[i] : 0u;
    out[i] = finish(oracle_extend(init, base + offsets[i], lengths[i]), flags);
  }
}

void oracle_batch_strided(const uint8_t *base, uint64_t stride, uint32_t len,
                          size_t n_blocks, const uint32_t *init_or_null, uint32_t *out,
                          uint32_t flags) {
  for (size_t i = 0; i < n_blocks; i++) {
    uint32_t init = init_or_null ? init_or_null[i] : 0u;
    out[i] = finish(oracle_extend(init, base + i * stride, len), flags);
  }
}

/* table/table_builder.cc:192-212 TableBuilder::WriteRawBlock trailer:
 * [type][LE32 Mask(Extend(Value(block),type))], then trailer[4]='!' (the
 * override happens AFTER the encode, :205-206).
 * ltc/stoc_file_client_impl.cpp:704-723: '!' is set BEFORE the encode, so the
 * stored CRC is intact.  tb_quirk selects the TableBuilder ordering. */
void oracle_trailer(const uint8_t *block, size_t n, uint8_t type, int tb_quirk,
                    uint8_t out5[5]) {
  uint32_t crc = oracle_value(block, n);
  crc = oracle_extend(crc, &type, 1);
  uint32_t m = oracle_mask(crc);
  out5[0] = type;
  if (!tb_quirk) out5[4] = '!';
  out5[1] = (uint8_t)m;
  out5[2] = (uint8_t)(m >> 8);
  out5[3] = (uint8_t)(m >> 16);
  out5[4] = (uint8_t)(m >> 24);
  if (tb_quirk) out5[4] = '!';
}

/* table/table.cc:434-440 Table::ReadBlock verify: crc over n+1 bytes (block +
 * type) against Unmask(DecodeFixed32(data+n+1)). Returns 1 if it matches. */
int oracle_verify(const uint8_t *data, size_t n) {
  uint32_t want = oracle_unmask(read_le32(data + n + 1));
  return oracle_value(data, n + 1) == want;
}

/* db/log_writer.cc:99-114 EmitPhysicalRecord: header crc =
 * Mask(Extend(type_crc_[t], payload, length)), type_crc_[t] = Value(&t, 1)
 * (db/log_writer.cc:16-21).  Writes the 4 crc bytes of the header at rec. */
void oracle_log_write(uint8_t *rec) {
  uint32_t len = (uint32_t)rec[4] | ((uint32_t)rec[5] << 8);
  uint8_t t = rec[6];
  uint32_t crc = oracle_mask(oracle_extend(oracle_value(&t, 1), rec + 7, len));
  rec[0] = (uint8_t)crc;
  rec[1] = (uint8_t)(crc >> 8);
  rec[2] = (uint8_t)(crc >> 16);
  rec[3] = (uint8_t)(crc >> 24);
}

/* db/log_reader.cc:251-262: Unmask(DecodeFixed32(header)) == Value(header+6, 1+length). */
int oracle_log_verify(const uint8_t *rec) {
  uint32_t len = (uint32_t)rec[4] | ((uint32_t)rec[5] << 8);
  return oracle_unmask(read_le32(rec)) == oracle_value(rec + 6, 1 + len);
}

/* db/log_reader.cc:196-262 ReadPhysicalRecord's per-record checks, in order,
 * for the record whose header starts at buf+off in a log image of buf_len
 * bytes that begins on a 32 KiB log-block boundary (db/log_format.h:27,
 * kBlockSize).  The reader holds the rest of the current block in buffer_
 * (a short read, i.e. the file's last partial block, sets eof_):
 *   - fewer than 7 bytes left for the header (:198-220): at or past the end
 *     of the file, or in the last partial block (eof_), the read ends -> 4
 *     (EOF, not reported); in a full block they are its trailer, skipped
 *     silently -> 5;
 *   - payload past the block (:228-239): with eof_ the record was cut by the
 *     end of the file -> 4, reported as EOF, not as a corruption; otherwise
 *     "bad record length" -> 2;
 *   - a kZeroType record of length 0 is skipped unreported (:241-247) -> 3;
 *   - else the CRC is checked (:249-262): 1 ok, 0 "checksum mismatch".
 * (The NOVA_LOG_* codes of include/nova_crc32c.h.) */
int oracle_log_check(const uint8_t *buf, uint64_t buf_len, uint64_t off) {
  const uint64_t kBlock = 32768, kHeader = 7;
  uint64_t end = (off / kBlock + 1) * kBlock;
  if (end > buf_len) end = buf_len;
  const int eof = end == buf_len && buf_len % kBlock != 0;  /* the block is the short last read */
  const int cut = eof ? 4 : 2;                                /* eof_ : bad length */
  if (off >= buf_len) return 4;                               /* :204-211: no bytes left */
  if (off + kHeader > end) return eof ? 4 : 5;                /* :204-211 : :198-203 trailer */
  const uint8_t *h = buf + off;
  uint32_t len = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
  if (off + kHeader + len > end) return cut;
  if (h[6] == 0 && len == 0) return 3;
  return oracle_unmask(read_le32(h)) == oracle_value(h + 6, 1 + len) ? 1 : 0;
}

/* ltc/stoc_file_client_impl.cpp:340-348: parity[i] = XOR over fragments of
 * backing_mem_[fragment.offset() + i] for i < parity_block_size_ (every
 * fragment contributes parity_len bytes from its start). */
void oracle_xor_parity(const uint8_t *base, const uint64_t *frag_off, size_t n_frags,
                       size_t parity_len, uint8_t *out) {
  for (size_t i = 0; i < parity_len; i++) {
    uint8_t b = 0;
    for (size_t f = 0; f < n_frags; f++) b ^= base[frag_off[f] + i];
    out[i] = b;
  }
}

/* Multi-threaded strided batch for the CPU baseline ("port" kind): one
 * pthread per core on contiguous shards, as BASELINE.md's CPU plan says. */
struct shard_arg {
  const uint8_t *base;
  uint64_t stride;
  uint32_t len;
  size_t lo, hi;
  uint32_t *out;
  int reps;
};

static void *shard_main(void *p) {
  struct shard_arg *a = (struct shard_arg *)p;
  for (int r = 0; r < a->reps; r++)
    for (size_t i = a->lo; i < a->hi; i++)
      a->out[i] = oracle_value(a->base + i * a->stride, a->len);
  return 0;
}

int oracle_batch_strided_mt(const uint8_t *base, uint64_t stride, uint32_t len,
                            size_t n_blocks, uint32_t *out, int threads, int reps) {
  ensure_tables();
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  struct shard_arg args[512];
  size_t per = (n_blocks + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    size_t lo = t * per, hi = lo + per;
    if (lo > n_blocks) lo = n_blocks;
    if (hi > n_blocks) hi = n_blocks;
    args[t] = (struct shard_arg){base, stride, len, lo, hi, out, reps};
    if (pthread_create(&tid[t], 0, shard_main, &args[t]) != 0) break;
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], 0);
  return started;
}

/* Multi-threaded variable-length batch: the checker for full-size batches
 * (every block of BASELINE config 3), same semantics as oracle_batch. */
struct vshard_arg {
  const uint8_t *base;
  const uint64_t *offsets;
  const uint32_t *lengths, *init;
  uint32_t *out;
  size_t lo, hi;
  uint32_t flags;
};

static void *vshard_main(void *p) {
  struct vshard_arg *a = (struct vshard_arg *)p;
  for (size_t i = a->lo; i < a->hi; i++) {
    uint32_t init = a->init ? a->init[i] : 0u;
    a->out[i] = finish(oracle_extend(init, a->base + a->offsets[i], a->lengths[i]), a->flags);
  }
  return 0;
}

int oracle_batch_mt(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                    const uint32_t *init_or_null, uint32_t *out, size_t n_blocks, uint32_t flags,
                    int threads) {
  ensure_tables();
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  struct vshard_arg args[512];
  size_t per = (n_blocks + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    size_t lo = t * per, hi = lo + per;
    if (lo > n_blocks) lo = n_blocks;
    if (hi > n_blocks) hi = n_blocks;
    args[t] = (struct vshard_arg){base, offsets, lengths, init_or_null, out, lo, hi, flags};
    if (pthread_create(&tid[t], 0, vshard_main, &args[t]) != 0) break;
    started++;
  }
  /* a thread that failed to start leaves its shard to this thread */
  for (int t = started; t < threads; t++) vshard_main(&args[t]);
  for (int t = 0; t < started; t++) pthread_join(tid[t], 0);
  return started;
}

/* benchmarks/db_bench.cc:635-652 Crc32c(): Value() over the same 4 KiB of 'x'
 * until total_bytes (500 MiB there) are checksummed, on the calling thread. */
uint32_t oracle_dbbench_crc32c(int64_t total_bytes) {
  uint8_t data[4096];
  memset(data, 'x', sizeof(data));
  uint32_t crc = 0;
  for (int64_t bytes = 0; bytes < total_bytes; bytes += 4096) crc = oracle_value(data, 4096);
  return crc;
}

/* splitmix64 counter form: word k of the stream seeded with `seed` is
 * mix(seed + (k+1)*gamma) -- the same bytes the sequential generator emits.
 * Shared by tests, bench and the device generator in novalsm_amd. */
static inline uint64_t sm64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_fill_splitmix64(uint8_t *dst, size_t nbytes, uint64_t seed, uint64_t first_word) {
  size_t nw = nbytes / 8;
  for (size_t k = 0; k < nw; k++) {
    uint64_t v = sm64_mix(seed + (first_word + k + 1) * 0x9E3779B97F4A7C15ull);
    memcpy(dst + 8 * k, &v, 8);
  }
  size_t rem = nbytes - 8 * nw;
  if (rem) {
    uint64_t v = sm64_mix(seed + (first_word + nw + 1) * 0x9E3779B97F4A7C15ull);
    memcpy(dst + 8 * nw, &v, rem);
  }
}

/* Expose the generated tables so tests can pin them against the reference's
 * literal values (through oracle/_ref). */
void oracle_tables(uint32_t byte_out[256], uint32_t stride_out[4][256]) {
  ensure_tables();
  memcpy(byte_out, byte_tab, sizeof(byte_tab));
  memcpy(stride_out, stride_tab, sizeof(stride_tab));
}
