// nova_crc32c.hpp -- C++ host API of the MI355X CRC32C engine.
//
// (1) leveldb::crc32c -- the exact signatures and semantics of NovaLSM's
//     util/crc32c.h:11-43, so the library is a link-time drop-in for
//     util/crc32c.cc (drop that file from the build, link libnova_crc32c.so).
// (2) nova::crc32c -- thin C++ wrappers over the C-ABI batch entry points
//     (include/nova_crc32c.h) for callers that batch per SSTable.
#ifndef NOVA_CRC32C_HPP_
#define NOVA_CRC32C_HPP_

#include <cstddef>
#include <cstdint>

#include "nova_crc32c.h"

namespace leveldb {
namespace crc32c {

// Return the crc32c of concat(A, data[0,n-1]) where init_crc is the crc32c of
// some string A (util/crc32c.h:14-17).  Defined in libnova_crc32c.so.
uint32_t Extend(uint32_t init_crc, const char* data, size_t n);

// util/crc32c.h:20-22
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;  // util/crc32c.h:24

// util/crc32c.h:28-31
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

// util/crc32c.h:34-37
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace leveldb

namespace nova {
namespace crc32c {

// Device batch over variable-length blocks (see nova_crc32c_batch).
inline int Batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                 const uint32_t* init_or_null, uint32_t* out, size_t n, uint32_t flags = 0,
                 void* stream = nullptr) {
  return nova_crc32c_batch(base, offsets, lengths, init_or_null, out, n, flags, stream);
}

// Device batch over fixed-stride blocks (see nova_crc32c_batch_strided).
inline int BatchStrided(const void* base, uint64_t stride, uint32_t len, size_t n, uint32_t* out,
                        const uint32_t* init_or_null = nullptr, uint32_t flags = 0,
                        void* stream = nullptr) {
  return nova_crc32c_batch_strided(base, stride, len, n, init_or_null, out, flags, stream);
}

// SSTable trailer writer / read-verify.
// large_blocks: the table's block_size is >= 16 KiB (scheduling hint only,
// NOVA_CRC32C_HINT_LARGE_BLOCKS; the trailers are identical either way).
inline int WriteTrailers(void* buf, const uint64_t* offsets, const uint32_t* sizes, size_t n,
                         uint8_t type, bool table_builder_quirk, void* stream = nullptr,
                         bool large_blocks = false) {
  return nova_sstable_write_trailers(buf, offsets, sizes, n,
                                     NOVA_CRC32C_TYPE(type) |
                                         (table_builder_quirk ? NOVA_TRAILER_TB_QUIRK : 0u) |
                                         (large_blocks ? NOVA_CRC32C_HINT_LARGE_BLOCKS : 0u),
                                     stream);
}
inline int VerifyBlocks(const void* buf, const uint64_t* offsets, const uint32_t* sizes, size_t n,
                        uint8_t* ok, uint32_t* n_bad, void* stream = nullptr) {
  return nova_sstable_verify_blocks(buf, offsets, sizes, n, ok, n_bad, stream);
}

// The same on an SSTable image in HOST memory (backing_mem_ / the ReadAll
// slab): chunks are copied H2D over pooled streams, results come back; the
// trailer bytes are stored by the host.  Synchronous.
inline int WriteTrailersHost(void* host_buf, const uint64_t* offsets, const uint32_t* sizes,
                             size_t n, uint8_t type, bool table_builder_quirk) {
  return nova_sstable_write_trailers_host(
      host_buf, offsets, sizes, n,
      NOVA_CRC32C_TYPE(type) | (table_builder_quirk ? NOVA_TRAILER_TB_QUIRK : 0u), 0, 3);
}
inline int VerifyBlocksHost(const void* host_buf, const uint64_t* offsets, const uint32_t* sizes,
                            size_t n, uint8_t* ok, uint32_t* n_bad) {
  return nova_sstable_verify_blocks_host(host_buf, offsets, sizes, n, ok, n_bad, 0, 3);
}

// Log / MANIFEST physical records of a log image.
// status[i] is one of NOVA_LOG_* (db/log_reader.cc:196-262).
inline int LogWriteCrcs(void* log, size_t log_len, const uint64_t* record_offsets, size_t n,
                        void* stream = nullptr) {
  return nova_log_write_crcs(log, log_len, record_offsets, n, stream);
}
inline int LogVerifyRecords(const void* log, size_t log_len, const uint64_t* record_offsets,
                            size_t n, uint8_t* status, uint32_t* n_bad, void* stream = nullptr) {
  return nova_log_verify_records(log, log_len, record_offsets, n, status, n_bad, stream);
}

inline uint32_t Combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return nova_crc32c_combine(crc_a, crc_b, len_b);
}

}  // namespace crc32c
}  // namespace nova

#endif  // NOVA_CRC32C_HPP_
