// Host-resident paths of the engine:
//   * nova_crc32c_stream_host -- BASELINE config 5: blocks in host memory (the
//     analogue of NovaLSM's RDMA-registered SSTable buffer, backing_mem_ in
//     ltc/stoc_file_client_impl.cpp:43-45 over nova_buf registered in
//     rdma/nova_rdma_rc_broker.cpp:31-35) stream H2D -> CRC kernel -> D2H in
//     chunks over several HIP streams so copies overlap the kernels.
//   * nova_port_accelerated_crc32c -- the reference's plug-in hook
//     port::AcceleratedCRC32C (port/port_stdcxx.h:179-189) backed by the GPU:
//     the buffer is cut into 4 KiB sub-blocks whose linear ("raw") CRCs are
//     computed by the HIP kernels and folded on the host with the GF(2) shift.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../include/nova_crc32c.h"
#include "gf2_crc32c.hpp"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int ensure(size_t bytes) {
    if (bytes <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return NOVA_E_NOMEM;
    n = bytes;
    return 0;
  }
};

struct PinBuf {
  void* p = nullptr;
  size_t n = 0;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
  int ensure(size_t bytes) {
    if (bytes <= n) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return NOVA_E_NOMEM;
    n = bytes;
    return 0;
  }
};

bool is_pinned(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeDevice ||
         attr.type == hipMemoryTypeManaged;
}

}  // namespace

extern "C" {

int nova_crc32c_stream_host(const void* host_base, uint64_t stride, uint32_t len,
                            size_t n_blocks, uint32_t* host_out, uint32_t flags,
                            size_t chunk_blocks, int n_streams) {
  if (n_blocks == 0) return 0;
  if (!host_base || !host_out || stride < len) return NOVA_E_INVAL;
  if (chunk_blocks == 0) chunk_blocks = 4096;
  if (n_streams < 1) n_streams = 1;
  if (n_streams > 8) n_streams = 8;
  int err = nova_device_init();
  if (err) return err;

  const size_t span = (n_blocks - 1) * stride + len;
  bool registered = false;
  if (!is_pinned(host_base)) {
    if (hipHostRegister(const_cast<void*>(host_base), span, hipHostRegisterDefault) != hipSuccess)
      return NOVA_E_NOMEM;
    registered = true;
  }
  const size_t chunk_span = (chunk_blocks - 1) * stride + len;
  std::vector<hipStream_t> streams(n_streams, nullptr);
  std::vector<DevBuf> dbuf(n_streams), dout(n_streams);
  PinBuf pout;
  int rc = pout.ensure(n_blocks * 4);
  for (int s = 0; s < n_streams && !rc; s++) {
    if (hipStreamCreateWithFlags(&streams[s], hipStreamNonBlocking) != hipSuccess) rc = NOVA_E_NODEV;
    if (!rc) rc = dbuf[s].ensure(chunk_span);
    if (!rc) rc = dout[s].ensure(chunk_blocks * 4);
  }
  const uint8_t* hb = static_cast<const uint8_t*>(host_base);
  size_t k = 0;
  for (size_t b0 = 0; b0 < n_blocks && !rc; b0 += chunk_blocks, k++) {
    const size_t m = (n_blocks - b0 < chunk_blocks) ? n_blocks - b0 : chunk_blocks;
    const int s = (int)(k % n_streams);
    const size_t bytes = (m - 1) * stride + len;
    hipError_t e = hipMemcpyAsync(dbuf[s].p, hb + b0 * stride, bytes, hipMemcpyHostToDevice,
                                  streams[s]);
    if (e != hipSuccess) { rc = (int)e; break; }
    rc = nova_crc32c_batch_strided(dbuf[s].p, stride, len, m, nullptr,
                                   static_cast<uint32_t*>(dout[s].p), flags, streams[s]);
    if (rc) break;
    e = hipMemcpyAsync(static_cast<uint32_t*>(pout.p) + b0, dout[s].p, m * 4,
                       hipMemcpyDeviceToHost, streams[s]);
    if (e != hipSuccess) rc = (int)e;
  }
  for (int s = 0; s < n_streams; s++) {
    if (streams[s]) {
      hipError_t e = hipStreamSynchronize(streams[s]);
      if (!rc && e != hipSuccess) rc = (int)e;
      (void)hipStreamDestroy(streams[s]);
    }
  }
  if (!rc) std::memcpy(host_out, pout.p, n_blocks * 4);
  if (registered) (void)hipHostUnregister(const_cast<void*>(host_base));
  return rc;
}

uint32_t nova_port_accelerated_crc32c(uint32_t crc, const char* buf, size_t size) {
  // Contract of port::AcceleratedCRC32C: the extended CRC, or 0 = cannot accelerate.
  if (size == 0) return crc;
  if (!buf || nova_device_init() != 0) return 0;
  constexpr uint32_t kSub = 4096;
  const size_t nsub = (size + kSub - 1) / kSub;
  const size_t full = size / kSub;
  thread_local DevBuf dbuf, dout;
  if (dbuf.ensure(size) || dout.ensure(nsub * 4)) return 0;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 0;
  std::vector<uint32_t> raw(nsub);
  int rc = (int)hipMemcpyAsync(dbuf.p, buf, size, hipMemcpyHostToDevice, s);
  if (!rc && full)
    rc = nova_crc32c_batch_strided(dbuf.p, kSub, kSub, full, nullptr,
                                   static_cast<uint32_t*>(dout.p), NOVA_CRC32C_RAW, s);
  const uint32_t tail = (uint32_t)(size - full * kSub);
  if (!rc && tail)
    rc = nova_crc32c_batch_strided(static_cast<uint8_t*>(dbuf.p) + full * kSub, tail, tail, 1,
                                   nullptr, static_cast<uint32_t*>(dout.p) + full,
                                   NOVA_CRC32C_RAW, s);
  if (!rc) rc = (int)hipMemcpyAsync(raw.data(), dout.p, nsub * 4, hipMemcpyDeviceToHost, s);
  if (!rc) rc = (int)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  if (rc) return 0;
  // raw(D) = fold of sub-block raws; Extend(crc, D) = ~(M_size(~crc) ^ raw(D)).
  using namespace nova::gf2;
  const Lin m_sub = shift_bytes(kSub);
  uint32_t acc = 0;
  for (size_t i = 0; i < full; i++) acc = m_sub(acc) ^ raw[i];
  if (tail) acc = shift_bytes(tail)(acc) ^ raw[full];
  return ~(shift_bytes(size)(~crc) ^ acc);
}

}  // extern "C"
