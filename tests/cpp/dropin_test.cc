// C++ drop-in check: compiled against include/nova_crc32c.hpp and linked with
// libnova_crc32c.so exactly as NovaLSM would link it.
// Mirrors the cases of util/crc32c_test.cc:14-61 (RFC 3720 B.4 vectors,
// Values, Extend chaining, Mask round trips) with the reference's names.
#include <cstdio>
#include <cstring>
#include <string>

#include "nova_crc32c.hpp"

using namespace leveldb;

static int failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                      \
    }                                                                  \
  } while (0)

int main() {
  char buf[32];
  std::memset(buf, 0, sizeof(buf));
  EXPECT(0x8a9136aau == crc32c::Value(buf, sizeof(buf)));
  std::memset(buf, 0xff, sizeof(buf));
  EXPECT(0x62a8ab43u == crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(i);
  EXPECT(0x46dd794eu == crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(31 - i);
  EXPECT(0x113fdb5cu == crc32c::Value(buf, sizeof(buf)));
  const unsigned char pdu[48] = {
      0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x14, 0, 0, 0, 0, 0, 0x04, 0,
      0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0};
  EXPECT(0xd9963a56u == crc32c::Value(reinterpret_cast<const char*>(pdu), sizeof(pdu)));
  EXPECT(crc32c::Value("a", 1) != crc32c::Value("foo", 3));
  EXPECT(crc32c::Value("hello world", 11) == crc32c::Extend(crc32c::Value("hello ", 6), "world", 5));
  const uint32_t crc = crc32c::Value("foo", 3);
  EXPECT(crc != crc32c::Mask(crc));
  EXPECT(crc != crc32c::Mask(crc32c::Mask(crc)));
  EXPECT(crc == crc32c::Unmask(crc32c::Mask(crc)));
  EXPECT(crc == crc32c::Unmask(crc32c::Unmask(crc32c::Mask(crc32c::Mask(crc)))));
  EXPECT(0xdcbc59fau == crc32c::Value("TestCRCBuffer", 13));  // util/crc32c.cc:479-481
  // table/table_builder.cc:202-206 trailer composition on 4096 x 'x'
  std::string blk(4096, 'x');
  char type = 0;
  uint32_t c = crc32c::Extend(crc32c::Value(blk.data(), blk.size()), &type, 1);
  EXPECT(crc32c::Mask(c) == 0x27d32401u);
  // crc32_combine
  std::string a = "abcdefghij", b = "0123456789012345678901";
  EXPECT(nova::crc32c::Combine(crc32c::Value(a.data(), a.size()), crc32c::Value(b.data(), b.size()),
                               b.size()) == crc32c::Value((a + b).data(), a.size() + b.size()));
  if (failures == 0) std::printf("==== PASSED dropin_test\n");
  return failures ? 1 : 0;
}
