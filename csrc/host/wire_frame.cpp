// See wire_frame.h.
#include "wire_frame.h"

#include <string.h>

#if defined(__x86_64__)
#include <nmmintrin.h>
#define P2FA_HAVE_SSE42_TARGET 1
#endif

namespace {

constexpr uint8_t kMagic[4] = {'P', '2', 'F', 'A'};
constexpr uint64_t kAlign = 64;
constexpr uint64_t kPrefixV1 = 12;  // magic, version, header_len
constexpr uint64_t kPrefixV2 = 24;  // + crc32c, payload_len

uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

struct Table {
  uint32_t t[256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[i] = c;
    }
  }
};
const Table& table() {
  static const Table tb;  // thread-safe one-time init
  return tb;
}

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t crc) {
  const uint32_t* t = table().t;
  for (size_t i = 0; i < n; ++i) crc = t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}

#ifdef P2FA_HAVE_SSE42_TARGET
__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = uint32_t(c);
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}
bool have_sse42() { return __builtin_cpu_supports("sse4.2"); }
#endif

uint64_t align_up(uint64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

}  // namespace

extern "C" {

uint32_t p2fa_crc32c(const uint8_t* data, size_t len, uint32_t crc) {
  crc = ~crc;
#ifdef P2FA_HAVE_SSE42_TARGET
  if (have_sse42()) return ~crc_hw(data, len, crc);
#endif
  return ~crc_sw(data, len, crc);
}

uint64_t p2fa_payload_offset(uint64_t header_len) { return align_up(kPrefixV2 + header_len); }

void p2fa_write_prefix(uint8_t* dst, uint32_t header_len, uint32_t crc, uint64_t payload_len) {
  const uint32_t version = 2;
  memcpy(dst, kMagic, 4);
  memcpy(dst + 4, &version, 4);
  memcpy(dst + 8, &header_len, 4);
  memcpy(dst + 12, &crc, 4);
  memcpy(dst + 16, &payload_len, 8);
}

int p2fa_validate(const uint8_t* buf, size_t len, p2fa_frame* out) {
  if (buf == nullptr || out == nullptr || len < kPrefixV1) return P2FA_TOO_SHORT;
  if (memcmp(buf, kMagic, 4) != 0) return P2FA_BAD_MAGIC;
  const uint32_t version = rd32(buf + 4);
  const uint64_t hlen = rd32(buf + 8);
  const uint64_t n = len;
  // v1 frames (no payload checksum) are refused: nothing emits them any more,
  // and accepting them would let a corrupted version field skip the CRC check
  if (version != 2) return P2FA_BAD_VERSION;
  if (n < kPrefixV2) return P2FA_TOO_SHORT;
  if (hlen > n - kPrefixV2) return P2FA_BAD_HEADER_LEN;
  const uint64_t start = align_up(kPrefixV2 + hlen);  // hlen < 2^32: no wrap
  const uint64_t plen = rd64(buf + 16);
  if (start > n || plen != n - start) return P2FA_BAD_PAYLOAD_LEN;
  const uint32_t crc = rd32(buf + 12);
  if (p2fa_crc32c(buf + start, size_t(plen), 0) != crc) return P2FA_BAD_CHECKSUM;
  out->version = 2;
  out->header_off = kPrefixV2;
  out->header_len = hlen;
  out->payload_off = start;
  out->payload_len = plen;
  out->crc = crc;
  return P2FA_OK;
}

}  // extern "C"
