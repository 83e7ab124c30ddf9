// Host fuzz driver for the wire-frame validator (csrc/host/wire_frame.cpp),
// built and run under AddressSanitizer + UndefinedBehaviorSanitizer by
// tests/test_native_sanitizers.py.  Any out-of-bounds read, overflow or UB
// aborts the process; the invariants below are checked on every result.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../csrc/host/wire_frame.h"

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                    \
    }                                                             \
  } while (0)

static std::vector<uint8_t> make_frame(std::mt19937_64& rng, size_t hlen, size_t plen) {
  std::vector<uint8_t> payload(plen), header(hlen);
  for (auto& b : payload) b = uint8_t(rng());
  for (auto& b : header) b = uint8_t('a' + rng() % 26);
  const uint64_t off = p2fa_payload_offset(hlen);
  // exact-size heap buffer: ASan catches any read past the end
  std::vector<uint8_t> f(off + plen, 0);
  p2fa_write_prefix(f.data(), uint32_t(hlen), p2fa_crc32c(payload.data(), plen, 0), plen);
  if (hlen) memcpy(f.data() + 24, header.data(), hlen);
  if (plen) memcpy(f.data() + off, payload.data(), plen);
  return f;
}

static int validate_exact(const std::vector<uint8_t>& f, size_t len, p2fa_frame* fr) {
  // copy into an allocation of exactly `len` bytes so over-reads are detected
  uint8_t* buf = static_cast<uint8_t*>(malloc(len ? len : 1));
  if (len) memcpy(buf, f.data(), len);
  const int rc = p2fa_validate(buf, len, fr);
  if (rc == P2FA_OK) {
    CHECK(fr->header_off + fr->header_len <= fr->payload_off);
    CHECK(fr->payload_off + fr->payload_len == len);
  }
  free(buf);
  return rc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937_64 rng(12345);
  // known-answer test: CRC32C("123456789") = 0xE3069283
  CHECK(p2fa_crc32c(reinterpret_cast<const uint8_t*>("123456789"), 9, 0) == 0xE3069283u);
  p2fa_frame fr;
  CHECK(p2fa_validate(nullptr, 0, &fr) == P2FA_TOO_SHORT);
  for (int it = 0; it < iters; ++it) {
    const size_t hlen = rng() % 300, plen = (it % 7 == 0) ? 0 : rng() % 5000;
    auto f = make_frame(rng, hlen, plen);
    CHECK(validate_exact(f, f.size(), &fr) == P2FA_OK);
    CHECK(fr.version == 2 && fr.payload_len == plen && fr.header_len == hlen);
    // every truncation is rejected (never read past the end)
    for (size_t cut = 0; cut < f.size(); cut += 1 + f.size() / 64) CHECK(validate_exact(f, cut, &fr) != P2FA_OK);
    // a flipped payload bit is always caught by the checksum
    if (plen) {
      auto g = f;
      g[fr.payload_off + rng() % plen] ^= uint8_t(1u << (rng() % 8));
      CHECK(validate_exact(g, g.size(), &fr) == P2FA_BAD_CHECKSUM);
    }
    // hostile length fields
    auto g = f;
    const uint32_t big32[] = {0xFFFFFFFFu, 0x7FFFFFFFu, uint32_t(f.size()), uint32_t(f.size() - 23)};
    memcpy(g.data() + 8, &big32[rng() % 4], 4);
    validate_exact(g, g.size(), &fr);
    g = f;
    const uint64_t big64[] = {~0ull, 1ull << 63, f.size(), uint64_t(plen) + 1};
    memcpy(g.data() + 16, &big64[rng() % 4], 8);
    CHECK(validate_exact(g, g.size(), &fr) != P2FA_OK || big64[0] == plen);
    // random prefix bytes and pure garbage
    g = f;
    for (int k = 0; k < 4; ++k) g[rng() % 24] = uint8_t(rng());
    validate_exact(g, g.size(), &fr);
    std::vector<uint8_t> junk(rng() % 200);
    for (auto& b : junk) b = uint8_t(rng());
    if (junk.size() >= 4 && rng() % 2) memcpy(junk.data(), "P2FA", 4);
    validate_exact(junk, junk.size(), &fr);
  }
  // v1 frames (no checksum) are refused
  std::vector<uint8_t> v1(64 + 8, 0);
  memcpy(v1.data(), "P2FA", 4);
  const uint32_t one = 1, h = 3;
  memcpy(v1.data() + 4, &one, 4);
  memcpy(v1.data() + 8, &h, 4);
  CHECK(validate_exact(v1, v1.size(), &fr) == P2FA_BAD_VERSION);
  printf("fuzz_wire: %d iterations, %d failures\n", iters, fails);
  return fails ? 1 : 0;
}
