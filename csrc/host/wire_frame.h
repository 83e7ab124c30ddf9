// Native validator for the p2pfl_amd tensor wire frame (learning/wire.py).
//
// Frame v2 (little endian):
//   "P2FA" | u32 version | u32 header_len | u32 crc32c(payload) | u64 payload_len |
//   header (UTF-8 JSON, header_len bytes) | zero pad to a 64-byte boundary | payload
// v1 frames (no checksum, no payload length) are still accepted.
//
// Everything a peer sends is untrusted: every length is checked against the
// buffer before it is used (no arithmetic can wrap), and the payload checksum
// is verified before Python parses the JSON header or builds tensors.  Built
// as a plain C ABI library (no torch, no HIP) so the host sanitizer test
// (tests/native/fuzz_wire.cpp under ASan/UBSan) covers exactly this code.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum p2fa_status {
  P2FA_OK = 0,
  P2FA_TOO_SHORT = 1,
  P2FA_BAD_MAGIC = 2,
  P2FA_BAD_VERSION = 3,
  P2FA_BAD_HEADER_LEN = 4,
  P2FA_BAD_PAYLOAD_LEN = 5,
  P2FA_BAD_CHECKSUM = 6,
};

typedef struct {
  uint32_t version;
  uint64_t header_off, header_len;    // JSON header bytes
  uint64_t payload_off, payload_len;  // raw tensor bytes
  uint32_t crc;                       // stored checksum (v2)
} p2fa_frame;

// CRC32C (Castagnoli), hardware-accelerated with SSE4.2 when available.
uint32_t p2fa_crc32c(const uint8_t* data, size_t len, uint32_t crc);
// Validates framing and (v2) the payload checksum; fills *out on success.
int p2fa_validate(const uint8_t* buf, size_t len, p2fa_frame* out);
// Writes the 24-byte v2 prefix (magic .. payload_len) for a frame.
void p2fa_write_prefix(uint8_t* dst, uint32_t header_len, uint32_t crc, uint64_t payload_len);
// Byte offset of the payload for a header of header_len bytes (v2).
uint64_t p2fa_payload_offset(uint64_t header_len);

#ifdef __cplusplus
}
#endif
