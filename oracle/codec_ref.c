/*
 * ORACLE (test infrastructure, never the product): plain-C restatement of the
 * batch codec, for bit-exact diffs at full BASELINE sizes where the numpy
 * restatement is slow.  Framing follows utils/packet.py:3-10 (seq u16 BE,
 * ack u16 BE, syn/ack/fin/offset byte, payload; :60-65, :80-81); the rudp7
 * layout puts the build-defined RFC 1071 checksum at bytes 5-6.  The checksum
 * is computed from its definition: big-endian 16-bit words over the frame
 * with the checksum field zero and an odd tail zero-padded.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static uint16_t fold_complement(uint64_t s) {
  while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
  return (uint16_t)(~s & 0xFFFFu);
}

/* RFC 1071 checksum of an arbitrary byte string. */
uint16_t oracle_inet_checksum(const uint8_t* data, size_t len) {
  uint64_t s = 0;
  size_t i = 0;
  for (; i + 1 < len; i += 2) s += ((uint64_t)data[i] << 8) | data[i + 1];
  if (i < len) s += (uint64_t)data[i] << 8;
  return fold_complement(s);
}

/* Checksum of one frame with the rudp7 checksum field counted as zero. */
static uint16_t frame_checksum(const uint8_t* f, size_t len, int layout) {
  uint64_t s = 0;
  for (size_t i = 0; i < len; ++i) {
    if (layout == 7 && (i == 5 || i == 6)) continue;
    s += (i & 1) ? (uint64_t)f[i] : ((uint64_t)f[i] << 8);
  }
  return fold_complement(s);
}

void oracle_encode(const uint16_t* seq, const uint16_t* ack, const uint8_t* flags,
                   const uint8_t* payload, uint64_t n, uint32_t L, int layout, uint8_t* frames,
                   uint16_t* csum) {
  const uint64_t F = (uint64_t)L + (uint64_t)layout;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    uint8_t* f = frames + (uint64_t)i * F;
    f[0] = (uint8_t)(seq[i] >> 8);
    f[1] = (uint8_t)seq[i];
    f[2] = (uint8_t)(ack[i] >> 8);
    f[3] = (uint8_t)ack[i];
    f[4] = flags[i];
    if (layout == 7) f[5] = f[6] = 0;
    memcpy(f + layout, payload + (uint64_t)i * L, L);
    const uint16_t c = frame_checksum(f, F, layout);
    if (layout == 7) {
      f[5] = (uint8_t)(c >> 8);
      f[6] = (uint8_t)c;
    }
    if (csum) csum[i] = c;
  }
}

/* ok: 1 good, 0 bad checksum, 2 short, 3 unverified (rudp5 without csum_in). */
void oracle_decode(const uint8_t* frames, uint64_t n, uint32_t F, int layout,
                   const uint16_t* csum_in, uint16_t* seq, uint16_t* ack, uint8_t* flags,
                   uint8_t* ok, uint16_t* csum) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const uint8_t* f = frames + (uint64_t)i * F;
    uint8_t b[7] = {0, 0, 0, 0, 0, 0, 0};
    for (uint32_t k = 0; k < 7 && k < F; ++k) b[k] = f[k];
    if (F < (uint32_t)layout) {
      seq[i] = F >= 2 ? (uint16_t)(b[0] << 8 | b[1]) : b[0];
      ack[i] = F >= 4 ? (uint16_t)(b[2] << 8 | b[3]) : b[2];
      flags[i] = b[4];
      ok[i] = 2;
      csum[i] = 0;
      continue;
    }
    seq[i] = (uint16_t)(b[0] << 8 | b[1]);
    ack[i] = (uint16_t)(b[2] << 8 | b[3]);
    flags[i] = b[4];
    const uint16_t c = frame_checksum(f, F, layout);
    csum[i] = c;
    if (layout == 7)
      ok[i] = c == (uint16_t)(b[5] << 8 | b[6]);
    else
      ok[i] = csum_in ? (c == csum_in[i]) : 3;
  }
}
