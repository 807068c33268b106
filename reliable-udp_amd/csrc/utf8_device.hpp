// Strict UTF-8 checks shared by the validation kernels (varlen.hip) and the
// decode kernels that validate in the same pass (decode.hip, varlen.hip).
//
// Strict UTF-8 (RFC 3629, as CPython's bytes.decode() accepts it, i.e. what
// utils/packet.py:73 enforces on every get_payload(), called per datagram at
// utils/reliableUDP.py:121): no overlongs (C0, C1, E0 80-9F, F0 80-8F), no
// surrogates (ED A0-BF), nothing above U+10FFFF (F4 90+, F5-FF), no stray or
// missing continuation bytes.  Byte-parallel: every byte is judged from itself
// and the three bytes before it, so a payload splits over lanes with no
// carried state (the approach of SIMD UTF-8 validators): byte c at payload
// index i, with p1 p2 p3 the bytes at i-1, i-2, i-3 (0 before the payload start):
//   c is a continuation byte  <=>  p1 is a 2/3/4-byte lead, or p2 a 3/4-byte
//                                  lead, or p3 a 4-byte lead ("expected")
//   C0 C1 F5..FF never appear; after E0 / ED / F0 / F4 the next byte lies in
//   A0-BF / 80-9F / 90-BF / 80-8F; and nothing is still expected at the end.
// A payload with no byte >= 0x80 is valid outright: the decode kernels OR
// their payload words as they sum them and run the byte checks only on
// frames that hold a high bit.
#pragma once
#include "codec_device.hpp"

namespace RUDP_NS {

__device__ __forceinline__ uint32_t utf8_need(uint32_t b) {  // continuation bytes a lead asks for
  return b >= 0xF0 ? 3u : b >= 0xE0 ? 2u : b >= 0xC0 ? 1u : 0u;
}

__device__ __forceinline__ bool utf8_byte_ok(uint32_t c, uint32_t p1, uint32_t p2, uint32_t p3) {
  const bool cont = (c & 0xC0u) == 0x80u;
  const bool expected = utf8_need(p1) >= 1 || utf8_need(p2) >= 2 || utf8_need(p3) >= 3;
  // p1..p3 that are themselves continuation bytes ask for nothing (need() of 80-BF is 0)
  if (cont != expected) return false;
  if (c == 0xC0 || c == 0xC1 || c >= 0xF5) return false;
  if (p1 == 0xE0 && c < 0xA0) return false;
  if (p1 == 0xED && c > 0x9F) return false;
  if (p1 == 0xF0 && c < 0x90) return false;
  if (p1 == 0xF4 && c > 0x8F) return false;
  return true;
}

// Something is still expected after the last three bytes p1 p2 p3.
__device__ __forceinline__ bool utf8_pending(uint32_t p1, uint32_t p2, uint32_t p3) {
  return utf8_need(p1) >= 1 || utf8_need(p2) >= 2 || utf8_need(p3) >= 3;
}

__device__ __forceinline__ uint32_t byte_of(u32x4 v, int k) {
  const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
  return (w >> (8 * (k & 3))) & 0xFFu;
}

// Bytes [lo, hi) of 16-byte chunk w, others zero (lo, hi relative to the chunk, any range).
__device__ __forceinline__ u32x4 keep_bytes(u32x4 w, int lo, int hi) {
  return make_u32x4(lo64(w) & byte_mask(lo, hi), hi64(w) & byte_mask(lo - 8, hi - 8));
}

__device__ __forceinline__ uint32_t high_bits(u32x4 w) { return (w.x | w.y | w.z | w.w) & 0x80808080u; }

// OR of `bits` over the G lanes of this lane's group (G a power of two <= 64).
__device__ __forceinline__ uint32_t group_or(uint32_t bits, uint32_t G) {
  for (uint32_t m = G >> 1; m > 0; m >>= 1) bits |= (uint32_t)__shfl_xor((int)bits, (int)m, 64);
  return bits;
}

// 16-entry byte table lookup for the four bytes of `idx` (each 0..15):
// two v_perm_b32 over the table's halves, the half picked by bit 3.
__device__ __forceinline__ uint32_t lookup16(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t idx) {
  const uint32_t sel = idx & 0x07070707u;
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, sel), hi = __builtin_amdgcn_perm(t3, t2, sel);
  const uint32_t b = idx & 0x08080808u;
  const uint32_t m = (b << 5) - (b >> 3);  // 0xFF in every byte whose bit 3 is set (no multiply)
  return (hi & m) | (lo & ~m);
}

// Bytes of `x` that are >= 0xE0 (p2 must be followed by two continuations) or,
// for `four`, >= 0xF0: bit 7 of each such byte.
__device__ __forceinline__ uint32_t at_least_e0(uint32_t x) { return x & (x << 1) & (x << 2) & 0x80808080u; }
__device__ __forceinline__ uint32_t at_least_f0(uint32_t x) { return at_least_e0(x) & (x << 3); }

// Error bits of four bytes `cur` given the four before them, `prev` (SWAR form
// of the lookup validator of Keiser & Lemire, "Validating UTF-8 in less than
// one instruction per byte"): every byte is checked against the byte before
// it through three 16-entry tables of the nibbles (too short, too long,
// overlong 2/3/4, surrogate, too large, two continuations), and against the
// two and three before it for the continuations a 3- or 4-byte lead asks for.
// Nonzero iff some byte of `cur` breaks strict UTF-8 given its predecessors.
__device__ __forceinline__ uint32_t utf8_dword_errors(uint32_t cur, uint32_t prev) {
  const uint32_t p1 = __builtin_amdgcn_alignbyte(cur, prev, 3);
  const uint32_t p2 = __builtin_amdgcn_alignbyte(cur, prev, 2);
  const uint32_t p3 = __builtin_amdgcn_alignbyte(cur, prev, 1);
  // tables: byte 1's high nibble, byte 1's low nibble, byte 2's high nibble
  // (bits: 0 too short, 1 too long, 2 overlong 3, 3 too large, 4 surrogate,
  // 5 overlong 2, 6 too large 1000 / overlong 4, 7 two continuations)
  const uint32_t sc = lookup16(0x02020202u, 0x02020202u, 0x80808080u, 0x49150121u, (p1 >> 4) & 0x0F0F0F0Fu) &
                      lookup16(0x8383A3E7u, 0xCBCBCB8Bu, 0xCBCBCBCBu, 0xCBCBDBCBu, p1 & 0x0F0F0F0Fu) &
                      lookup16(0x01010101u, 0x01010101u, 0xBABAAEE6u, 0x01010101u, (cur >> 4) & 0x0F0F0F0Fu);
  const uint32_t must23 = at_least_e0(p2) | at_least_f0(p3);
  return must23 ^ sc;
}

// Strict UTF-8 check of one frame's payload bytes [s, fe) by G lanes (lane g
// takes aligned chunks c_lo + g, + G, ...): `chunk(c)` returns aligned chunk c
// and `prev(x)` the dword of bytes x-4 .. x-1 (x a multiple of 16; only bytes
// at or past s are used).  Bytes outside [s, fe) count as 0 (ASCII): a
// sequence cut by the payload's end then fails on the 0 after it, and a chunk
// that ends the payload exactly checks what its last bytes still expect.  An
// all-ASCII chunk with no lead byte just before it is valid outright.
// Returns nonzero if this lane saw an invalid byte (it stops there).
template <class Chunk, class Prev>
__device__ __forceinline__ uint32_t utf8_check_frame(uint64_t s, uint64_t fe, uint32_t g, uint32_t G,
                                                     Chunk chunk, Prev prev_dw) {
  uint32_t bad = 0;
  if (fe <= s) return 0;
  const uint64_t c_lo = s >> 4, c_hi = (fe - 1u) >> 4;
  for (uint64_t c = c_lo + g; c <= c_hi && !bad; c += G) {  // a lane stops at its first invalid chunk
    const uint64_t x = c << 4;
    const int lo_b = (int)((int64_t)s - (int64_t)x), hi_b = (int)((int64_t)fe - (int64_t)x);
    const u32x4 v = keep_bytes(chunk(c), lo_b, hi_b);
    // the three bytes before the chunk that belong to the payload (bytes 1-3 of the dword)
    const uint32_t prev = prev_dw(x) & (uint32_t)byte_mask(lo_b + 4, 4);
    // ASCII, and no lead byte (11xxxxxx) just before: nothing to check
    if (!high_bits(v) && !(prev & (prev << 1) & 0x80808000u)) continue;
    uint32_t err = utf8_dword_errors(v.x, prev) | utf8_dword_errors(v.y, v.x) | utf8_dword_errors(v.z, v.y) |
                   utf8_dword_errors(v.w, v.z);
    if (c == c_hi && hi_b >= 16)  // the payload ends with this chunk: nothing may still be expected
      err |= utf8_pending(v.w >> 24, (v.w >> 16) & 0xFFu, (v.w >> 8) & 0xFFu) ? 1u : 0u;
    bad = err ? 1u : 0u;
  }
  return bad;
}

// Lane g of `lanes` judges a contiguous slice of the payload bytes [s, s + len)
// of a byte-addressed buffer (no alignment needed); nonzero if it saw an invalid byte.
__device__ __forceinline__ uint32_t utf8_slice(const unsigned char* fr, uint64_t s, uint64_t len, uint32_t g,
                                               uint32_t lanes) {
  if (len == 0) return 0;
  const uint64_t per = (len + lanes - 1) / lanes;
  const uint64_t b0 = g * per, b1 = b0 + per < len ? b0 + per : len;
  if (b0 >= b1) return 0;
  uint32_t p3 = b0 >= 3 ? fr[s + b0 - 3] : 0u;
  uint32_t p2 = b0 >= 2 ? fr[s + b0 - 2] : 0u;
  uint32_t p1 = b0 >= 1 ? fr[s + b0 - 1] : 0u;
  uint32_t bad = 0;
  for (uint64_t i = b0; i < b1; ++i) {
    const uint32_t c = fr[s + i];
    bad |= utf8_byte_ok(c, p1, p2, p3) ? 0u : 1u;
    p3 = p2;
    p2 = p1;
    p1 = c;
  }
  if (b1 == len) bad |= utf8_pending(p1, p2, p3) ? 1u : 0u;  // last slice: nothing may still be expected
  return bad;
}

// The same for one lane over a short run of bytes [s, fe) of a byte array
// (small frames: the whole payload by its frame's lane).
template <class Byte>
__device__ __forceinline__ uint32_t utf8_check_bytes(uint32_t s, uint32_t fe, Byte byte_at) {
  uint32_t p1 = 0, p2 = 0, p3 = 0;
  for (uint32_t i = s; i < fe; ++i) {
    const uint32_t c = byte_at(i);
    if (!utf8_byte_ok(c, p1, p2, p3)) return 1u;
    p3 = p2;
    p2 = p1;
    p1 = c;
  }
  return utf8_pending(p1, p2, p3) ? 1u : 0u;
}

}  // namespace rudp
