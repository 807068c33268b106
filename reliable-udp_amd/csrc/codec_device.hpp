// Device-side helpers shared by the gfx950 codec kernels.
//
// Checksum arithmetic (RFC 1071):
//   S = seq + ack + (flags << 8) + sum_m LE16(payload[2m], payload[2m+1])
// Both layouts put the payload at an ODD frame offset (5 or 7), so a payload
// byte at even index j lands at an odd frame position and is the LOW byte of
// its big-endian frame word: the frame-word sum of the payload equals the sum
// of the payload read as little-endian u16 words — which is what a
// little-endian dword load gives for free, no byte swap anywhere.  The
// header words are seq, ack and flags<<8 (the checksum field counts as 0).
#pragma once
// The diagnostics build (RUDP_TOOLS) puts every internal name in a namespace
// of its own, so its kernels and functions (whose argument structs differ
// from the product's) can never bind to the product library's in one process.
#ifndef RUDP_NS
#if defined(RUDP_TOOLS) && RUDP_TOOLS
#define RUDP_NS rudp_tools
#else
#define RUDP_NS rudp
#endif
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace RUDP_NS {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;  // 4 waves of 64

// An MI355X deals a launch's workgroups round-robin over its 8 XCDs (blocks
// b, b + 8, ... run on one XCD, each XCD with its own L2).  xcd_tile(b, nt)
// renumbers them so XCD x owns the contiguous run of tiles
// [x*per + min(x, rem), ...) of nt = per*8 + rem: every XCD streams its own
// slice of the batch front to back.  Bijective over [0, nt).
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nt) {
  const uint32_t per = nt / kXcds, rem = nt % kXcds;
  const uint32_t x = b % kXcds, k = b / kXcds;
  return x * per + (x < rem ? x : rem) + k;
}

// Reductions over a lane group of G lanes (G a power of two, groups aligned
// to G lanes, every lane of the group active): DPP row operations up to 16
// lanes -- quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror, each
// pairing a lane with one in the other half of its 2/4/8/16 -- instead of a
// ds_bpermute round trip per step; the 32- and 64-lane steps stay shuffles.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_row(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t group_sum(uint32_t x, uint32_t G) {
  if (G >= 2u) x += dpp_row<0xB1>(x);
  if (G >= 4u) x += dpp_row<0x4E>(x);
  if (G >= 8u) x += dpp_row<0x141>(x);
  if (G >= 16u) x += dpp_row<0x140>(x);
  if (G >= 32u) x += (uint32_t)__shfl_xor((int)x, 16, 64);
  if (G >= 64u) x += (uint32_t)__shfl_xor((int)x, 32, 64);
  return x;
}
__device__ __forceinline__ uint32_t group_or_rows(uint32_t x, uint32_t G) {
  if (G >= 2u) x |= dpp_row<0xB1>(x);
  if (G >= 4u) x |= dpp_row<0x4E>(x);
  if (G >= 8u) x |= dpp_row<0x141>(x);
  if (G >= 16u) x |= dpp_row<0x140>(x);
  if (G >= 32u) x |= (uint32_t)__shfl_xor((int)x, 16, 64);
  if (G >= 64u) x |= (uint32_t)__shfl_xor((int)x, 32, 64);
  return x;
}

// Maximum of a u32 over the whole wave (DPP row steps, then two shuffles).
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
  x = max(x, dpp_row<0xB1>(x));
  x = max(x, dpp_row<0x4E>(x));
  x = max(x, dpp_row<0x141>(x));
  x = max(x, dpp_row<0x140>(x));
  x = max(x, (uint32_t)__shfl_xor((int)x, 16, 64));
  x = max(x, (uint32_t)__shfl_xor((int)x, 32, 64));
  return x;
}

// Sum of a u64 over the whole wave: the 16-lane steps by DPP on the two
// halves (carry added by hand), the 32- and 64-lane steps as shuffles.
template <int CTRL>
__device__ __forceinline__ void add64_rows(uint32_t& lo, uint32_t& hi) {
  const uint32_t l2 = dpp_row<CTRL>(lo), h2 = dpp_row<CTRL>(hi);
  const uint32_t s = lo + l2;
  hi = hi + h2 + (s < lo ? 1u : 0u);
  lo = s;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  add64_rows<0xB1>(lo, hi);
  add64_rows<0x4E>(lo, hi);
  add64_rows<0x141>(lo, hi);
  add64_rows<0x140>(lo, hi);
  uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// End-around-carry fold of a 32-bit partial sum to 16 bits.
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xFFFFu) + (s >> 16);
  s = (s & 0xFFFFu) + (s >> 16);
  return s;
}

// A partial word sum of any size brought to at most 0x1FFFE with its value
// mod 0xFFFF and its zero-ness kept (2^16 = 1 mod 0xFFFF): a checksum folded
// from such parts equals the one folded from the exact total.  The decode
// paths that take frames of any length (untrusted offsets) fold before sums
// could pass 2^32.
__device__ __forceinline__ uint32_t fold_keep(uint64_t s) {
  s = (s & 0xFFFFFFFFull) + (s >> 32);
  s = (s & 0xFFFFull) + (s >> 16);
  s = (s & 0xFFFFull) + (s >> 16);
  return (uint32_t)s;
}

// Sum of the eight little-endian u16 halves of a 16-byte vector.
// (v_dot2_u32_u16 against {1, 1} adds a dword's two u16 halves to an
// accumulator in one instruction, where the masks, shifts and adds took ~4)
typedef unsigned short rudp_us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t le16_acc(uint32_t x, uint32_t acc) {
  const rudp_us2 one = {1, 1};
  return __builtin_amdgcn_udot2(__builtin_bit_cast(rudp_us2, x), one, acc, false);
}
// Byte sums by position parity with v_dot4_u32_u8: bytes 0 and 2 (even) or 1
// and 3 (odd) of x added to acc in one instruction.
__device__ __forceinline__ uint32_t even_bytes_acc(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_udot4(x, 0x00010001u, acc, false);
}
__device__ __forceinline__ uint32_t odd_bytes_acc(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_udot4(x, 0x01000100u, acc, false);
}
__device__ __forceinline__ uint32_t even_bytes(u32x4 w) {
  return even_bytes_acc(w.w, even_bytes_acc(w.z, 0u)) + even_bytes_acc(w.y, even_bytes_acc(w.x, 0u));
}
__device__ __forceinline__ uint32_t odd_bytes(u32x4 w) {
  return odd_bytes_acc(w.w, odd_bytes_acc(w.z, 0u)) + odd_bytes_acc(w.y, odd_bytes_acc(w.x, 0u));
}
__device__ __forceinline__ uint32_t le16_sum(u32x4 v) {
  return le16_acc(v.w, le16_acc(v.z, 0u)) + le16_acc(v.y, le16_acc(v.x, 0u));
}

// RFC 1071 checksum of one packet from its payload word sum and header.
__device__ __forceinline__ uint32_t packet_csum(uint32_t payload_sum, uint32_t seq, uint32_t ack,
                                                uint32_t flags) {
  return (~fold16(payload_sum + seq + ack + (flags << 8))) & 0xFFFFu;
}

// Header bytes in frame order packed little-endian into a u64 (byte p of the
// frame at bits 8p).  H = 5 leaves the checksum out.
template <int H>
__device__ __forceinline__ uint64_t pack_header(uint32_t seq, uint32_t ack, uint32_t flags,
                                                uint32_t csum) {
  uint64_t h = (uint64_t)(seq >> 8) | ((uint64_t)(seq & 0xFFu) << 8) |
               ((uint64_t)(ack >> 8) << 16) | ((uint64_t)(ack & 0xFFu) << 24) |
               ((uint64_t)(flags & 0xFFu) << 32);
  if (H == 7) h |= ((uint64_t)(csum >> 8) << 40) | ((uint64_t)(csum & 0xFFu) << 48);
  return h;
}

// Mask of bytes [a, b) of an 8-byte word; a and b may lie outside [0, 8].
__device__ __forceinline__ uint64_t byte_mask(int a, int b) {
  a = a < 0 ? 0 : a;
  b = b > 8 ? 8 : b;
  if (b <= a) return 0ull;
  uint64_t upto_b = (b >= 8) ? ~0ull : ((1ull << (8 * b)) - 1ull);
  uint64_t below_a = (a == 0) ? 0ull : ((1ull << (8 * a)) - 1ull);
  return upto_b & ~below_a;
}

__device__ __forceinline__ uint64_t lo64(u32x4 v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }
__device__ __forceinline__ uint64_t hi64(u32x4 v) { return (uint64_t)v.z | ((uint64_t)v.w << 32); }
__device__ __forceinline__ u32x4 make_u32x4(uint64_t lo, uint64_t hi) {
  u32x4 r;
  r.x = (uint32_t)lo;
  r.y = (uint32_t)(lo >> 32);
  r.z = (uint32_t)hi;
  r.w = (uint32_t)(hi >> 32);
  return r;
}

// 16 bytes starting at an arbitrary byte offset of a 4-byte-aligned region,
// from five aligned dword reads and a byte funnel shift.
__device__ __forceinline__ u32x4 window16_dw(const uint32_t* base_dw, uint32_t byte_off) {
  const uint32_t* w = base_dw + (byte_off >> 2);
  uint32_t sh = byte_off & 3u;
  uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  u32x4 r;
  r.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
  r.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
  r.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
  r.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
  return r;
}

// 16 bytes from a 32-byte register pair (a = bytes 0-15, b = bytes 16-31)
// starting at byte `sh` (0..15): dword select then byte funnel.
__device__ __forceinline__ u32x4 funnel32(u32x4 a, u32x4 b, uint32_t sh) {
  // s_i = dword (i + sh/4) of a:b as two select levels on plain scalars.  No
  // array here on purpose: hipcc turns selects between elements of a private
  // array back into a runtime index and demotes the array to LDS/scratch.
  const bool two = (sh & 8u) != 0, one = (sh & 4u) != 0;
  const uint32_t bs = sh & 3u;
  const uint32_t e0 = two ? a.z : a.x, e1 = two ? a.w : a.y, e2 = two ? b.x : a.z,
                 e3 = two ? b.y : a.w, e4 = two ? b.z : b.x, e5 = two ? b.w : b.y;
  const uint32_t s0 = one ? e1 : e0, s1 = one ? e2 : e1, s2 = one ? e3 : e2, s3 = one ? e4 : e3,
                 s4 = one ? e5 : e4;
  u32x4 r;
  r.x = __builtin_amdgcn_alignbyte(s1, s0, bs);
  r.y = __builtin_amdgcn_alignbyte(s2, s1, bs);
  r.z = __builtin_amdgcn_alignbyte(s3, s2, bs);
  r.w = __builtin_amdgcn_alignbyte(s4, s3, bs);
  return r;
}

// 16 bytes at frames[off], off 16-byte aligned; bytes at or past `total`
// read as zero (only the last packets of a batch take the byte path).
__device__ __forceinline__ u32x4 load16_guarded(const unsigned char* frames, uint64_t off,
                                                uint64_t total) {
  if (off + 16 <= total)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(frames + off));
  uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
  for (uint32_t b = 0; b < 16; ++b) {
    const uint32_t v = (off + b < total) ? (uint32_t)frames[off + b] << (8 * (b & 3)) : 0u;
    if (b < 4) d0 |= v;
    else if (b < 8) d1 |= v;
    else if (b < 12) d2 |= v;
    else d3 |= v;
  }
  u32x4 r;
  r.x = d0;
  r.y = d1;
  r.z = d2;
  r.w = d3;
  return r;
}

// Aligned 16-B chunk X of the output around a packet's header, P = the
// output offset of its payload: the previous packet's last payload bytes
// (`tail`: its last 16), the header bytes `h` (frame order, packed
// little-endian) and the first payload bytes (`head`).  X is one of the one
// or two chunks [floor16(P - H), ceil16(P)).
template <int H>
__device__ __forceinline__ u32x4 header_chunk(uint64_t X, uint64_t P, uint64_t h, u32x4 tail,
                                              u32x4 head) {
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const int k0 = (int)(int64_t)(X - (P - H));  // frame position of chunk byte 0 (> -16)
  u32x4 w = zero;
  if (k0 < 0) w = funnel32(tail, zero, (uint32_t)(k0 + 16));  // previous payload's last bytes
  const uint32_t d = (uint32_t)(P - X);                        // payload starts d bytes in
  if (d < 16) {
    const u32x4 hp = funnel32(zero, head, 16u - d);
    w.x |= hp.x; w.y |= hp.y; w.z |= hp.z; w.w |= hp.w;
  }
  uint64_t lo = lo64(w), hi = hi64(w);
  if (k0 >= 0) {
    lo |= h >> (8 * k0);
  } else {
    const int sh = -k0;
    if (sh < 8) {
      lo |= h << (8 * sh);
      hi |= h >> (64 - 8 * sh);
    } else {
      hi |= h << (8 * (sh - 8));
    }
  }
  return make_u32x4(lo, hi);
}

}  // namespace rudp
