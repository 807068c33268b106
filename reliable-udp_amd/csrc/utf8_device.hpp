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

// OR of `bits` over the G lanes of this lane's group (G a power of two <= 64,
// every lane of the group active): DPP rows, codec_device.hpp.
__device__ __forceinline__ uint32_t group_or(uint32_t bits, uint32_t G) { return group_or_rows(bits, G); }

// Per-dword inputs of the table check, computed once per dword and shared by
// the dword's own check and the next one's (which needs the bytes before it).
// The nibble tables are looked up on the dword's OWN bytes (a table is
// bytewise, so looking up the bytes and then shifting the results by one byte
// equals shifting the bytes and looking them up): t1 = the "byte before" table
// of its high nibble, t12 = t1 ANDed with the "byte before" table of its low
// nibble (they only ever meet ANDed), t3 = the "this byte" table of its high
// nibble.  A 16-entry table is v_perm_b32 on the nibble's bits 0-2 over 8
// bytes and a blend by bit 3 (a mask of 0xFF per byte whose nibble is 8-15).
// The high-nibble tables need no blend: their selector is bits 4-6 for a byte
// >= 0x80 and a constant entry for an ASCII byte, one v_bitop3_b32 over the
// byte's sign mask -- entry 0 (a continuation's) as the byte before, entry 7
// (0xF_'s, "too short" only) as this byte.  A continuation's "byte before"
// entry, "two continuations", then also stands for an ASCII byte before (Keiser
// & Lemire's "too long"): the error it misses, a continuation after ASCII that
// a lead 2-3 bytes back still owes, is the lead's own "too short" one or two
// bytes earlier in the same payload.  That frees the "too long" bit: in t1 it
// marks a 3- or 4-byte lead (E_, F_) and bit 3 ("too large", F_ only) a 4-byte
// lead, which give the continuations owed 2 and 3 bytes on with no table of
// their own (utf8_dword_errors).
struct Utf8Pre {
  uint32_t t12, t3, t1;
};
// v_bitop3_b32 (gfx950; truth table indexed by s0 s1 s2 as bits 2 1 0): it
// issues faster than v_bfi_b32 / v_or3_b32 (profiles/r05/sweeps/valu_issue_rates.json)
__device__ __forceinline__ uint32_t blend(uint32_t m, uint32_t a, uint32_t b) {
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);  // (m & a) | (~m & b)
}
__device__ __forceinline__ uint32_t or_and(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xA8);  // (a | b) & c
}
__device__ __forceinline__ uint32_t and_xor(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x6A);  // (a & b) ^ c
}
__device__ __forceinline__ uint32_t or3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xFE);  // a | b | c
}
// A 64-bit left shift of a dword pair: one v_lshlrev_b64 issues at the cost
// of one 32-bit left shift (valu_issue_rates.json), so two dwords' shifted
// copies cost one; the compiler would split it into a shift and a v_alignbit.
template <int K>
__device__ __forceinline__ uint64_t shl64(uint64_t x) {
  uint64_t r;
  asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(K), "v"(x));
  return r;
}
template <int K>
__device__ __forceinline__ uint64_t shr64(uint64_t x) {
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(K), "v"(x));
  return r;
}
// The table inputs of dword x given x << 4, x << 12, x << 8 and x >> 4 (of the
// left shifts only bits 15 and 31 are read: the sign bits of bytes 1 and 3
// that v_perm_b32's selectors 8-11 replicate, so a pair's high dword may carry
// the low dword's bits below them; of x >> 4 only bits 0-2 of each byte, so a
// pair's low dword may carry the high dword's bits in bits 28-31).
__device__ __forceinline__ Utf8Pre utf8_pre_from(uint32_t x, uint32_t x4, uint32_t x12, uint32_t x8, uint32_t xr4) {
  const uint32_t sel_lo = x & 0x07070707u, m_lo = __builtin_amdgcn_perm(x4, x12, 0x0B090A08u);  // bit 3 of each byte
  const uint32_t m_hi = __builtin_amdgcn_perm(x, x8, 0x0B090A08u);                              // bit 7
  const uint32_t sel_c = __builtin_amdgcn_bitop3_b32(m_hi, xr4, 0x07070707u, 0x80);  // m & hi: ASCII -> 0
  const uint32_t sel_s = __builtin_amdgcn_bitop3_b32(m_hi, xr4, 0x07070707u, 0x8A);  // 7 & (hi | ~m): ASCII -> 7
  // table bits: 0 too short, 1 (t1) a 3/4-byte lead, 2 overlong 3, 3 too large
  // (t1: a 4-byte lead), 4 surrogate, 5 overlong 2, 6 two continuations (or
  // one after ASCII), 7 too large 1000 / overlong 4
  Utf8Pre p;
  // as the byte before, its high nibble: entries 8-B (and ASCII) 0x40, C 0x21, D 0x01, E 0x17, F 0x8B
  p.t1 = __builtin_amdgcn_perm(0x8B170121u, 0x40404040u, sel_c);
  // as the byte before, its low nibble: all 16 entries
  const uint32_t t2 = blend(m_lo, __builtin_amdgcn_perm(0xCBCBDBCBu, 0xCBCBCBCBu, sel_lo),
                            __builtin_amdgcn_perm(0xCBCBCB4Bu, 0x434363E7u, sel_lo));
  p.t12 = p.t1 & t2;
  // as this byte, its high nibble: 8-B the continuation classes, C-F (and ASCII) 0x01 (too short)
  p.t3 = __builtin_amdgcn_perm(0x01010101u, 0x78786CE4u, sel_s);
  return p;
}
__device__ __forceinline__ Utf8Pre utf8_pre(uint32_t x) { return utf8_pre_from(x, x << 4, x << 12, x << 8, x >> 4); }
// utf8_pre(0), spelled out (the 64-bit shifts are asm, which the compiler does
// not fold): the inputs of any ASCII dword as the bytes before another
__device__ __forceinline__ Utf8Pre utf8_pre_zero() { return Utf8Pre{0x40404040u, 0x01010101u, 0x40404040u}; }
// Two consecutive dwords (x0 before x1) with one 64-bit shift per amount.
__device__ __forceinline__ void utf8_pre2(uint32_t x0, uint32_t x1, Utf8Pre& p0, Utf8Pre& p1) {
  const uint64_t x = ((uint64_t)x1 << 32) | x0;
  const uint64_t x4 = shl64<4>(x), x12 = shl64<12>(x), x8 = shl64<8>(x), xr4 = shr64<4>(x);
  p0 = utf8_pre_from(x0, (uint32_t)x4, (uint32_t)x12, (uint32_t)x8, (uint32_t)xr4);
  p1 = utf8_pre_from(x1, (uint32_t)(x4 >> 32), (uint32_t)(x12 >> 32), (uint32_t)(x8 >> 32), (uint32_t)(xr4 >> 32));
}

// Error bits of the four bytes of a dword (`c`: utf8_pre of it) given the four
// before it (`p`), the SWAR form of the lookup validator of Keiser & Lemire
// ("Validating UTF-8 in less than one instruction per byte"): every byte is
// checked against the byte before it through the three nibble tables, and
// against the two and three before it for the continuations a 3- or 4-byte
// lead asks for.  Nonzero iff some byte breaks strict UTF-8 given its
// predecessors.
__device__ __forceinline__ uint32_t utf8_dword_errors(const Utf8Pre& c, const Utf8Pre& p) {
  const uint32_t t12 = __builtin_amdgcn_alignbyte(c.t12, p.t12, 3);  // byte i: the byte before's tables
  // a continuation is owed from 2 bytes after a 3/4-byte lead (t1 bit 1 two
  // bytes back) and 3 after a 4-byte lead (t1 bit 3 three bytes back), both
  // moved to bit 6 by one funnel shift of the dword pair each
  const uint32_t must23 =
      or_and(__builtin_amdgcn_alignbit(c.t1, p.t1, 11), __builtin_amdgcn_alignbit(c.t1, p.t1, 5), 0x40404040u);
  return and_xor(t12, c.t3, must23);
}

// One payload of V 16-byte windows by the GL lanes of a lane group (GL a
// power of two, 1..16, the groups aligned within the 16-lane DPP rows; lane
// g: windows g, g + GL, ...; `win(v)` returns window v, payload byte 16v on):
// its strict UTF-8 check and, with SUM, the caller's sums (`acc(w, in)` for
// every window, `in` = 0 for one past the end) in the same pass, so every
// window is read from LDS once.  With SUM the first round pair is summed and
// tested: if no window of the wave holds a high bit, the rest is the plain
// sums loop (ASCII waves pay one test) and any high bit it meets goes to *hib
// for the caller's own check (*checked stays false); else the check runs from
// that pair to the end (*checked = true).  A window's bytes before are window
// v - 1's last dword: lane g - 1's this round, lane GL - 1's the round before
// for lane 0 -- at GL = 16 one row_ror:1 of the last dword's table inputs
// serves both, below it a row_shr:1 and a row_ror:(17 - GL).  Rounds go in
// pairs, so the carry alternates registers instead of being copied back.
// Bytes before the payload and after it count as 0, so a sequence cut by its
// end fails on the zero dword the lane holding window V - 1 checks last.
// Returns nonzero if this lane saw an invalid byte; the caller ORs it over the
// group.  Every lane of the group must run it; with SUM it sets the issue
// priority to 0 while it checks (1 after).
// SHORT: V may be under 2 GL + 1 (the varlen tiles' short payloads); without
// it the first round pair is taken to be whole.
template <bool SUM, bool SHORT = true, uint32_t GL = 16, class Window, class Acc>
__device__ __forceinline__ uint32_t utf8_check_windows_rows(uint32_t V, uint32_t g, Window win, Acc acc,
                                                            uint32_t* hib = nullptr, bool* checked = nullptr) {
  static_assert(GL >= 1 && GL <= 16 && (GL & (GL - 1)) == 0, "lane groups of 1-16 lanes");
  const Utf8Pre zero = utf8_pre_zero();
  uint32_t c12 = zero.t12, c1 = zero.t1;  // lane 0's bytes before: zeros (or ASCII)
  Utf8Pre last = zero;
  uint32_t err = 0;
  // in = 0: a window past the payload's end (stale or a clamped re-read), judged but not counted
  auto check = [&](const u32x4& w, bool in) {
    Utf8Pre p1, p2, p3, p4;
    utf8_pre2(w.x, w.y, p1, p2);
    utf8_pre2(w.z, w.w, p3, p4);
    Utf8Pre p0;
    if constexpr (GL == 1) {  // one lane a frame: the lane's own previous window
      p0.t12 = c12;
      p0.t1 = c1;
      c12 = p4.t12;
      c1 = p4.t1;
    } else if constexpr (GL == 16) {
      const uint32_t r12 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t12, 0x121, 0xF, 0xF, false);  // row_ror:1
      const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t1, 0x121, 0xF, 0xF, false);
      p0.t12 = g ? r12 : c12;
      p0.t1 = g ? r1 : c1;
      c12 = r12;
      c1 = r1;
    } else {
      // (every DPP read with the whole group active: a lane the read names must
      // not be masked off by the select that follows)
      constexpr int kRor = 0x120 + (17 - (int)GL);  // lane g = 0 <- lane GL - 1 of its group
      const uint32_t s12 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t12, 0x111, 0xF, 0xF, false);  // row_shr:1
      const uint32_t s1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t1, 0x111, 0xF, 0xF, false);
      const uint32_t r12 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t12, kRor, 0xF, 0xF, false);
      const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)p4.t1, kRor, 0xF, 0xF, false);
      p0.t12 = g ? s12 : c12;
      p0.t1 = g ? s1 : c1;
      c12 = r12;
      c1 = r1;
    }
    const uint32_t e = or3(utf8_dword_errors(p1, p0), utf8_dword_errors(p2, p1), utf8_dword_errors(p3, p2)) |
                       utf8_dword_errors(p4, p3);
    err |= in ? e : 0u;
    last = p4;
  };
  // Rounds of GL windows, every lane in each (a lane's window is in range
  // whenever its predecessor's is, so what it reads across the group was
  // computed that round; the lane holding window V - 1 is never past the end later).
  const uint32_t rounds = (V + GL - 1u) / GL;
  uint32_t j = 0;
  if (SUM) {
    // the first round pair summed and tested for high bits: none in the wave,
    // and the rest is the plain sums loop, any high bit it meets left to the
    // caller's check (*hib); else the check starts with that pair
    auto hbits = [](const u32x4& w) { return or3(w.x, w.y, w.z) | w.w; };
    if (SHORT && V == 0u) return 0u;
    const uint32_t v1 = g + GL;
    const bool in0 = !SHORT || g < V, in1 = !SHORT || v1 < V;
    const u32x4 w0 = win(in0 ? g : V - 1u), w1 = win(in1 ? v1 : V - 1u);
    acc(w0, in0);
    acc(w1, in1);
    if (!__any((((in0 ? hbits(w0) : 0u) | (in1 ? hbits(w1) : 0u)) & 0x80808080u) != 0u)) {
      for (uint32_t v = g + 2u * GL; v < V; v += GL) {
        const u32x4 w = win(v);
        acc(w, true);
        *hib |= hbits(w);
      }
      return 0u;
    }
    __builtin_amdgcn_s_setprio(0);
    *checked = true;
    check(w0, in0);
    check(w1, in1);
    j = 2u;
  }
  for (; j + 2u <= rounds; j += 2u) {  // the first of a pair is always in range (GL (j + 1) < V)
    const uint32_t v = g + GL * j, v1 = v + GL;
    const u32x4 w0 = win(v), w1 = win(v1 < V ? v1 : V - 1u);
    if (SUM) {
      acc(w0, true);
      acc(w1, v1 < V);
    }
    check(w0, true);
    check(w1, v1 < V);
  }
  if (j < rounds) {
    const uint32_t v = g + GL * j;
    const u32x4 w = win(v < V ? v : V - 1u);
    if (SUM) acc(w, v < V);
    check(w, v < V);
  }
  if (V && g == ((V - 1u) & (GL - 1u))) err |= utf8_dword_errors(zero, last);  // nothing may still be expected
  if (SUM) __builtin_amdgcn_s_setprio(1);
  return err;
}
// The 16-lane form (the tiles' MTU shapes).
template <bool SUM, bool SHORT = true, class Window, class Acc>
__device__ __forceinline__ uint32_t utf8_check_windows_row16(uint32_t V, uint32_t g, Window win, Acc acc,
                                                             uint32_t* hib = nullptr, bool* checked = nullptr) {
  return utf8_check_windows_rows<SUM, SHORT, 16>(V, g, win, acc, hib, checked);
}

// Strict UTF-8 of one payload of L bytes by a lane group of GL lanes, with
// nothing else to do on its bytes (the validation kernels): `win(v)` returns
// the payload-aligned window v (any LDS alignment; the last one is masked
// here).  The first round pair is tested for high bits (utf8_check_windows_rows
// with SUM and no sums): with one in the wave the check runs from there;
// without, the rest is read for high bits alone, and a frame that shows one
// is checked over all its windows.  Nonzero if this lane saw an invalid byte;
// every lane of the group must run it.
template <uint32_t GL, class Window>
__device__ __forceinline__ uint32_t utf8_check_payload_rows(uint32_t L, uint32_t g, Window raw) {
  const uint32_t V = (L + 15u) >> 4;
  auto win = [&](uint32_t v) {
    u32x4 w = raw(v);
    if (16u * v + 16u > L) w = keep_bytes(w, 0, (int)(L - 16u * v));
    return w;
  };
  auto none = [](const u32x4&, bool) {};
  uint32_t hib = 0;
  bool checked = false;
  uint32_t bad = utf8_check_windows_rows<true, true, GL>(V, g, win, none, &hib, &checked);
  if (!checked) {
    hib = group_or_rows(hib, GL);
    if (__any((hib & 0x80808080u) != 0u) && (hib & 0x80808080u)) {
      __builtin_amdgcn_s_setprio(0);
      bad = utf8_check_windows_rows<false, true, GL>(V, g, win, none);
      __builtin_amdgcn_s_setprio(1);
    }
  }
  return bad;
}
// The same at a run-time group size: 2-16 lanes (`ok` false for any other G,
// which the caller checks its own way).
template <class Window>
__device__ __forceinline__ uint32_t utf8_check_payload_group(uint32_t L, uint32_t g, uint32_t G, Window raw) {
  return G == 16u  ? utf8_check_payload_rows<16>(L, g, raw)
         : G == 8u ? utf8_check_payload_rows<8>(L, g, raw)
         : G == 4u ? utf8_check_payload_rows<4>(L, g, raw)
                   : utf8_check_payload_rows<2>(L, g, raw);
}

// Strict UTF-8 check of one frame's payload bytes [s, fe) by G lanes (lane g
// takes aligned chunk pairs from c_lo + 2g, every 2G): `chunk(c)` returns aligned chunk c
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
  // lane g takes chunk pairs (c_lo + 2g, + 1), (+ 2G, + 2G + 1), ...: the second
  // chunk's "bytes before" are the first's last dword, already at hand
  for (uint64_t c0 = c_lo + 2u * g; c0 <= c_hi && !bad; c0 += 2u * (uint64_t)G) {  // stops at its first invalid chunk
    uint32_t last = 0;  // the previous chunk's last dword (masked to the payload)
    Utf8Pre q_last;
    bool have_q = false;
#pragma unroll
    for (uint32_t k = 0; k < 2u; ++k) {
      const uint64_t c = c0 + k;
      if (c > c_hi || bad) break;
      const uint64_t x = c << 4;
      const int lo_b = (int)((int64_t)s - (int64_t)x), hi_b = (int)((int64_t)fe - (int64_t)x);
      // an inner chunk (it and the four bytes before it all payload) needs no masks
      const bool inner = lo_b <= -4 && hi_b >= 16;
      const u32x4 raw = chunk(c);
      const u32x4 v = inner ? raw : keep_bytes(raw, lo_b, hi_b);
      // the bytes before the chunk that belong to the payload (bytes 1-3 of the dword)
      uint32_t prev = last;
      if (k == 0) {
        const uint32_t pd = prev_dw(x);
        prev = inner ? pd : pd & (uint32_t)byte_mask(lo_b + 4, 4);
      }
      last = v.w;
      // ASCII, and no lead byte (11xxxxxx) just before: nothing to check (one
      // test: the chunk's high bits, OR bit 6 of the bytes before where bit 7 is set too)
      if (!(or_and(or3(v.x, v.y, v.z), v.w, 0x80808080u) |
            __builtin_amdgcn_bitop3_b32(prev >> 1, prev, 0x40404000u, 0x80))) {
        have_q = false;
        continue;
      }
      const Utf8Pre q0 = have_q ? q_last : utf8_pre(prev);
      Utf8Pre q1, q2, q3, q4;
      utf8_pre2(v.x, v.y, q1, q2);
      utf8_pre2(v.z, v.w, q3, q4);
      uint32_t err = utf8_dword_errors(q1, q0) | utf8_dword_errors(q2, q1) | utf8_dword_errors(q3, q2) |
                     utf8_dword_errors(q4, q3);
      if (c == c_hi && hi_b >= 16)  // the payload ends with this chunk: nothing may still be expected
        err |= utf8_pending(v.w >> 24, (v.w >> 16) & 0xFFu, (v.w >> 8) & 0xFFu) ? 1u : 0u;
      bad = err ? 1u : 0u;
      q_last = q4;
      have_q = true;
    }
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
