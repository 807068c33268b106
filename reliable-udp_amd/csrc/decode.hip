// Batched parse + verify (decode) kernels for gfx950.
//
// Replaces the per-packet decode of the reference, utils/reliableUDP.py:118-123
// and :67-73: Packet(data) (utils/packet.py:16) -> get_header_field seq/ack/
// syn/ack/fin (:29-40) -> get_payload (:68-73), plus verification of the
// build-defined RFC 1071 checksum.
//
// Fast kernel (payload_len % 16 == 0, tile within 64 KiB of LDS):
// decode_tile_kernel.  A workgroup owns T = 256/G frames (T % 16 == 0, so the
// tile starts 16-B aligned); phase 1 streams the tile's T*F bytes into LDS as
// one contiguous run; G lanes per frame sum its payload's LE u16 halves from
// byte-shifted LDS windows; the leader parses the header (rudp5 sideband
// checksums are loaded before phase 1) and the outputs go out as whole dwords
// through LDS.  With payload_out, the tile's payloads stream out as one
// contiguous run.  Every frame byte leaves HBM once.  Frames too large for an
// LDS tile take decode_verify_kernel (aligned chunks, parity-weighted sums) or
// decode_vec_kernel (register windows).  Any other shape (payloads not a
// multiple of 16 B, unaligned views) decodes through the varlen tiles with
// implicit offsets (capi.hip rudp_decode_utf8, VarlenArgs::stride).
#include "codec_device.hpp"
#include "internal.hpp"
#include "utf8_device.hpp"

namespace RUDP_NS {

__device__ __forceinline__ u32x4 window16_global(const unsigned char* frames, uint64_t off,
                                                 uint64_t total) {
  const uint64_t al = off & ~15ull;
  const u32x4 a = load16_guarded(frames, al, total);
  const u32x4 b = load16_guarded(frames, al + 16, total);
  return funnel32(a, b, (uint32_t)(off & 15u));
}

// PRELOADED (rudp5): `inband` carries the sideband checksum the caller
// already loaded; otherwise it is read here.
template <int H, bool PRELOADED = false>
__device__ __forceinline__ void finish_packet(const DecodeArgs& a, uint64_t p, uint32_t sum,
                                              uint32_t seq, uint32_t ack, uint32_t flags,
                                              uint32_t inband) {
  const uint32_t c = packet_csum(sum, seq, ack, flags);
  uint8_t ok;
  if (H == 7)
    ok = (c == inband) ? 1 : 0;
  else if (a.csum_in)
    ok = (c == (PRELOADED ? inband : (uint32_t)a.csum_in[p])) ? 1 : 0;  // rudp5: the sideband value
  else
    ok = 3;
  a.seq[p] = (uint16_t)seq;
  a.ack[p] = (uint16_t)ack;
  a.flags[p] = (uint8_t)flags;
  a.ok[p] = ok;
  if (a.csum_out) a.csum_out[p] = (uint16_t)c;
}

template <int H>
__global__ void __launch_bounds__(kBlock) decode_vec_kernel(DecodeArgs a) {
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog;
  const uint32_t G = 1u << glog;
  const uint32_t q = tid >> glog;
  const uint32_t g = tid & (G - 1u);
  const uint64_t p = (uint64_t)blockIdx.x * (kBlock >> glog) + q;
  const bool valid = p < a.n;
  const uint32_t F = a.F;
  const uint32_t L = F - H;
  const uint32_t V = L >> 4;
  const uint64_t total = a.n * (uint64_t)F;
  const uint64_t fbase = p * (uint64_t)F;

  uint32_t sum = 0;
  if (valid) {
    for (uint32_t v0 = g; v0 < V; v0 += 4u * G) {
      u32x4 w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t v = v0 + (uint32_t)u * G;
        if (v < V) w[u] = window16_global(a.frames, fbase + H + 16ull * v, total);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t v = v0 + (uint32_t)u * G;
        if (v < V) {
          sum += le16_sum(w[u]);
          if (a.payload_out)
            __builtin_nontemporal_store(
                w[u], reinterpret_cast<u32x4*>(a.payload_out + p * (uint64_t)L + 16ull * v));
        }
      }
    }
  }
  for (uint32_t m = G >> 1; m > 0; m >>= 1) sum += __shfl_xor(sum, (int)m, 64);
  if (g == 0 && valid) {
    const u32x4 h = window16_global(a.frames, fbase, total);
    const uint32_t seq = ((h.x & 0xFFu) << 8) | ((h.x >> 8) & 0xFFu);
    const uint32_t ack = (((h.x >> 16) & 0xFFu) << 8) | (h.x >> 24);
    const uint32_t flags = h.y & 0xFFu;
    const uint32_t inband = (((h.y >> 8) & 0xFFu) << 8) | ((h.y >> 16) & 0xFFu);
    finish_packet<H>(a, p, sum, seq, ack, flags, inband);
  }
}

// Zero-copy verify (no payload_out): G lanes per packet load the ALIGNED
// 16-byte chunks that overlap the packet's frame [p*F, p*F + F) exactly once
// each (coalesced dwordx4 across the group; the two boundary chunks are
// shared with the neighbour packets and come from L2).  No realignment: the
// frame's big-endian word sum is a parity-weighted byte sum — a byte at
// frame position k is the high byte of its word iff k is even, and since F
// is odd, k = x - p*F has the parity of x + p for global offset x.  So each
// lane sums bytes at even / odd global offsets (masked to the frame at the
// two boundary chunks) and weights them by the packet's parity.  The header
// comes from the group's first two chunks (lanes 0 and 1, one shuffle).  The
// in-band checksum's own bytes are then taken back out of the exact integer
// sum before the fold.
template <int H>
__global__ void __launch_bounds__(kBlock) decode_verify_kernel(DecodeArgs a) {
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog;
  const uint32_t G = 1u << glog;
  const uint32_t q = tid >> glog;
  const uint32_t g = tid & (G - 1u);
  const uint64_t p = (uint64_t)blockIdx.x * (kBlock >> glog) + q;
  const bool valid = p < a.n;
  const uint64_t F = a.F;
  const uint64_t total = a.n * F;
  const uint64_t fstart = p * F;
  const uint64_t fend = fstart + F;
  const uint64_t c_lo = fstart >> 4;
  const uint32_t nchunks = valid ? (uint32_t)(((fend - 1) >> 4) - c_lo + 1) : 0u;

  uint32_t even_sum = 0, odd_sum = 0;  // byte sums at even / odd global offsets
  u32x4 first = {0u, 0u, 0u, 0u};
  for (uint32_t i0 = g; i0 < nchunks; i0 += 8u * G) {
    uint32_t even = 0, odd = 0;  // (v_dot4_u32_u8 byte sums, codec_device.hpp)
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = i0 + (uint32_t)u * G;
      if (i < nchunks) v[u] = load16_guarded(a.frames, (c_lo + i) << 4, total);
    }
    if (i0 == g) first = v[0];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = i0 + (uint32_t)u * G;
      if (i < nchunks) {
        u32x4 w = v[u];
        if (i == 0 || i + 1 == nchunks) {  // boundary chunk: keep this frame's bytes only
          const int64_t cb = (int64_t)((c_lo + i) << 4);
          const int lo = (int)((int64_t)fstart - cb), hi = (int)((int64_t)fend - cb);
          const uint64_t l = lo64(w) & byte_mask(lo, hi), h = hi64(w) & byte_mask(lo - 8, hi - 8);
          w = make_u32x4(l, h);
        }
        even += even_bytes(w);
        odd += odd_bytes(w);
      }
    }
    even_sum += even;
    odd_sum += odd;
  }
  // frame position parity = parity(x + p): even-offset bytes are high bytes iff p is even
  uint32_t sum = (p & 1u) ? (even_sum + (odd_sum << 8)) : ((even_sum << 8) + odd_sum);
  for (uint32_t m = G >> 1; m > 0; m >>= 1) sum += __shfl_xor(sum, (int)m, 64);
  // header bytes: frame start lies in the group's first chunk, at most 6 bytes spill into the next
  const int src = (int)((threadIdx.x & 63u) + 1u);
  u32x4 next;
  next.x = __shfl(first.x, src, 64);
  next.y = __shfl(first.y, src, 64);
  next.z = __shfl(first.z, src, 64);
  next.w = __shfl(first.w, src, 64);
  if (g == 0 && valid) {
    const u32x4 h = funnel32(first, next, (uint32_t)(fstart & 15u));
    const uint32_t seq = ((h.x & 0xFFu) << 8) | ((h.x >> 8) & 0xFFu);
    const uint32_t ack = (((h.x >> 16) & 0xFFu) << 8) | (h.x >> 24);
    const uint32_t flags = h.y & 0xFFu;
    const uint32_t inband = (((h.y >> 8) & 0xFFu) << 8) | ((h.y >> 16) & 0xFFu);
    // the sum above covered the whole frame; the checksum field (bytes 5, 6:
    // odd then even position) contributed byte-swapped — take it back out
    const uint32_t payload_and_rest =
        sum - seq - ack - (flags << 8) - (H == 7 ? (((inband & 0xFFu) << 8) | (inband >> 8)) : 0u);
    finish_packet<H>(a, p, payload_and_rest, seq, ack, flags, inband);
  }
}

#if RUDP_TOOLS
// Diagnostics: a decode tile's timeline (100 MHz wall clock), XCD and CU, as
// 6 u64 at trace[6 * block]: {start, staged, summed, end, XCC, CU}.  Thread 0
// records each stamp, so "end" is thread 0's end (outputs of the other waves
// may still be in flight).
__device__ __forceinline__ void decode_trace_record(const DecodeArgs& a, uint32_t block, uint64_t t_start,
                                                    uint64_t t_staged, uint64_t t_summed) {
  if (!a.trace || threadIdx.x != 0) return;
  const uint64_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID[3:0]
  u32x4* rec = reinterpret_cast<u32x4*>(a.trace + 6ull * block);
  rec[0] = make_u32x4(t_start, t_staged);
  rec[1] = make_u32x4(t_summed, (uint64_t)wall_clock64());
  rec[2] = make_u32x4(xcc, (uint64_t)__smid());
}
#endif

// Decode through LDS, verify-only or with payload copy-out: the mirror of the
// encode tile kernel.  A workgroup owns T = 256/G frames; T is a multiple of
// 16, so the tile's frames start 16-byte aligned.  Phase 1 streams them into
// LDS like a copy (lane t: vectors t, t+256, ...).  Phase 2: G lanes per frame
// read the payload back as byte-shifted LDS windows (5 ds_read_b32 +
// v_alignbyte) and sum the LE u16 halves; the group leader parses the header
// out of LDS.  Copy-out streams the same windows to payload_out as one
// contiguous run per tile.
// U8: each payload's strict UTF-8 check in the same pass (a.valid; the
// reference decodes every payload, utils/reliableUDP.py:121 ->
// utils/packet.py:73): the windows' high bits are OR'ed as they are summed,
// and only a frame with a high bit runs the byte checks over its LDS chunks.
// FUSE (U8, 16 lanes a frame, payloads of 1 KiB and more; launch_decode_tile_u8
// picks it): a payload whose first windows hold a high bit has its sums and
// its UTF-8 check in one pass.  Its own instantiation, so the other shapes run
// the code they were measured with.
template <int H, bool COPY, bool U8, bool FUSE = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(U8 ? 8 : 1))) decode_tile_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog;
  const uint32_t G = 1u << glog;
  const uint32_t T = kBlock >> glog;
  const uint32_t q = tid >> glog;
  const uint32_t g = tid & (G - 1u);
  const uint64_t p0 = (uint64_t)(a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x) * T;
  const uint64_t left = a.n - p0;
  const uint32_t Tv = left < T ? (uint32_t)left : T;
  const uint32_t F = a.F;
  const uint32_t L = F - H;
#if RUDP_TOOLS
  const uint64_t t_start = a.trace ? (uint64_t)wall_clock64() : 0ull;
  uint64_t t_staged = 0, t_summed = 0;
#endif
  // Issue priority (U8): every phase at 1 but the byte checks of a wave whose
  // frames hold a high bit, at 0, so the few instructions of the CU's other
  // tiles' staging and sums are not held behind a long check, which wins
  // issue by age otherwise; ASCII tiles keep one priority throughout.
  if (U8) __builtin_amdgcn_s_setprio(1);
  const uint64_t total = a.n * (uint64_t)F;
  const uint64_t base = p0 * (uint64_t)F;  // 16-byte aligned: T % 16 == 0
  const uint32_t nbytes = Tv * F;
  const uint32_t nvec = (nbytes + 15u) >> 4;
  u32x4* tile = reinterpret_cast<u32x4*>(lds);
  // rudp5 sideband checksums: the leaders load theirs before phase 1, so the
  // round trip overlaps the frame stream instead of following the sums.
  uint32_t want_cs = 0;
  if (H == 5 && a.csum_in && (tid & ((1u << a.glog) - 1u)) == 0 && (tid >> a.glog) < Tv)
    want_cs = a.csum_in[p0 + (tid >> a.glog)];
  // Lanes are dealt vectors from the tile's first 64-B boundary on (the 0-3
  // vectors before it go last): every wave's 1 KiB load covers whole sectors.
  uint32_t npre = a.align64 ? (uint32_t)((-reinterpret_cast<uintptr_t>(a.frames + base)) & 63u) >> 4 : 0u;
  if (npre > nvec) npre = nvec;
  for (uint32_t v0 = tid; v0 < nvec; v0 += 8u * kBlock) {
    u32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      uint32_t v = v0 + (uint32_t)u * kBlock + npre;
      v = v < nvec ? v : v - nvec;
      if (v0 + (uint32_t)u * kBlock < nvec) r[u] = load16_guarded(a.frames, base + 16ull * v, total);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      uint32_t v = v0 + (uint32_t)u * kBlock + npre;
      v = v < nvec ? v : v - nvec;
      if (v0 + (uint32_t)u * kBlock < nvec) tile[v] = r[u];
    }
  }
  __syncthreads();
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_staged = (uint64_t)wall_clock64();
#endif
  const uint32_t* dw = reinterpret_cast<const uint32_t*>(lds);
  // the leader's header window, read now so its LDS round trip overlaps the sums
  u32x4 hdr = make_u32x4(0ull, 0ull);
  if (g == 0 && q < Tv) hdr = window16_dw(dw, q * F);
  uint32_t sum = 0, hib = 0, u8bad = 0;
  const uint64_t p = p0 + q;
  const uint32_t V = L >> 4;
  // FUSE: a payload whose first windows hold a high bit has its windows read
  // once for its sums and its UTF-8 check (`fused`, wave-uniform)
  bool fused = false;
  if (FUSE) {
    if (q < Tv) {
      const uint32_t pay = q * F + H;
      u8bad = utf8_check_windows_row16<true, false>(  // (V >= 64)
          V, g, [&](uint32_t v) { return window16_dw(dw, pay + 16u * v); },
          [&](const u32x4& w, bool in) { sum += in ? le16_sum(w) : 0u; }, &hib, &fused);
    }
  } else if (q < Tv) {
    const uint32_t pay = q * F + H;  // LDS byte offset of the payload
    for (uint32_t v = g; v < V; v += G) {
      const u32x4 w = window16_dw(dw, pay + 16u * v);
      sum += le16_sum(w);
      if (U8) hib |= w.x | w.y | w.z | w.w;
    }
  }

  if (COPY) {
    // The tile's payload_out range is contiguous (Tv*L bytes, 16-B aligned):
    // store it as one stream, lane t taking vectors t, t+256, ... so every
    // wave-instruction writes 1 KiB contiguous.  Vector j is vector j % V of
    // packet j / V, tracked incrementally (no per-vector division).
    // From the first 64-B boundary on, as phase 1 (the wrapped tail is
    // re-derived by one division).
    const uint32_t nv = Tv * V;
    const uint32_t dq = kBlock / V, dv = kBlock % V;
    u32x4* dst = reinterpret_cast<u32x4*>(a.payload_out + p0 * (uint64_t)L);
    uint32_t jpre = a.align64 ? (uint32_t)((-(reinterpret_cast<uintptr_t>(dst))) & 63u) >> 4 : 0u;
    if (jpre > nv) jpre = nv;
    uint32_t j = tid + jpre;
    if (j >= nv) j -= nv;
    uint32_t qj = j / V, vj = j - qj * V;
    for (uint32_t k = tid; k < nv; k += kBlock) {
      __builtin_nontemporal_store(window16_dw(dw, qj * F + H + 16u * vj), dst + j);
      j += kBlock;
      if (j >= nv) {
        j -= nv;
        qj = j / V;
        vj = j - qj * V;
      } else {
        qj += dq;
        vj += dv;
        if (vj >= V) { vj -= V; ++qj; }
      }
    }
  }
  sum = group_sum(sum, G);
  if (U8) hib = group_or_rows(hib, G);
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_summed = (uint64_t)wall_clock64();
#endif
  if (fused) {
    u8bad = group_or_rows(u8bad, 16u) ? 1u : 0u;
  } else if (U8 && __any((hib & 0x80808080u) != 0)) {  // the byte checks, for waves whose frames hold a high bit
    __builtin_amdgcn_s_setprio(0);
    if (G == 16u) {
      // each payload over the windows the sums read, the bytes before a window handed on by DPP
      if ((hib & 0x80808080u) && q < Tv) {  // hib and q are the row's (the frame's)
        u8bad = utf8_check_windows_row16<false>(
            V, g, [&](uint32_t v) { return window16_dw(dw, q * F + H + 16u * v); }, [](const u32x4&, bool) {});
      }
      u8bad = group_or_rows(u8bad, 16u) ? 1u : 0u;
    } else if (G >= 2u) {
      // 2-8 lanes a frame: the same window check in lane groups (DPP within the rows)
      if ((hib & 0x80808080u) && q < Tv) {  // hib and q are the group's (the frame's)
        auto win = [&](uint32_t v) { return window16_dw(dw, q * F + H + 16u * v); };
        auto none = [](const u32x4&, bool) {};
        u8bad = G == 8u   ? utf8_check_windows_rows<false, true, 8>(V, g, win, none)
                : G == 4u ? utf8_check_windows_rows<false, true, 4>(V, g, win, none)
                          : utf8_check_windows_rows<false, true, 2>(V, g, win, none);
      }
      u8bad = group_or_rows(u8bad, G) ? 1u : 0u;
    } else {  // one lane a frame (payloads of 16-63 B): its windows in turn
      if ((hib & 0x80808080u) && q < Tv)
        u8bad = utf8_check_windows_rows<false, true, 1>(
            V, g, [&](uint32_t v) { return window16_dw(dw, q * F + H + 16u * v); }, [](const u32x4&, bool) {});
    }
    __builtin_amdgcn_s_setprio(1);
  }
  if (!a.stage_out) {
    if (g == 0 && q < Tv) {
      const u32x4 h = hdr;
      const uint32_t seq = ((h.x & 0xFFu) << 8) | ((h.x >> 8) & 0xFFu);
      const uint32_t ack = (((h.x >> 16) & 0xFFu) << 8) | (h.x >> 24);
      const uint32_t flags = h.y & 0xFFu;
      const uint32_t inband = (((h.y >> 8) & 0xFFu) << 8) | ((h.y >> 16) & 0xFFu);
      finish_packet<H, true>(a, p, sum, seq, ack, flags, H == 5 ? want_cs : inband);
      if (U8) a.valid[p] = u8bad ? 0 : 1;
    }
#if RUDP_TOOLS
    decode_trace_record(a, blockIdx.x, t_start, t_staged, t_summed);
#endif
    return;
  }
  // Outputs staged in LDS after the tile (seq, ack, csum u16 [T]; flags, ok
  // u8 [T]), then written as whole dwords: one wave-instruction covers 256 B
  // of an output array instead of each leader storing 1-2 bytes into five.
  const uint32_t st = (nbytes + 32u + 15u) & ~15u;
  uint16_t* s_seq = reinterpret_cast<uint16_t*>(lds + st);
  uint16_t* s_ack = s_seq + T;
  uint16_t* s_cs = s_ack + T;
  uint8_t* s_flags = reinterpret_cast<uint8_t*>(s_cs + T);
  uint8_t* s_ok = s_flags + T;
  uint8_t* s_valid = s_ok + T;  // U8
  if (g == 0 && q < Tv) {
    const u32x4 h = hdr;
    const uint32_t seq = ((h.x & 0xFFu) << 8) | ((h.x >> 8) & 0xFFu);
    const uint32_t ack = (((h.x >> 16) & 0xFFu) << 8) | (h.x >> 24);
    const uint32_t flags = h.y & 0xFFu;
    const uint32_t inband = (((h.y >> 8) & 0xFFu) << 8) | ((h.y >> 16) & 0xFFu);
    const uint32_t c = packet_csum(sum, seq, ack, flags);
    uint8_t ok;
    if (H == 7) ok = (c == inband) ? 1 : 0;
    else if (a.csum_in) ok = (c == want_cs) ? 1 : 0;
    else ok = 3;
    s_seq[q] = (uint16_t)seq;
    s_ack[q] = (uint16_t)ack;
    s_cs[q] = (uint16_t)c;
    s_flags[q] = (uint8_t)flags;
    s_ok[q] = ok;
    if (U8) s_valid[q] = u8bad ? 0 : 1;
  }
  __syncthreads();
  if (Tv == T) {  // T % 16 == 0 and p0 % 16 == 0: every array slice is dword aligned
    const uint32_t w16 = T / 2u, w8 = T / 4u;
    const uint32_t* l_seq = reinterpret_cast<const uint32_t*>(s_seq);
    const uint32_t* l_ack = reinterpret_cast<const uint32_t*>(s_ack);
    const uint32_t* l_cs = reinterpret_cast<const uint32_t*>(s_cs);
    const uint32_t* l_fl = reinterpret_cast<const uint32_t*>(s_flags);
    const uint32_t* l_ok = reinterpret_cast<const uint32_t*>(s_ok);
    const uint32_t* l_valid = reinterpret_cast<const uint32_t*>(s_valid);
    for (uint32_t i = tid; i < w16; i += kBlock) {
      reinterpret_cast<uint32_t*>(a.seq + p0)[i] = l_seq[i];
      reinterpret_cast<uint32_t*>(a.ack + p0)[i] = l_ack[i];
      if (a.csum_out) reinterpret_cast<uint32_t*>(a.csum_out + p0)[i] = l_cs[i];
    }
    for (uint32_t i = tid; i < w8; i += kBlock) {
      reinterpret_cast<uint32_t*>(a.flags + p0)[i] = l_fl[i];
      reinterpret_cast<uint32_t*>(a.ok + p0)[i] = l_ok[i];
      if (U8) reinterpret_cast<uint32_t*>(a.valid + p0)[i] = l_valid[i];
    }
  } else {
    for (uint32_t i = tid; i < Tv; i += kBlock) {
      a.seq[p0 + i] = s_seq[i];
      a.ack[p0 + i] = s_ack[i];
      if (a.csum_out) a.csum_out[p0 + i] = s_cs[i];
      a.flags[p0 + i] = s_flags[i];
      a.ok[p0 + i] = s_ok[i];
      if (U8) a.valid[p0 + i] = s_valid[i];
    }
  }
#if RUDP_TOOLS
  decode_trace_record(a, blockIdx.x, t_start, t_staged, t_summed);
#endif
}

template <int H, bool COPY, bool U8, bool FUSE = false>
static int launch_decode_tile(const DecodeArgs& args, size_t lds, uint64_t blocks, hipStream_t stream) {
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_tile_kernel<H, COPY, U8, FUSE>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((decode_tile_kernel<H, COPY, U8, FUSE>), dim3((uint32_t)blocks), dim3(kBlock), lds, stream,
                     args);
  return (int)hipGetLastError();
}

template <int H, bool COPY>
static int launch_decode_tile_u8(const DecodeArgs& args, size_t lds, uint64_t blocks, hipStream_t stream) {
  if (!args.valid) return launch_decode_tile<H, COPY, false>(args, lds, blocks, stream);
  // one pass for the sums and the check at 16 lanes a frame from 1 KiB payloads on
  // (at 512 B the ASCII frames' high-bit test costs more than the second read
  // saves: profiles/r06/sweeps/utf8_fused_ab.json)
  if (args.glog == 4u && (args.F - (uint32_t)H) / 16u >= 64u)
    return launch_decode_tile<H, COPY, true, true>(args, lds, blocks, stream);
  return launch_decode_tile<H, COPY, true>(args, lds, blocks, stream);
}

int launch_decode(const DecodeArgs& args, int layout, DecodePath path, hipStream_t stream) {
  if (args.n == 0) return 0;
  {
    const uint32_t per_block = kBlock >> args.glog;
    const uint64_t blocks = (args.n + per_block - 1) / per_block;
    if (path == DecodePath::kCopyTile || path == DecodePath::kVerifyTile) {
      size_t lds = ((size_t)per_block * args.F + 32 + 15) & ~size_t(15);
      if (args.stage_out) lds += (args.valid ? 9u : 8u) * per_block;  // staged outputs
      // Resident tiles per CU: verify-only wants every tile it can get; the
      // copy-out (read + write, like encode) runs best at 5 for tiles over
      // 14 KiB (1M x 1024 B 0.348 -> 0.340 ms, x 1472 B 0.518 -> 0.515; verify
      // at 5: 0.169 -> 0.209 ms; profiles/r01/sweeps/decode_percu.json).
      int per_cu = tuning().decode_blocks_per_cu;
      if (per_cu < 0) per_cu = (path == DecodePath::kCopyTile && (size_t)per_block * args.F > 14336u) ? 5 : 0;
      if (per_cu > 0) {
        const size_t want = ((size_t)(160 * 1024) / (size_t)per_cu) & ~size_t(15);
        if (want > lds) lds = want;
      }
      if (path == DecodePath::kCopyTile)
        return layout == 7 ? launch_decode_tile_u8<7, true>(args, lds, blocks, stream)
                           : launch_decode_tile_u8<5, true>(args, lds, blocks, stream);
      return layout == 7 ? launch_decode_tile_u8<7, false>(args, lds, blocks, stream)
                         : launch_decode_tile_u8<5, false>(args, lds, blocks, stream);
    }
    if (path == DecodePath::kVerify) {
      if (layout == 7)
        hipLaunchKernelGGL(decode_verify_kernel<7>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
      else
        hipLaunchKernelGGL(decode_verify_kernel<5>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
    } else if (layout == 7) {
      hipLaunchKernelGGL(decode_vec_kernel<7>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
    } else {
      hipLaunchKernelGGL(decode_vec_kernel<5>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
    }
  }
  return (int)hipGetLastError();
}

}  // namespace rudp
