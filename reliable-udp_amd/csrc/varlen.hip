// Variable-length batches and strict UTF-8 validation.
//
// The reference's real traffic is 5-9 byte frames: one character of UTF-8
// payload per datagram (utils/reliableUDP.py:11, :60).  A varlen batch is the
// header table plus len[N] (+ optional payload_off[N]) over one payload
// buffer.  Frame offsets are the exclusive scan of len[i] + H (scan.hip, a
// three-pass reduce-then-scan; hipcub in the tools build's sweeps), so the frames
// come out packed back to back exactly as N calls of Packet.to_byte() would
// be concatenated.
//
// Packed payloads (the common case) encode through LDS tiles of T packets
// (encode_varlen_tile_kernel; prebuilt header chunks and a one-window phase 2
// when every frame of the tile is >= 32 B); hints of 128 B and up decode and
// validate UTF-8 through LDS tiles of consecutive frames.  Otherwise vector
// kernels (16-byte aligned chunks, G lanes per packet from the caller's
// mean-length hint) when the buffers are 16-byte aligned, byte-granular
// kernels (8 lanes per packet) when not.  Numbers: DESIGN.md §3.
#include <map>
#include <mutex>
#include <vector>

#include "codec_device.hpp"
#include "internal.hpp"
#include "scan_device.hpp"
#include "utf8_device.hpp"
#if RUDP_TOOLS
#include <hipcub/hipcub.hpp>
#endif

namespace RUDP_NS {

constexpr uint32_t kVarLanes = 8;

// Sync-free calls: an earlier kernel of the call found the batch invalid.
// Uniform (a kernel argument), so this is one scalar load per wave.
__device__ __forceinline__ bool call_failed(const uint32_t* status) { return status && *status; }

// A batch's offsets: the frame_off array, or (FX) a fixed stride
// (VarlenArgs::stride, frame_off null).  A template argument, not a branch:
// the varlen kernels compile exactly as they did without the fixed-stride
// form (a runtime choice in the encode tile cost 1M x 1472 B 0.539 -> 0.570
// ms and ragged lengths 0.603 -> 0.690 in an A/B against the round-5 build,
// profiles/r06/sweeps/stride_template.json), and the FX instantiations read
// no offsets at all.
template <bool FX>
__device__ __forceinline__ uint64_t fo_at(const VarlenArgs& a, uint64_t p) {
  if (FX) return a.fo_base + p * a.stride;
  return a.frame_off[p];
}
template <int H, bool FX>
__device__ __forceinline__ uint32_t len_at(const VarlenArgs& a, uint64_t p) {
  if (FX) return (uint32_t)a.stride - (uint32_t)H;
  return a.len[p];
}
// Payload offset of packet p, whose frame starts at fo.
template <int H, bool FX>
__device__ __forceinline__ uint64_t po_at(const VarlenArgs& a, uint64_t p, uint64_t fo) {
  if (FX) return fo - p * (uint64_t)H + a.po_delta;
  return a.payload_off ? a.payload_off[p] : fo - p * (uint64_t)H;
}
// The byte-granular kernels (the diagnostics build's varlen_vec = 0 form) choose at run time.
__device__ __forceinline__ uint64_t fo_rt(const VarlenArgs& a, uint64_t p) {
  return a.frame_off ? fo_at<false>(a, p) : fo_at<true>(a, p);
}

#if RUDP_TOOLS
struct FrameLen {
  const uint32_t* len;
  uint32_t H;
  __host__ __device__ uint64_t operator()(uint64_t i) const { return (uint64_t)len[i] + H; }
};
#endif

template <int H>
__global__ void __launch_bounds__(kBlock) encode_varlen_kernel(VarlenArgs a) {
  if (call_failed(a.status)) return;
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid = p < a.n;
  uint32_t sum = 0;
  uint64_t fo = 0;
  if (valid) {
    const uint32_t L = a.frame_off ? len_at<H, false>(a, p) : len_at<H, true>(a, p);
    fo = fo_rt(a, p);
    const uint64_t po = a.frame_off ? po_at<H, false>(a, p, fo) : po_at<H, true>(a, p, fo);
    for (uint32_t j = g; j < L; j += kVarLanes) {
      const uint32_t b = a.payload[po + j];
      sum += (j & 1u) ? (b << 8) : b;  // LE u16 word sum (payload at an odd frame offset)
      a.frames[fo + H + j] = (unsigned char)b;
    }
  }
  for (uint32_t m = kVarLanes >> 1; m > 0; m >>= 1) sum += __shfl_xor(sum, (int)m, 64);
  if (valid) {
    const uint32_t s = a.seq_in[p], k = a.ack_in[p], f = a.flags_in[p];
    const uint32_t c = packet_csum(sum, s, k, f);
    const uint64_t h = pack_header<H>(s, k, f, c);
    for (uint32_t i = g; i < (uint32_t)H; i += kVarLanes) a.frames[fo + i] = (unsigned char)(h >> (8 * i));
    if (g == 0 && a.csum) a.csum[p] = (uint16_t)c;
  }
}

// 16 payload bytes starting at signed offset s; only aligned chunks that
// overlap the packet's own range [lo, hi) are loaded (others read as zero),
// so nothing outside the caller's payload is touched.
__device__ __forceinline__ u32x4 payload_window(const unsigned char* base, int64_t s, uint64_t lo,
                                                uint64_t hi) {
  const int64_t a0 = s & ~(int64_t)15;
  u32x4 x = {0u, 0u, 0u, 0u}, y = {0u, 0u, 0u, 0u};
  if (hi == lo) return x;
  if (a0 + 16 > (int64_t)lo && a0 < (int64_t)hi) x = *reinterpret_cast<const u32x4*>(base + a0);
  if (a0 + 32 > (int64_t)lo && a0 + 16 < (int64_t)hi) y = *reinterpret_cast<const u32x4*>(base + a0 + 16);
  return funnel32(x, y, (uint32_t)(s & 15));
}

// The payload bytes of one aligned 16-byte output chunk of frame
// [fo, fo + F), from a funnel-shifted input window; other bytes zero.
// k0 = X - fo (>= -15) is the frame position of chunk byte 0.
template <int H>
__device__ __forceinline__ void frame_chunk(const unsigned char* payload, uint64_t po, uint64_t pend,
                                            int k0, uint32_t F, uint64_t* lo, uint64_t* hi) {
  const u32x4 w = payload_window(payload, (int64_t)po + k0 - H, po, pend);
  *lo = lo64(w) & byte_mask(H - k0, (int)F - k0);
  *hi = hi64(w) & byte_mask(H - k0 - 8, (int)F - k0 - 8);
}

// LE16 word sum of the bytes of a 16-byte chunk (lo, hi), where chunk byte b
// is payload index j = j0 + b; even j are low bytes.
__device__ __forceinline__ uint32_t payload_le16_sum(uint64_t lo, uint64_t hi, int j0) {
  const uint64_t ev = (lo & 0x00FF00FF00FF00FFull) + (hi & 0x00FF00FF00FF00FFull);
  const uint64_t od = ((lo >> 8) & 0x00FF00FF00FF00FFull) + ((hi >> 8) & 0x00FF00FF00FF00FFull);
  const uint32_t e = (uint32_t)((ev & 0xFFFF) + ((ev >> 16) & 0xFFFF) + ((ev >> 32) & 0xFFFF) + (ev >> 48));
  const uint32_t o = (uint32_t)((od & 0xFFFF) + ((od >> 16) & 0xFFFF) + ((od >> 32) & 0xFFFF) + (od >> 48));
  return (j0 & 1) ? ((e << 8) + o) : (e + (o << 8));
}

__device__ __forceinline__ void store_owned(unsigned char* dst, int b_lo, int b_hi, uint64_t lo,
                                            uint64_t hi) {
  if (b_lo == 0 && b_hi == 16) {
    *reinterpret_cast<u32x4*>(dst) = make_u32x4(lo, hi);
  } else {
    for (int b = b_lo; b < b_hi; ++b)
      dst[b] = (unsigned char)(b < 8 ? lo >> (8 * b) : hi >> (8 * (b - 8)));
  }
}

// Vectorized varlen encode (payload and frames buffers 16-byte aligned), one
// pass: G lanes per packet walk the aligned 16-byte chunks of the frame
// [fo, fo+F).  Each chunk's payload bytes come from a funnel-shifted window of
// the input (two aligned loads shared with the neighbour lanes, so every
// payload byte leaves HBM once), are summed into the packet's LE16 sum
// (payload byte j is a low byte iff j is even; j = k - H for frame position
// k) and are stored at once: interior chunks as one dwordx4 store, the two
// chunks shared with neighbour frames bytewise.  Only the one or two chunks
// holding header bytes wait for the group's sum; they are rebuilt and
// written after the shfl reduction.
// G = 2^glog lanes (g = 0..G-1, one aligned group of a wave) encode packet p.
// fo_in: the frame's offset when the caller already has it (~0: read frame_off).
template <int H, bool FX = false>
__device__ __forceinline__ void encode_varlen_packet(const VarlenArgs& a, uint64_t p, bool valid, uint32_t g,
                                                     uint32_t glog, uint64_t fo_in = ~0ull) {
  const uint32_t G = 1u << glog;
  const uint32_t L = valid ? len_at<H, FX>(a, p) : 0u;
  const uint64_t fo = valid ? (fo_in != ~0ull ? fo_in : fo_at<FX>(a, p)) : 0;
  const uint64_t po = valid ? po_at<H, FX>(a, p, fo) : 0;
  const uint64_t pend = po + L;
  const uint32_t F = L + H;
  const uint64_t x_lo = fo >> 4;
  const uint32_t nout = valid ? (uint32_t)(((fo + F - 1) >> 4) - x_lo + 1) : 0u;
  // chunks 0 .. nhdr-1 hold header bytes (frame positions < H)
  const uint32_t nhdr = (uint32_t)(((fo + H - 1) >> 4) - x_lo + 1);

  uint32_t sum = 0;
  // Rounds of U chunks per lane: all 2U window loads are issued before any
  // store (the compiler cannot move loads across stores to `frames`).
  constexpr uint32_t U = 4;
  for (uint32_t i0 = g; i0 < nout; i0 += U * G) {
    u32x4 wx[U], wy[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * G;
      wx[u] = make_u32x4(0ull, 0ull);
      wy[u] = make_u32x4(0ull, 0ull);
      if (i < nout && i >= nhdr) {
        const int64_t s0 = (int64_t)po + ((int64_t)((x_lo + i) << 4) - (int64_t)fo) - H;
        const int64_t a0 = s0 & ~(int64_t)15;
        if (a0 + 16 > (int64_t)po && a0 < (int64_t)pend)
          wx[u] = *reinterpret_cast<const u32x4*>(a.payload + a0);
        if (a0 + 32 > (int64_t)po && a0 + 16 < (int64_t)pend)
          wy[u] = *reinterpret_cast<const u32x4*>(a.payload + a0 + 16);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * G;
      if (i < nout && i >= nhdr) {
        const uint64_t X = (x_lo + i) << 4;
        const int k0 = (int)((int64_t)X - (int64_t)fo);  // >= H here: no header bytes
        const u32x4 w = funnel32(wx[u], wy[u], (uint32_t)((po + (uint64_t)k0 - H) & 15u));
        const uint64_t lo = lo64(w) & byte_mask(H - k0, (int)F - k0);
        const uint64_t hi = hi64(w) & byte_mask(H - k0 - 8, (int)F - k0 - 8);
        store_owned(a.frames + X, 0, (int)F - k0 < 16 ? (int)F - k0 : 16, lo, hi);
        sum += payload_le16_sum(lo, hi, k0 - H);
      }
    }
  }
  // Header chunks: their payload bytes now, the header once the sum is known.
  uint64_t hlo[2] = {0ull, 0ull}, hhi[2] = {0ull, 0ull};
#pragma unroll
  for (uint32_t i = 0; i < 2; ++i) {
    if (i < nhdr && (i & (G - 1u)) == g && valid) {
      const int k0 = (int)((int64_t)((x_lo + i) << 4) - (int64_t)fo);
      frame_chunk<H>(a.payload, po, pend, k0, F, &hlo[i], &hhi[i]);
      sum += payload_le16_sum(hlo[i], hhi[i], k0 - H);
    }
  }
  sum = group_sum(sum, G);
  if (!valid) return;
  const uint32_t s = a.seq_in[p], k = a.ack_in[p], f = a.flags_in[p];
  const uint32_t c = packet_csum(sum, s, k, f);
  if (g == 0 && a.csum) a.csum[p] = (uint16_t)c;
  const uint64_t h = pack_header<H>(s, k, f, c);
#pragma unroll
  for (uint32_t i = 0; i < 2; ++i) {
    if (i < nhdr && (i & (G - 1u)) == g) {
      const uint64_t X = (x_lo + i) << 4;
      const int k0 = (int)((int64_t)X - (int64_t)fo);
      uint64_t lo = hlo[i], hi = hhi[i];
      if (k0 >= 0) {
        lo |= h >> (8 * k0);
      } else {
        const int sh = -k0;  // 1..15: the frame starts sh bytes into the chunk
        if (sh < 8) {
          lo |= h << (8 * sh);
          hi |= h >> (64 - 8 * sh);
        } else {
          hi |= h << (8 * (sh - 8));
        }
      }
      store_owned(a.frames + X, k0 < 0 ? -k0 : 0, (int)F - k0 < 16 ? (int)F - k0 : 16, lo, hi);
    }
  }
}

template <int H, bool FX = false>
__global__ void __launch_bounds__(kBlock) encode_varlen_vec_kernel(VarlenArgs a) {
  if (call_failed(a.status)) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog;
  const uint64_t p = (uint64_t)blockIdx.x * (kBlock >> glog) + (tid >> glog);
  encode_varlen_packet<H, FX>(a, p, p < a.n, tid & ((1u << glog) - 1u), glog);
}

// LDS layout of the varlen encode tile: header words u64[T], tile-relative
// frame offsets u32[T + 1], the chunk -> frame map u8[] or u16[], the
// block-sum pass's u32 sums of the run's 128-B blocks, then the payload run
// (guard, cap bytes, guard).  Shared by the launcher (LDS size) and the kernel.
constexpr uint32_t kVTGuard = 32;
// The map holds one u8 (owner frame) per output chunk, or with the coded map
// (vhc == 2) one u16: owner frame in bits 0-7, bit 15 = pure payload chunk,
// else bit 8 = header chunk of the next frame and bit 9 = its slot; bit 14 =
// the chunk touches a header of a frame under kVHCMinFrame bytes, which has
// no prebuilt chunks: phase 2 walks its frames.
__host__ __device__ inline uint32_t vt_map_bytes(uint32_t T, uint32_t cap, uint32_t H, uint32_t wide) {
  return (((cap + T * H) >> 4) + 4u) << (wide ? 1 : 0);
}
// Frames of at least this many bytes: an aligned 16-B chunk overlaps at most
// one header, and the 16 payload bytes before a frame's payload belong to the
// previous frame (the varlen tile's fast phase 2).
constexpr uint32_t kVHCMinFrame = 32;

// the block sums: one u32 per 128 B of run (own region, so the map can be
// built while other packets' lanes still read them)
__host__ __device__ inline uint32_t vt_blk_bytes(uint32_t cap) { return ((cap >> 7) + 4u) * 4u; }
__host__ __device__ inline uint32_t vt_blk_off(uint32_t T, uint32_t cap, uint32_t H, uint32_t wide) {
  return (8u * T + 4u * (T + 1u) + vt_map_bytes(T, cap, H, wide) + 3u) & ~3u;
}
__host__ __device__ inline uint32_t vt_pay_off(uint32_t T, uint32_t cap, uint32_t H, uint32_t wide) {
  return (vt_blk_off(T, cap, H, wide) + vt_blk_bytes(cap) + 15u) & ~15u;
}

// The block-sum pass (tile_sums 2).  Summing a packet's payload chunk by
// chunk out of LDS gives its G lanes work in proportion to its length, so a
// tile of ragged lengths waits for its longest packet.  Instead every 128-B
// block of the run gets its even- and odd-address byte sums as phase 1
// streams it through registers (8 lanes hold the block's 8 vectors), and a
// packet's G lanes add the block sums inside its payload plus the 16 chunks
// of its two edge blocks, masked: one LDS read per 128 payload bytes instead
// of 8.
// Even/odd byte sums of a 16-B chunk, packed e | o << 16 (each at most 2040).
__device__ __forceinline__ uint32_t eo_sum(uint64_t lo, uint64_t hi) {
  const u32x4 w = make_u32x4(lo, hi);  // (each at most 8 * 255: packs into 16 bits)
  return even_bytes(w) | (odd_bytes(w) << 16);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
// Sum over 8 consecutive lanes (all 8 active).
__device__ __forceinline__ uint32_t octet_sum(uint32_t x) {
  x += dpp_u32<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_u32<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_u32<0x141>(x);  // row_half_mirror: the other quad of the 8
  return x;
}

// Varlen encode of a PACKED payload buffer (payload_off == null) through an
// LDS tile: the same shape as the fixed-length encode_tile_kernel (encode.hip)
// with per-frame bounds from frame_off.  A workgroup owns packets
// [p0, p0 + T): their payloads are one contiguous input run
// [fo[p0] - p0*H, fo[p0+T] - (p0+T)*H) and their frames one contiguous output
// run [fo[p0], fo[p0+T]).
//   phase 1  the run's aligned 16-B vectors stream into LDS like a copy;
//            the tile's frame offsets go to LDS.
//   sums     G lanes per packet read the packet's aligned LDS chunks, mask the
//            two edge chunks to the payload and sum LE16 words by address
//            parity; the group leader writes the header word.  The same lanes
//            fill the map from each output chunk to the frame holding its
//            first byte.
//   phase 2  output-stationary: each lane owns aligned 16-B output chunks and
//            ORs in every frame the chunk touches (one or two for MTU frames, up
//            to four for header-only ones): header bytes from the header word,
//            payload bytes from a byte-shifted LDS window.  The chunks shared
//            with the neighbour tiles are written bytewise.
// A tile whose run exceeds tile_cap (lengths far above the caller's hint)
// encodes its packets with the per-packet vector path instead.
// Byte tiles (chosen by the scan per call, when enough packet tiles would
// overflow): a workgroup frames the packets whose payload starts in one span
// of S payload bytes instead, their lanes per packet from their count.  The
// grid covers both forms; a tile learns its packets from the scan's records.
// W: minimum waves per SIMD the register allocation must allow (1 = none).
template <int H, int W, bool FX = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W))) encode_varlen_tile_kernel(VarlenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t Tl = a.tile_Tl, cap = a.tile_cap;
  uint64_t* lds_hdr = reinterpret_cast<uint64_t*>(lds);
  uint32_t* lds_fo = reinterpret_cast<uint32_t*>(lds + 8u * Tl);
  const bool wide = a.vhc == 2u;  // coded chunk map (u16 entries)
  const bool blk_sums = a.tile_sums == 2u;  // the block-sum pass
  uint8_t* lds_map = reinterpret_cast<uint8_t*>(lds_fo + Tl + 1u);
  uint16_t* lds_map16 = reinterpret_cast<uint16_t*>(lds_map);
  uint32_t* lds_blk = reinterpret_cast<uint32_t*>(lds + vt_blk_off(Tl, cap, H, wide ? 1u : 0u));
  unsigned char* lds_pay = lds + vt_pay_off(Tl, cap, H, wide ? 1u : 0u);

  const uint32_t tid = threadIdx.x;
#if RUDP_TOOLS
  const uint64_t t_start = a.trace ? (uint64_t)wall_clock64() : 0ull;  // diagnostics: tile phases
  uint64_t t_loaded = 0, t_summed = 0, t_mapped = 0;
  __shared__ unsigned long long s_last[3];  // latest wave: sums, map, header chunks done
  if (a.trace && tid < 3u) s_last[tid] = 0ull;
#endif
  // Tile records (checked calls, a.span_rec): the scan chose the form for
  // the whole call and wrote one record {frame_off[p], p} per workgroup for
  // its first packet, so a tile's first loads are its two adjacent records
  // whatever the form -- packet tiles of tile_T packets or byte tiles (the
  // packets whose payload starts in one span of S bytes); the workgroups the
  // chosen form does not need hold empty records spread over the grid.
  // Unchecked calls: packet tiles from frame_off directly.
  const uint32_t b = blockIdx.x;
  uint64_t p0, fo0, fo_end;
  uint32_t Tv, Tall, T, glog;
  if (a.span_rec) {
    const uint32_t t = a.xcd ? xcd_tile(b, gridDim.x) : b;
    const SpanRec r0 = a.span_rec[t], r1 = a.span_rec[t + 1];
    // (clamped, so a rejected batch's records stay in range)
    p0 = r0.p < a.n ? r0.p : a.n;
    const uint64_t p1 = r1.p < a.n ? (r1.p > p0 ? r1.p : p0) : a.n;
    Tall = (uint32_t)(p1 - p0);
    if (Tall == 0) return;
    T = a.bt_slots;
    Tv = Tall < T ? Tall : T;
    fo0 = r0.fo;
    fo_end = r1.fo;  // frame_off[p0 + Tv] when Tall <= T (else the per-packet path)
    // lanes per packet: as many as the tile's packet count leaves
    glog = 0;
    while (glog < 6u && (Tv << (glog + 1u)) <= kBlock) ++glog;
  } else {
    const uint32_t ptiles = (uint32_t)((a.n + a.tile_T - 1u) / a.tile_T);
    if (b >= ptiles) return;
    p0 = (uint64_t)(a.xcd ? xcd_tile(b, ptiles) : b) * a.tile_T;
    T = a.tile_T;
    Tv = Tall = a.n - p0 < a.tile_T ? (uint32_t)(a.n - p0) : a.tile_T;
    fo0 = fo_at<FX>(a, p0);
    fo_end = fo_at<FX>(a, p0 + Tv);
    glog = a.tile_glog;
  }
  const uint32_t G = 1u << glog, q = tid >> glog, g = tid & (G - 1u);
  // Header-table loads before phase 1: their latency overlaps its stream
  // instead of following the barrier.
  uint32_t t_seq = 0, t_ack = 0, t_flags = 0;
  if (a.early_table && g < 2u && q < Tv) {  // (lanes 0 and 1 each build a header chunk)
    t_seq = a.seq_in[p0 + q];
    t_ack = a.ack_in[p0 + q];
    t_flags = a.flags_in[p0 + q];
  }
  if (call_failed(a.status)) return;
  const uint64_t po0 = fo0 - p0 * (uint64_t)H + (FX ? a.po_delta : 0ull);
  const uint64_t po_end = fo_end - (p0 + Tv) * (uint64_t)H + (FX ? a.po_delta : 0ull);
  const uint64_t A = po0 & ~15ull;
  const uint64_t run = ((po_end + 15u) & ~15ull) - A;
  if (Tall > T || run > cap) {  // uniform over the workgroup
    for (uint32_t q0 = 0; q0 < Tall; q0 += kBlock >> glog)  // (byte tiles may hold more than T packets)
      encode_varlen_packet<H, FX>(a, p0 + q0 + q, q0 + q < Tall, g, glog);
    return;
  }
  const bool early_tab = a.early_table;

  // ---- phase 1: payload run -> LDS, frame offsets ------------------------
  {
    // The tile's T + 1 frame offsets (at most two per lane): issued before the
    // payload stream so their round trip overlaps it (early_fo).
    uint32_t fo_r0 = 0, fo_r1 = 0;
    if (a.early_fo) {
      if (tid <= Tv) fo_r0 = (uint32_t)(fo_at<FX>(a, p0 + tid) - fo0);
      if (tid + kBlock <= Tv) fo_r1 = (uint32_t)(fo_at<FX>(a, p0 + tid + kBlock) - fo0);
    }
    const u32x4* src = reinterpret_cast<const u32x4*>(a.payload + A);
    u32x4* dst = reinterpret_cast<u32x4*>(lds_pay + kVTGuard);
    const uint32_t nvec = (uint32_t)(run >> 4);
    constexpr uint32_t P = 8;
    for (uint32_t v0 = tid; v0 < nvec; v0 += P * kBlock) {
      u32x4 r[P];
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * kBlock;
        if (v < nvec) r[u] = __builtin_nontemporal_load(src + v);
      }
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * kBlock;
        if (v < nvec) dst[v] = r[u];
        // block sums from the registers: whole 128-B blocks only (uniform
        // per 8 lanes; the run's partial last block is never inside a
        // packet's payload, only its edge)
        if (blk_sums && (v | 7u) < nvec) {
          const uint32_t eo = octet_sum(eo_sum(lo64(r[u]), hi64(r[u])));
          if ((tid & 7u) == 0) lds_blk[v >> 3] = eo;  // (e, o at most 16320 each)
        }
      }
    }
    if (a.early_fo) {
      if (tid <= Tv) lds_fo[tid] = fo_r0;
      if (tid + kBlock <= Tv) lds_fo[tid + kBlock] = fo_r1;
    } else {
      for (uint32_t i = tid; i <= Tv; i += kBlock) lds_fo[i] = (uint32_t)(fo_at<FX>(a, p0 + i) - fo0);
    }
  }
  __syncthreads();
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_loaded = (uint64_t)wall_clock64();
#endif

  // ---- per-packet sums, header words, chunk -> frame map ------------------
  const uint32_t shift = kVTGuard + (uint32_t)(po0 & 15u);  // LDS offset of payload byte po0
  const uint32_t nbytes = (uint32_t)(fo_end - fo0);
  const uint32_t lead = (uint32_t)(-(uintptr_t)(a.frames + fo0)) & 15u;
  uint32_t sum = 0;
  if (q < Tv) {
    const uint32_t fs = lds_fo[q], fe = lds_fo[q + 1];
    const uint32_t Lq = fe - fs - H;
    const uint32_t d = shift + fs - q * H;  // LDS offset of the packet's first payload byte
    if (Lq) {
      if (blk_sums) {
        // the 16 chunks of the blocks holding the payload's first and last
        // bytes (each masked to the payload), then the block sums between
        const u32x4* run16 = reinterpret_cast<const u32x4*>(lds_pay + kVTGuard);
        const uint32_t x0 = d - kVTGuard, x1 = x0 + Lq;  // run offsets
        const uint32_t j0 = x0 >> 7, j1 = (x1 - 1u) >> 7;
        uint32_t e = 0, o = 0;
        for (uint32_t c = g; c < 16u; c += G) {
          const uint32_t cx = ((c < 8u ? j0 : j1) << 7) + ((c & 7u) << 4);
          if ((c < 8u || j1 != j0) && cx < x1 && cx + 16u > x0) {  // (no reads past the run)
            const u32x4 w = run16[cx >> 4];
            const int lo = (int)x0 - (int)cx, hi = (int)x1 - (int)cx;
            const uint32_t eo = eo_sum(lo64(w) & byte_mask(lo, hi), hi64(w) & byte_mask(lo - 8, hi - 8));
            e += eo & 0xFFFFu;
            o += eo >> 16;
          }
        }
        for (uint32_t j = j0 + 1u + g; j < j1; j += G) {
          const uint32_t bs = lds_blk[j];
          e += bs & 0xFFFFu;
          o += bs >> 16;
        }
        sum = (d & 1u) ? (e << 8) + o : e + (o << 8);  // payload byte x - d is a low byte when even
      } else {
        const u32x4* pay16 = reinterpret_cast<const u32x4*>(lds_pay);
        const uint32_t c1 = (d + Lq - 1u) >> 4;
        for (uint32_t c = (d >> 4) + g; c <= c1; c += G) {
          const u32x4 v = pay16[c];
          const int rel = (int)(c << 4) - (int)d;  // payload index of chunk byte 0
          const uint64_t lo = lo64(v) & byte_mask(-rel, (int)Lq - rel);
          const uint64_t hi = hi64(v) & byte_mask(-rel - 8, (int)Lq - rel - 8);
          sum += payload_le16_sum(lo, hi, rel);
        }
      }
    }
  }
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_summed = (uint64_t)wall_clock64();  // (thread 0's own sums done)
  if (a.trace && (tid & 63u) == 0) atomicMax(&s_last[0], (unsigned long long)wall_clock64());
#endif
  // The map, in the same pass (the block sums have their own LDS region).
  // map[k] = the frame r whose bytes [fs, fe) hold output unit k's first byte
  // lead + 16k; with the coded map also the chunk's class for the fast phase
  // 2: pure payload of r, or one of the prebuilt header chunks of r (chunk
  // starts in r's header) or r + 1 -- which exist only for frames of
  // kVHCMinFrame bytes and up: a chunk over a shorter frame's header is left
  // to the frame walk (bit 14).
  auto map_entry = [&](uint32_t k, uint32_t r, uint32_t fs, uint32_t fe) {
    if (!wide) {
      lds_map[k] = (uint8_t)r;
      return;
    }
    const uint32_t x = lead + 16u * k;
    const int k0 = (int)x - (int)fs;
    uint32_t e = r;
    if (k0 >= H && x + 16u <= fe) {
      e |= 0x8000u;
    } else {
      const uint32_t nxt = k0 >= H ? 1u : 0u;
      const uint32_t fsp = nxt ? fe : fs;
      const int i0 = fsp >= lead ? (int)((fsp - lead) >> 4) : -1;
      e |= (nxt << 8) | ((uint32_t)((int)k - i0) & 1u) << 9;
      const uint32_t hlen = nxt ? (r + 1u < Tv ? lds_fo[r + 2u] - fe : 0u) : fe - fs;
      if (hlen < kVHCMinFrame) e |= 0x4000u;
    }
    lds_map16[k] = (uint16_t)e;
  };
  if (RUDP_TOOLS && a.map_bal) {  // (measured slower at equal lengths: diagnostics build only)
    // by units: lane tid takes units [tid kc, (tid + 1) kc) whatever frames
    // they fall in, so a tile of ragged lengths does not wait for its longest
    // frame's G lanes (a frame's units are its length / 16)
    const uint32_t K = nbytes > lead ? (nbytes - lead + 15u) >> 4 : 0u;
    const uint32_t kc = K / kBlock + 1u;
    uint32_t k = tid * kc;
    const uint32_t kend = k + kc < K ? k + kc : K;
    if (k < kend) {
      uint32_t x = lead + 16u * k;
      uint32_t lo = 0, hi = Tv - 1u;  // the first frame ending past x
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lds_fo[mid + 1u] > x) hi = mid;
        else lo = mid + 1u;
      }
      uint32_t r = lo, fs = lds_fo[r], fe = lds_fo[r + 1u];
      for (; k < kend; ++k, x += 16u) {
        while (x >= fe) {
          ++r;
          fs = fe;
          fe = lds_fo[r + 1u];
        }
        map_entry(k, r, fs, fe);
      }
    }
  } else if (q < Tv) {
    // (the class test hoisted out of the loop, as round 3 had it: through
    // map_entry, ragged lengths ran 0.607 -> 0.632 ms, profiles/r05/sweeps/
    // varlen_encode_bisect.json)
    const uint32_t fs = lds_fo[q], fe = lds_fo[q + 1];
    const uint32_t klo = fs > lead ? (fs - lead + 15u) >> 4 : 0u;
    const uint32_t khi = fe > lead ? (fe - lead + 15u) >> 4 : 0u;
    if (wide) {
      for (uint32_t k = klo + g; k < khi; k += G) {
        const uint32_t x = lead + 16u * k;
        const int k0 = (int)x - (int)fs;
        uint32_t e = q;
        if (k0 >= H && x + 16u <= fe) {
          e |= 0x8000u;
        } else {
          const uint32_t nxt = k0 >= H ? 1u : 0u;
          const uint32_t fsp = nxt ? fe : fs;
          const int i0 = fsp >= lead ? (int)((fsp - lead) >> 4) : -1;
          e |= (nxt << 8) | ((uint32_t)((int)k - i0) & 1u) << 9;
          const uint32_t hlen = nxt ? (q + 1u < Tv ? lds_fo[q + 2u] - fe : 0u) : fe - fs;
          if (hlen < kVHCMinFrame) e |= 0x4000u;
        }
        lds_map16[k] = (uint16_t)e;
      }
    } else {
      for (uint32_t k = klo + g; k < khi; k += G) lds_map[k] = (uint8_t)q;
    }
  }
#if RUDP_TOOLS
  if (a.trace && (tid & 63u) == 0) atomicMax(&s_last[1], (unsigned long long)wall_clock64());
#endif
  sum = group_sum(sum, G);
  // The header word and the frame's (up to) two header chunks: lanes 0 and 1
  // of the packet build one chunk each (the leader both when G = 1).
  const uint32_t hl = G >= 2u ? 2u : 1u;
  if (g < hl && q < Tv) {
    const uint64_t p = p0 + q;
    const bool late = !early_tab;
    const uint32_t s = late ? a.seq_in[p] : t_seq, k = late ? a.ack_in[p] : t_ack,
                   f = late ? a.flags_in[p] : t_flags;
    const uint32_t c = packet_csum(sum, s, k, f);
    const uint64_t hw = pack_header<H>(s, k, f, c);
    if (g == 0) {
      lds_hdr[q] = hw;
      if (a.csum) a.csum[p] = (uint16_t)c;
    }
    const uint32_t fs = lds_fo[q], fe = lds_fo[q + 1];
    if (a.vhc && fe - fs >= kVHCMinFrame) {
      // This frame's header chunks (the full output chunks over [fs, fs + H))
      // for phase 2's fast path.  Payloads are contiguous in LDS: the bytes of
      // a slot-0 chunk before fs are the last payload bytes before this
      // frame's (the map sends a chunk here only when they are the previous
      // frame's payload, never its header).
      const uint32_t d = shift + fs - q * H;
      const u32x4 tail = window16_dw(reinterpret_cast<const uint32_t*>(lds_pay), d - 16u);
      const u32x4 head = window16_dw(reinterpret_cast<const uint32_t*>(lds_pay), d);
      const int i0 = fs >= lead ? (int)((fs - lead) >> 4) : -1;
      u32x4* hc = reinterpret_cast<u32x4*>(lds + a.hc_off) + 2u * q;
      for (uint32_t sl = g; sl < 2u; sl += hl) {
        const int i = i0 + (int)sl;
        const int X = (int)lead + 16 * i;
        if (X >= (int)(fs + H)) break;
        if (i >= 0 && (uint32_t)i < (nbytes > lead ? (nbytes - lead) >> 4 : 0u))
          hc[sl] = header_chunk<H>((uint64_t)X, (uint64_t)(fs + H), hw, tail, head);
      }
    }
  }
#if RUDP_TOOLS
  if (a.trace) atomicMax(&s_last[2], (unsigned long long)wall_clock64());  // (after its lanes' stores)
#endif
  // u8 map: the fast phase 2 when every frame of the tile is at least
  // kVHCMinFrame bytes (then a chunk overlaps at most one header); the coded
  // map decides chunk by chunk.
  const bool vfast = __syncthreads_and(q >= Tv || lds_fo[q + 1] - lds_fo[q] >= kVHCMinFrame) && a.vhc;
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_mapped = (uint64_t)wall_clock64();
#endif

  // ---- phase 2: aligned 16-B output chunks ---------------------------------
  unsigned char* out = a.frames + fo0;
  const uint32_t nfull = nbytes > lead ? (nbytes - lead) >> 4 : 0u;
  // full chunks dealt from the first 64-B boundary on (whole sectors per wave store)
  uint32_t npre = a.align64 ? ((uint32_t)(-reinterpret_cast<uintptr_t>(out)) & 63u) >> 4 : 0u;
  if (npre > nfull) npre = nfull;
  const uint32_t* pay_dw = reinterpret_cast<const uint32_t*>(lds_pay);
  // unit k < nfull: full chunk i = (k + npre) mod nfull at tile offset
  // lead + 16i; then the partial head [0, lead) and tail [lead + 16*nfull,
  // nbytes), written bytewise.
  for (uint32_t k = tid; k < nfull + 2u; k += kBlock) {
#if RUDP_TOOLS
    if ((a.diag & 1u) && k >= nfull) continue;  // ablation: the edge units not stored
#endif
    uint32_t x, hi_b, r;
    if (k < nfull) {
      const uint32_t i = k + npre < nfull ? k + npre : k + npre - nfull;
      x = lead + 16u * i; hi_b = 16u;
      if (wide) {
        const uint32_t e = lds_map16[i];
        if (!(e & 0x4000u)) {
          // pure payload: one LDS window at shift + x - (r + 1) H; otherwise a
          // prebuilt header chunk, no frame offsets needed
          const uint32_t rr = e & 0xFFu;
          u32x4 v;
          if (e & 0x8000u)
            v = window16_dw(pay_dw, shift + x - (rr + 1u) * (uint32_t)H);
          else
            v = reinterpret_cast<const u32x4*>(lds + a.hc_off)[2u * (rr + ((e >> 8) & 1u)) + ((e >> 9) & 1u)];
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + x));
          continue;
        }
        r = e & 0xFFu;
      } else {
        r = lds_map[i];
      }
    } else if (k == nfull) {
      x = 0; hi_b = lead < nbytes ? lead : nbytes; r = 0;
    } else {
      x = lead + 16u * nfull; hi_b = nbytes > x ? nbytes - x : 0u;
      r = hi_b ? (wide ? (lds_map16[nfull] & 0xFFu) : lds_map[nfull]) : 0u;
    }
    if (hi_b == 0) continue;
    if (vfast && k < nfull) {
      // pure payload of frame r: one LDS window; otherwise the prebuilt
      // header chunk of frame r (its own header) or r + 1
      const uint32_t fs = lds_fo[r], fe = lds_fo[r + 1];
      const int k0 = (int)x - (int)fs;
      u32x4 v;
      if (k0 >= H && (uint32_t)k0 + 16u <= fe - fs) {
        v = window16_dw(pay_dw, shift + fs - r * H + (uint32_t)k0 - H);
      } else {
        const uint32_t ph = k0 < H ? r : r + 1u;
        const uint32_t fsp = k0 < H ? fs : fe;
        const int i0 = fsp >= lead ? (int)((fsp - lead) >> 4) : -1;
        v = reinterpret_cast<const u32x4*>(lds + a.hc_off)[2u * ph + (uint32_t)((int)((x - lead) >> 4) - i0)];
      }
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + x));
      continue;
    }
    uint64_t lo = 0, hi = 0;
    // frames r, r+1, ... are back to back: each one starts where the last ended
    for (uint32_t fs = lds_fo[r < Tv ? r : 0]; r < Tv; ++r) {
      const uint32_t fe = lds_fo[r + 1];
      const int F = (int)(fe - fs);
      const int k0 = (int)x - (int)fs;  // frame position of chunk byte 0 (> -16)
      if (k0 < H) {
        const uint64_t h = lds_hdr[r];
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
      }
      if (F > H && k0 + 16 > H && k0 < F) {
        const uint32_t d = shift + fs - r * H;  // LDS offset of payload byte 0 of frame r
        const u32x4 w = window16_dw(pay_dw, (uint32_t)((int)d + k0 - H));
        lo |= lo64(w) & byte_mask(H - k0, F - k0);
        hi |= hi64(w) & byte_mask(H - k0 - 8, F - k0 - 8);
      }
      if (fe >= x + 16u) break;
      fs = fe;
    }
    if (hi_b == 16u) {
      __builtin_nontemporal_store(make_u32x4(lo, hi), reinterpret_cast<u32x4*>(out + x));
    } else {
      for (uint32_t b = 0; b < hi_b; ++b)
        out[x + b] = (unsigned char)(b < 8 ? lo >> (8 * b) : hi >> (8 * (b - 8)));
    }
  }
#if RUDP_TOOLS
  if (a.trace) {  // diagnostics: {start, loaded, summed, mapped, end, XCC, Tv | records << 16 | vfast << 17, bytes,
                  //               latest wave's sums, map, header chunks done, 0}
    __syncthreads();
    if (tid == 0) {
      u32x4* rec = reinterpret_cast<u32x4*>(a.trace + 12ull * blockIdx.x);
      rec[0] = make_u32x4(t_start, t_loaded);
      rec[1] = make_u32x4(t_summed, t_mapped);
      rec[2] = make_u32x4((uint64_t)wall_clock64(), __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20));
      rec[3] = make_u32x4((uint64_t)Tv | (a.span_rec ? 1ull << 16 : 0ull) | (vfast ? 1ull << 17 : 0ull), (uint64_t)nbytes);
      rec[4] = make_u32x4(s_last[0], s_last[1]);
      rec[5] = make_u32x4(s_last[2], 0ull);
    }
  }
#endif
}

// Byte limit of a decode's frames: the caller's buffer size for checked
// calls, else (unchecked callers) the last offset.
template <bool FX = false>
__device__ __forceinline__ uint64_t frames_limit(const VarlenArgs& a) {
  return a.lim_checked ? a.frames_lim : fo_at<FX>(a, a.n);
}

// A frame whose offsets are invalid: no byte of it is read.
__device__ __forceinline__ void decode_varlen_reject(const VarlenArgs& a, uint64_t p) {
  a.seq[p] = 0;
  a.ack[p] = 0;
  a.flags[p] = 0;
  a.ok[p] = RUDP_OK_BAD_OFFSETS;
  if (a.csum_out) a.csum_out[p] = 0;
  if (a.valid) a.valid[p] = 0;  // nothing of it was read, so nothing is vouched for
  if (a.status_out) atomicOr(a.status_out, RUDP_ST_OFFSETS);
}

// U8: the payload's strict UTF-8 check in the same pass (a.valid).  Here the
// lanes judge contiguous slices of the payload (utf8_slice), byte-granular as
// the sum loop is.
template <int H, bool U8>
__global__ void __launch_bounds__(kBlock) decode_varlen_kernel(VarlenArgs a) {
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid = p < a.n;
  uint64_t acc = 0, F = 0;  // (frames of any length: the sum is folded before the lanes add)
  uint64_t fo = 0;
  bool bad = false;
  if (valid) {
    fo = fo_rt(a, p);
    const uint64_t fe = fo_rt(a, p + 1);
    bad = fo > fe || fe > (a.lim_checked ? a.frames_lim : fo_rt(a, a.n));
    F = bad ? 0u : fe - fo;
    for (uint64_t j = (uint64_t)H + g; j < F; j += kVarLanes) {
      const uint32_t b = a.frames[fo + j];
      acc += ((j - H) & 1u) ? (b << 8) : b;
    }
  }
  uint32_t sum = fold_keep(acc);
  uint32_t u8bad = 0;
  if (U8) {
    if (valid && F > (uint32_t)H) u8bad = utf8_slice(a.frames, fo + H, F - H, g, kVarLanes);
    for (uint32_t m = kVarLanes >> 1; m > 0; m >>= 1) u8bad |= __shfl_xor(u8bad, (int)m, 64);
  }
  for (uint32_t m = kVarLanes >> 1; m > 0; m >>= 1) sum += __shfl_xor(sum, (int)m, 64);
  if (valid && g == 0) {
    if (bad) {
      decode_varlen_reject(a, p);
      return;
    }
    if (U8) a.valid[p] = u8bad ? 0 : 1;
    uint32_t b[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < 7; ++i)
      if (i < F) b[i] = a.frames[fo + i];
    uint32_t seq = (b[0] << 8) | b[1], ack = (b[2] << 8) | b[3];
    if (F < (uint64_t)H) {  // short frame: fields truncated as utils/packet.py:31 slices them
      if (F < 2) seq = b[0];
      if (F < 4) ack = b[2];
      a.seq[p] = (uint16_t)seq;
      a.ack[p] = (uint16_t)ack;
      a.flags[p] = (uint8_t)b[4];
      a.ok[p] = 2;
      if (a.csum_out) a.csum_out[p] = 0;
      return;
    }
    const uint32_t c = packet_csum(sum, seq, ack, b[4]);
    uint8_t ok;
    if (H == 7) ok = c == ((b[5] << 8) | b[6]) ? 1 : 0;
    else ok = a.csum_in ? (c == a.csum_in[p] ? 1 : 0) : 3;
    a.seq[p] = (uint16_t)seq;
    a.ack[p] = (uint16_t)ack;
    a.flags[p] = (uint8_t)b[4];
    a.ok[p] = ok;
    if (a.csum_out) a.csum_out[p] = (uint16_t)c;
  }
}

// The group leader's part of a varlen decode: `payload_sum` is the frame's
// big-endian word sum over its payload bytes only (the callers mask the
// header out as they sum), `h` its first 16 bytes (little-endian packed).
template <int H>
__device__ __forceinline__ void decode_varlen_finish(const VarlenArgs& a, uint64_t p, uint32_t F,
                                                     uint32_t payload_sum, u32x4 h) {
  const uint32_t b0 = h.x & 0xFFu, b1 = (h.x >> 8) & 0xFFu, b2 = (h.x >> 16) & 0xFFu,
                 b3 = h.x >> 24, b4 = h.y & 0xFFu, b5 = (h.y >> 8) & 0xFFu,
                 b6 = (h.y >> 16) & 0xFFu;
  if (F < (uint32_t)H) {  // short frame: fields truncated as utils/packet.py:31 slices them
    const uint32_t c0 = F > 0 ? b0 : 0u, c1 = F > 1 ? b1 : 0u, c2 = F > 2 ? b2 : 0u,
                   c3 = F > 3 ? b3 : 0u, c4 = F > 4 ? b4 : 0u;
    a.seq[p] = (uint16_t)(F >= 2 ? (c0 << 8) | c1 : c0);
    a.ack[p] = (uint16_t)(F >= 4 ? (c2 << 8) | c3 : c2);
    a.flags[p] = (uint8_t)c4;
    a.ok[p] = 2;
    if (a.csum_out) a.csum_out[p] = 0;
    return;
  }
  const uint32_t seq = (b0 << 8) | b1, ack = (b2 << 8) | b3, flags = b4;
  const uint32_t inband = (b5 << 8) | b6;
  const uint32_t c = packet_csum(payload_sum, seq, ack, flags);
  uint8_t ok;
  if (H == 7) ok = c == inband ? 1 : 0;
  else ok = a.csum_in ? (c == a.csum_in[p] ? 1 : 0) : 3;
  a.seq[p] = (uint16_t)seq;
  a.ack[p] = (uint16_t)ack;
  a.flags[p] = (uint8_t)flags;
  a.ok[p] = ok;
  if (a.csum_out) a.csum_out[p] = (uint16_t)c;
}

// Vectorized varlen decode (frames buffer 16-byte aligned): G lanes per
// frame load the ALIGNED 16-byte chunks overlapping [off[p], off[p+1]) once
// each, mask the chunks at the frame's edges to its payload bytes, and sum
// bytes at even and odd global offsets separately.  A byte at frame position
// k = x - off[p] is the high byte of its big-endian word iff k is even, i.e.
// iff x and off[p] have the same parity, which picks the weighting per frame
// (the fixed-stride decode_verify_kernel's trick with the frame start in
// place of p*F).  The header comes from the group's first two chunks.  G is
// chosen on the host from the batch's mean frame length; any G >= 2 gives the
// same answer.
// U8: the payload's strict UTF-8 check in the same pass: the (masked) payload
// words' high bits are OR'ed as they are summed, and only a frame that holds
// one runs the byte checks (its chunks again, from L2, in lane groups:
// utf8_check_windows_rows).
template <int H, bool U8, int PL = 0, bool FX = false>
__device__ __forceinline__ void decode_varlen_frame(const VarlenArgs& a, uint64_t p, bool valid, uint32_t g,
                                                    uint32_t glog) {
  const uint32_t tid = threadIdx.x;
  const uint32_t G = 1u << glog;
  const uint64_t total = frames_limit<FX>(a);
  uint64_t fstart = valid ? fo_at<FX>(a, p) : 0;
  uint64_t fend = valid ? fo_at<FX>(a, p + 1) : 0;
  const bool bad = valid && (fstart > fend || fend > total);
  if (bad) fstart = fend = 0;  // nothing of it is read
  const uint64_t c_lo = fstart >> 4;
  const uint32_t nchunks = fend > fstart ? (uint32_t)(((fend - 1) >> 4) - c_lo + 1) : 0u;

  uint32_t even_sum = 0, odd_sum = 0;  // byte sums at even / odd global offsets
  uint32_t hib = 0;                     // U8: high bits of the payload bytes
  const uint64_t ps = fstart + H;       // payload start
  u32x4 first = {0u, 0u, 0u, 0u};
  // loads in flight per lane: 8, or 6 with the UTF-8 check (its registers keep the
  // tile kernels that inline this at 6 waves per SIMD); PL: the caller's choice
  constexpr int P = PL ? PL : (U8 ? 6 : 8);
  for (uint32_t i0 = g; i0 < nchunks; i0 += (uint32_t)P * G) {
    uint32_t even = 0, odd = 0;  // at most 32 dwords per round: packed halves cannot overflow
    u32x4 v[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const uint32_t i = i0 + (uint32_t)u * G;
      if (i < nchunks) v[u] = load16_guarded(a.frames, (c_lo + i) << 4, total);
    }
    if (i0 == g) first = v[0];
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const uint32_t i = i0 + (uint32_t)u * G;
      if (i < nchunks) {
        u32x4 w = v[u];
        if (i <= 1 || i + 1 == nchunks) {  // chunks at the frame's edges: its payload bytes only
          const int64_t cb = (int64_t)((c_lo + i) << 4);
          w = keep_bytes(w, (int)((int64_t)ps - cb), (int)((int64_t)fend - cb));
        }
        if (U8) hib |= w.x | w.y | w.z | w.w;
        even += (w.x & 0x00FF00FFu) + (w.y & 0x00FF00FFu) + (w.z & 0x00FF00FFu) + (w.w & 0x00FF00FFu);
        odd += ((w.x >> 8) & 0x00FF00FFu) + ((w.y >> 8) & 0x00FF00FFu) +
               ((w.z >> 8) & 0x00FF00FFu) + ((w.w >> 8) & 0x00FF00FFu);
      }
    }
    // (folded as they go: a frame may be of any length)
    even_sum = fold_keep(even_sum) + (even & 0xFFFFu) + (even >> 16);
    odd_sum = fold_keep(odd_sum) + (odd & 0xFFFFu) + (odd >> 16);
  }
  even_sum = fold_keep(even_sum);
  odd_sum = fold_keep(odd_sum);
  // even global offsets are high bytes iff the frame starts at an even offset
  uint32_t sum = (fstart & 1u) ? (even_sum + (odd_sum << 8)) : ((even_sum << 8) + odd_sum);
  sum = group_sum(sum, G);
  if (U8) hib = group_or_rows(hib, G);
  uint32_t u8bad = 0;
  if (U8 && __any((hib & 0x80808080u) != 0)) {  // the byte checks, for frames with a high bit
    if ((hib & 0x80808080u) && valid && !bad && fend > ps) {
      if (PL == 0 && G >= 2u && G <= 16u) {
        // the payload's aligned chunks again (from L2), the edge ones masked to
        // it, in lane groups: the bytes before a chunk handed on by DPP (the
        // vector kernel's form; the tiles' over-budget frames keep the
        // chunk-pair check, so the tile kernels' code stays as measured)
        const uint64_t c0 = ps >> 4, c1 = (fend - 1u) >> 4;
        auto chunk = [&](uint32_t v) {
          const uint64_t cb = (c0 + v) << 4;
          u32x4 w = load16_guarded(a.frames, cb, total);
          if (v == 0u || c0 + v == c1) w = keep_bytes(w, (int)((int64_t)ps - (int64_t)cb), (int)((int64_t)fend - (int64_t)cb));
          return w;
        };
        auto none = [](const u32x4&, bool) {};
        const uint32_t nc = (uint32_t)(c1 - c0 + 1u);
        u8bad = G == 16u  ? utf8_check_windows_rows<false, true, 16>(nc, g, chunk, none)
                : G == 8u ? utf8_check_windows_rows<false, true, 8>(nc, g, chunk, none)
                : G == 4u ? utf8_check_windows_rows<false, true, 4>(nc, g, chunk, none)
                          : utf8_check_windows_rows<false, true, 2>(nc, g, chunk, none);
      } else {
        u8bad = utf8_check_frame(ps, fend, g, G, [&](uint64_t c) { return load16_guarded(a.frames, c << 4, total); },
                                 [&](uint64_t x) {
                                   return x >= 4 ? *reinterpret_cast<const uint32_t*>(a.frames + x - 4) : 0u;
                                 });
      }
    }
    u8bad = group_or(u8bad, G);
  }
  const int src = (int)((tid & 63u) + 1u);
  u32x4 next;
  next.x = __shfl(first.x, src, 64);
  next.y = __shfl(first.y, src, 64);
  next.z = __shfl(first.z, src, 64);
  next.w = __shfl(first.w, src, 64);
  if (g != 0 || !valid) return;
  if (bad) {
    decode_varlen_reject(a, p);
    return;
  }
  if (U8) a.valid[p] = u8bad ? 0 : 1;
  const uint64_t F = fend - fstart;
  decode_varlen_finish<H>(a, p, F < 0xFFFFFFFFull ? (uint32_t)F : 0xFFFFFFFFu, sum,
                          funnel32(first, next, (uint32_t)(fstart & 15u)));
}

template <int H, bool U8, bool FX = false>
__global__ void __launch_bounds__(kBlock) decode_varlen_vec_kernel(VarlenArgs a) {
  const uint32_t glog = a.glog;
  const uint64_t p = (uint64_t)blockIdx.x * (kBlock >> glog) + (threadIdx.x >> glog);
  decode_varlen_frame<H, U8, 0, FX>(a, p, p < a.n, threadIdx.x & ((1u << glog) - 1u), glog);
}

// Varlen decode through an LDS tile (the fixed-length decode tile's shape):
// a workgroup owns T = 256 / G consecutive frames, whose bytes are one
// contiguous run [frame_off[p0], frame_off[p0 + T]).  Phase 1 streams the run
// into LDS as a copy (every wave-instruction 1 KiB contiguous) and puts the
// tile's frame offsets there; phase 2 gives G lanes to each frame, which sum
// its payload's aligned LDS chunks by address parity (as decode_varlen_vec_kernel
// does from HBM), and the leader parses the header from LDS.  A tile whose run
// exceeds tile_cap (lengths far above the hint) decodes its frames with the
// per-frame vector path inside the same launch.
// Block sums (a.tile_sums == 2, the encode tile's scheme): phase 1 also takes
// the even/odd byte sums of every whole 128-B block of the run from the
// registers it streams through (and, U8, whether the block holds a high
// bit), so a frame's G lanes read the 16 chunks of its two edge blocks and
// one word per block between: work per frame nearly independent of its
// length, where chunk by chunk a tile of ragged lengths waits for its longest
// frame.
__host__ __device__ inline uint32_t dvt_blk_off(uint32_t T, uint32_t cap) {
  return (((((T + 1u) * 4u) + 15u) & ~15u) + kVTGuard + cap + 32u + 15u) & ~15u;
}
__host__ __device__ inline uint32_t dvt_lds_bytes(uint32_t T, uint32_t cap, bool blk) {
  return blk ? dvt_blk_off(T, cap) + ((cap >> 7) + 4u) * 4u : ((((T + 1u) * 4u) + 15u) & ~15u) + kVTGuard + cap + 32u;
}
// OR over 8 consecutive lanes (all 8 active).
__device__ __forceinline__ uint32_t octet_or(uint32_t x) {
  x |= dpp_u32<0xB1>(x);
  x |= dpp_u32<0x4E>(x);
  x |= dpp_u32<0x141>(x);
  return x;
}

// R4: a lane reads its payload chunks four at a time (one LDS wait per four
// instead of one per chunk: the longest frame's chain of LDS round trips is
// what a wave of ragged lengths waits for).
// FUSE (U8, 2-16 lanes a frame, chunk sums; launch_decode_varlen_t picks it): a
// frame's payload chunks are summed and UTF-8 checked in one pass when the
// first two chunk rounds of the wave hold a high bit.  Its own instantiation,
// so the other forms keep the code they were measured with.
template <int H, bool U8, uint32_t NT = kBlock, bool R4 = false, bool FX = false, bool FUSE = false>
__global__ void __launch_bounds__(NT) decode_varlen_tile_kernel(VarlenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog, G = 1u << glog, T = NT >> glog;
  const uint32_t q = tid >> glog, g = tid & (G - 1u);
  uint32_t* lds_fo = reinterpret_cast<uint32_t*>(lds);                       // [T + 1]
  unsigned char* img = lds + ((((T + 1u) * 4u) + 15u) & ~15u) + kVTGuard;   // the run
  const uint64_t p0 = (uint64_t)(a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x) * T;
  const uint64_t left = a.n - p0;
  const uint32_t Tv = left < T ? (uint32_t)left : T;
  const uint64_t fo0 = fo_at<FX>(a, p0), fo_end = fo_at<FX>(a, p0 + Tv);
  // Block sums for every tile (tile_sums 2), or (1) for a tile of uneven frames:
  // every wave reads the tile's T + 1 <= 64 offsets itself (the same lines as
  // wave 0's early ones), so the choice is the same in all four without a
  // barrier; a longest frame over 1.25x the tile's mean takes block sums (the
  // lane groups of a ragged tile then have about equal work), an even tile
  // keeps the chunk sums (no DPP work in its streaming phase).
  // (the choice is made once the run's first loads are in flight: it costs the
  // staging no round trip)
  // (both forms measured slower than chunk sums where lengths are equal, the per-tile
  // choice too: diagnostics build only; profiles/r05/sweeps/varlen_decode_adaptive_blocks.json)
  bool blk = RUDP_TOOLS && a.tile_sums == 2u;
  const bool adapt = RUDP_TOOLS && a.tile_sums == 1u && Tv == 16u;  // (16-frame tiles: MTU-scale hints)
  uint32_t len_adapt = 0;
  if (adapt && (tid & 63u) < 16u) {
    const uint64_t d = fo_at<FX>(a, p0 + (tid & 63u) + 1u) - fo_at<FX>(a, p0 + (tid & 63u));
    len_adapt = d < 0xFFFFFFFFull ? (uint32_t)d : 0xFFFFFFFFu;
  }
  const uint64_t total = frames_limit<FX>(a);
  const uint64_t A = fo0 & ~15ull;
  const uint64_t run = ((fo_end + 15u) & ~15ull) - A;
  if (fo0 > fo_end || fo_end > total || run > a.tile_cap) {  // uniform over the workgroup
    decode_varlen_frame<H, U8, 6, FX>(a, p0 + q, q < Tv, g, glog);
    return;
  }
  // The block words: tile_sums 2, a region of their own after the run's budget;
  // per tile (1), right after the run inside its budget (no LDS beyond the chunk
  // form's, which would cost a tile per CU at MTU hints: 27.1 vs 26.3 KB), for
  // tiles that leave room for them.
  uint32_t* lds_blk = reinterpret_cast<uint32_t*>(
      a.tile_sums == 2u ? lds + dvt_blk_off(T, a.tile_cap) : img + run + 16u);  // [run / 128 + 2]
  const bool blk_room = run + 16u + (run >> 5) + 8u <= a.tile_cap;
  // tile-relative offsets; one outside [A, fo_end] reads as 0xFFFFFFFF
  const uint64_t span_end = fo_end - A;
  auto rel = [&](uint64_t o) { return o - A <= span_end ? (uint32_t)(o - A) : 0xFFFFFFFFu; };
  {
    // T = 256 / G <= 128 frames: one offset per lane, loaded before the run (early_fo)
    const uint32_t fo_r = a.early_fo && tid <= Tv ? rel(fo_at<FX>(a, p0 + tid)) : 0u;
    const uint32_t nvec = (uint32_t)(run >> 4);
    u32x4* dst = reinterpret_cast<u32x4*>(img);
    constexpr uint32_t P = 8;
    const bool decide = adapt && nvec >= NT;  // (every lane then runs the first round)
    auto stage = [&](uint32_t v0, bool first) {
      u32x4 r[P];
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * NT;
        if (v < nvec) r[u] = load16_guarded(a.frames, A + 16ull * v, total);
      }
      if (first && decide) {
        // the tile's longest frame against its mean: lane i < 16 of every wave
        // holds frame i's length (its two offsets, loaded with the tile's first
        // ones), a DPP max over the row, the first lane's value for the wave
        uint32_t mx = len_adapt;
        mx = max(mx, dpp_row<0xB1>(mx));
        mx = max(mx, dpp_row<0x4E>(mx));
        mx = max(mx, dpp_row<0x141>(mx));
        mx = max(mx, dpp_row<0x140>(mx));
        mx = (uint32_t)__builtin_amdgcn_readfirstlane((int)mx);
        blk = blk_room && (uint64_t)mx * 16u * 4u > (fo_end - fo0) * 5u;
      }
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * NT;
        if (v < nvec) dst[v] = r[u];
        // block sums from the registers: whole 128-B blocks only (uniform per 8
        // lanes; a partial last block is only ever an edge block of a frame)
        if (blk && (v | 7u) < nvec) {
          uint32_t eo = octet_sum(eo_sum(lo64(r[u]), hi64(r[u])));  // e, o at most 16320 each
          if (U8 && octet_or(high_bits(r[u]))) eo |= 0x8000u;      // the block holds a high bit
          if ((tid & 7u) == 0) lds_blk[v >> 3] = eo;
        }
      }
    };
    uint32_t v0 = tid;
    if (v0 < nvec) {
      stage(v0, true);
      v0 += P * NT;
    }
    for (; v0 < nvec; v0 += P * NT) stage(v0, false);
    if (a.early_fo) {
      if (tid <= Tv) lds_fo[tid] = fo_r;
    } else {
      for (uint32_t i = tid; i <= Tv; i += NT) lds_fo[i] = rel(fo_at<FX>(a, p0 + i));
    }
  }
  __syncthreads();
  const uint32_t glog2 = glog, G2 = G, q2 = q, g2 = g;
  const u32x4* img16 = reinterpret_cast<const u32x4*>(img);
  auto frame = [&](const uint32_t q) {
    const uint32_t fs = lds_fo[q], fe = lds_fo[q + 1];
    // A pair out of order, or an offset outside the tile's run: the frame may
    // still be valid (its own pair in order and inside the buffer is all the
    // rule asks) but reach past the staged bytes, so it decodes from HBM, where
    // the rule is applied to its true offsets.  Uniform over the frame's lanes.
    if (fs > fe || fe > (uint32_t)span_end) {
      decode_varlen_frame<H, U8, 6, FX>(a, p0 + q, true, g2, glog2);
      return;
    }
    // the leader's header window, read now so its LDS round trip overlaps the sums
    u32x4 hdr = make_u32x4(0ull, 0ull);
    if (g2 == 0) hdr = window16_dw(reinterpret_cast<const uint32_t*>(img), fs);
    uint32_t even_sum = 0, odd_sum = 0;  // byte sums at even / odd offsets (A is even)
    uint32_t hib = 0;                     // U8: high bits of the payload bytes
    const uint32_t ps = fs + (uint32_t)H;
    bool fused = false;                   // FUSE: the check ran with the sums (wave-uniform)
    uint32_t u8bad_f = 0;
    if (FUSE && fe > ps) {
      // the payload's aligned chunks (the two edge ones masked to it), summed by
      // address parity and, once the wave's first two chunk rounds hold a high
      // bit, UTF-8 checked in the same pass (utf8_device.hpp: the bytes before
      // a chunk handed across the DPP row; bytes outside the payload are 0)
      const uint32_t c0 = ps >> 4, c1 = (fe - 1u) >> 4;
      auto chunk = [&](uint32_t v) {
        const uint32_t c = c0 + v;
        u32x4 w = img16[c];
        if (c == c0 || c == c1) w = keep_bytes(w, (int)ps - (int)(c << 4), (int)fe - (int)(c << 4));
        return w;
      };
      auto sums = [&](const u32x4& w, bool in) {
        const uint32_t e = even_bytes_acc(w.w, even_bytes_acc(w.z, even_bytes_acc(w.y, even_bytes_acc(w.x, 0u))));
        const uint32_t o = odd_bytes_acc(w.w, odd_bytes_acc(w.z, odd_bytes_acc(w.y, odd_bytes_acc(w.x, 0u))));
        even_sum += in ? e : 0u;
        odd_sum += in ? o : 0u;
      };
      const uint32_t nc = c1 - c0 + 1u;
      u8bad_f = G2 == 16u ? utf8_check_windows_rows<true, true, 16>(nc, g2, chunk, sums, &hib, &fused)
                : G2 == 8u ? utf8_check_windows_rows<true, true, 8>(nc, g2, chunk, sums, &hib, &fused)
                : G2 == 4u ? utf8_check_windows_rows<true, true, 4>(nc, g2, chunk, sums, &hib, &fused)
                           : utf8_check_windows_rows<true, true, 2>(nc, g2, chunk, sums, &hib, &fused);
    } else if (blk && fe > ps) {
      // the 16 chunks of the blocks holding the payload's first and last bytes
      // (each masked to the payload), then the block words between
      const uint32_t j0 = ps >> 7, j1 = (fe - 1u) >> 7;
      for (uint32_t c = g2; c < 16u; c += G2) {
        const uint32_t cx = ((c < 8u ? j0 : j1) << 7) + ((c & 7u) << 4);
        if ((c < 8u || j1 != j0) && cx < fe && cx + 16u > ps) {
          const u32x4 w = keep_bytes(img16[cx >> 4], (int)ps - (int)cx, (int)fe - (int)cx);
          const uint32_t eo = eo_sum(lo64(w), hi64(w));
          even_sum += eo & 0xFFFFu;
          odd_sum += eo >> 16;
          if (U8) hib |= w.x | w.y | w.z | w.w;
        }
      }
      for (uint32_t j = j0 + 1u + g2; j < j1; j += G2) {
        const uint32_t bs = lds_blk[j];
        even_sum += bs & 0x7FFFu;
        odd_sum += bs >> 16;
        if (U8) hib |= (bs & 0x8000u) ? 0x80u : 0u;
      }
    } else if (fe > ps) {  // the payload's chunks, the edge ones masked to it
      const uint32_t c0 = ps >> 4, c1 = (fe - 1u) >> 4;
      auto add = [&](u32x4 w, uint32_t c) {
        if (c == c0 || c == c1) w = keep_bytes(w, (int)ps - (int)(c << 4), (int)fe - (int)(c << 4));
        if (U8) hib |= w.x | w.y | w.z | w.w;
        even_sum = even_bytes_acc(w.w, even_bytes_acc(w.z, even_bytes_acc(w.y, even_bytes_acc(w.x, even_sum))));
        odd_sum = odd_bytes_acc(w.w, odd_bytes_acc(w.z, odd_bytes_acc(w.y, odd_bytes_acc(w.x, odd_sum))));
      };
      if (R4) {
        for (uint32_t c = c0 + g2; c <= c1; c += 4u * G2) {
          u32x4 w[4];
#pragma unroll
          for (uint32_t u = 0; u < 4u; ++u) {
            const uint32_t cu = c + u * G2;
            w[u] = cu <= c1 ? img16[cu] : make_u32x4(0ull, 0ull);
          }
#pragma unroll
          for (uint32_t u = 0; u < 4u; ++u)
            if (c + u * G2 <= c1) add(w[u], c + u * G2);
        }
      } else {
        for (uint32_t c = c0 + g2; c <= c1; c += G2) add(img16[c], c);
      }
    }
    // even offsets are high bytes iff the frame starts at an even offset
    uint32_t sum = (fs & 1u) ? (even_sum + (odd_sum << 8)) : ((even_sum << 8) + odd_sum);
    sum = group_sum(sum, G2);
    if (U8) hib = group_or_rows(hib, G2);
    if (U8) {  // a frame with a high bit in its payload: the byte checks, from LDS
      uint32_t u8bad = 0;
      if (fused) {
        u8bad = group_or(u8bad_f, G2);
      } else if (__any((hib & 0x80808080u) != 0)) {
        if (hib & 0x80808080u) {
          const uint32_t* idw = reinterpret_cast<const uint32_t*>(img);  // kVTGuard bytes before it
          if (G2 >= 2u && G2 <= 16u) {
            // 2-16 lanes a frame: over payload-aligned windows, the bytes before a
            // window handed across the lane group by DPP (utf8_device.hpp); the
            // last window masked to the payload (the run's budget has 32 B past its end)
            const uint32_t L = fe - ps, V = (L + 15u) >> 4;
            auto win = [&](uint32_t v) {
              u32x4 w = window16_dw(idw, ps + 16u * v);
              if (16u * v + 16u > L) w = keep_bytes(w, 0, (int)(L - 16u * v));
              return w;
            };
            auto none = [](const u32x4&, bool) {};
            u8bad = G2 == 16u  ? utf8_check_windows_rows<false, true, 16>(V, g2, win, none)
                    : G2 == 8u ? utf8_check_windows_rows<false, true, 8>(V, g2, win, none)
                    : G2 == 4u ? utf8_check_windows_rows<false, true, 4>(V, g2, win, none)
                               : utf8_check_windows_rows<false, true, 2>(V, g2, win, none);
          } else {
            u8bad = utf8_check_frame(ps, fe, g2, G2, [&](uint64_t c) { return img16[c]; },
                                     [&](uint64_t x) { return idw[(int64_t)(x >> 2) - 1]; });
          }
        }
        u8bad = group_or(u8bad, G2);
      }
      if (g2 == 0) a.valid[p0 + q] = u8bad ? 0 : 1;
    }
    if (g2 == 0)
      decode_varlen_finish<H>(a, p0 + q, fe - fs, sum, hdr);
  };
  if (q2 < Tv) frame(q2);
}

// ---------------------------------------------------------------------------
// Varlen decode by byte spans (checked calls, a.span_rec set).
//
// Frame tiles (decode_varlen_tile_kernel) hold T frames each: with ragged
// lengths their runs spread (16 frames of U[0, 2944] B: 23.5 KiB +- 3.4 KiB),
// a quarter overflow the LDS budget into the per-frame path, and the G lanes
// of a frame sum its chunks while the wave waits for its longest frame.  Here
// workgroup k decodes the frames that START in bytes [k S, (k + 1) S) of the
// buffer (decode_span_index_kernel found them), so every run is S plus at
// most its last frame, and the lanes split the run's chunks evenly: lane l
// sums chunks [l kc, (l + 1) kc) whatever frames they hold.  A frame's
// payload sum is then the difference of two prefix sums of the run, at its
// payload start and end: a lane records the prefix at every boundary inside
// its chunks, a scan over the lanes makes those prefixes absolute, and the
// frame's leader subtracts.  Offsets not in order, or past the buffer: the
// index pass raises span_flag, and the launch decodes frame by frame (every
// pair checked, decode_varlen_frame).
#if RUDP_TOOLS  // measured slower than the frame tiles: the diagnostics build only
constexpr uint32_t kSpanNF = 128;  // frames of one span held in LDS (more: per-frame path)

// one record per span (and one past the last): first frame starting at or
// past k S, and its offset.  Thread i <= n writes the spans whose first frame
// is i; threads past n write the spans past the last offset.
__global__ void __launch_bounds__(kBlock) decode_span_index_kernel(const uint64_t* fo, uint64_t n, uint64_t lim,
                                                                   uint32_t S, uint32_t nt, SpanRec* rec,
                                                                   uint32_t* flag, uint32_t epoch) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i <= n) {
    const uint64_t x = fo[i];
    const uint64_t xp = i ? fo[i - 1] : 0u;
    if (x > lim || xp > x) {
      *flag = epoch;
      return;
    }
    const uint64_t k1 = x / S;
    for (uint64_t k = i ? xp / S + 1u : 0u; k <= k1; ++k) rec[k] = SpanRec{x, (uint32_t)i, 0u};
  } else if (i <= n + 1u + nt) {
    const uint64_t k = i - n - 1u;
    const uint64_t x = fo[n];
    if (x <= lim && k > x / S) rec[k] = SpanRec{x, (uint32_t)n, 0u};
  }
}

__host__ __device__ inline uint32_t dsp_pre_off() { return (((kSpanNF + 1u) * 4u) + 15u) & ~15u; }
__host__ __device__ inline uint32_t dsp_img_off() {
  // fo u32[NF + 1] | boundary prefixes u32[2 NF] | their high-byte counts u16[2 NF] |
  // wave sums u64[4] | wave counts u32[4] | lane prefixes u64[256] | lane counts u16[256] | guard | run
  return ((dsp_pre_off() + 8u * kSpanNF + 4u * kSpanNF + 32u + 16u + 8u * kBlock + 2u * kBlock + 15u) & ~15u) +
         kVTGuard;
}
__host__ __device__ inline uint32_t dsp_lds_bytes(uint32_t cap) { return dsp_img_off() + cap + 32u; }

template <int H, bool U8>
__global__ void __launch_bounds__(kBlock) decode_varlen_span_kernel(VarlenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog, G = 1u << glog, T = kBlock >> glog;
  const uint32_t q = tid >> glog, g = tid & (G - 1u);
  const uint32_t nt = (uint32_t)a.span_count;
  // the flag and the span's two records in one round trip
  const uint32_t k = blockIdx.x >= nt ? 0u : a.xcd ? xcd_tile(blockIdx.x, nt) : blockIdx.x;
  const uint32_t flag = *a.span_flag;
  const SpanRec r0 = a.span_rec[k], r1 = a.span_rec[k + 1];
  if (flag == a.span_epoch) {  // offsets out of order or past the buffer: frame by frame
    const uint64_t p = (uint64_t)blockIdx.x * T + q;
    if ((uint64_t)blockIdx.x * T < a.n) decode_varlen_frame<H, U8, 4>(a, p, p < a.n, g, glog);
    return;
  }
  if (blockIdx.x >= nt) return;
  const uint32_t nf = r1.p - r0.p;
  if (nf == 0) return;
  const uint64_t f0 = r0.p;
  const uint64_t A = r0.fo & ~15ull;
  const uint64_t run = ((r1.fo + 15u) & ~15ull) - A;
  if (nf > kSpanNF || run > a.tile_cap) {  // uniform: the span's frames one by one from HBM
    for (uint32_t base = 0; base < nf; base += T)
      decode_varlen_frame<H, U8, 4>(a, f0 + base + q, base + q < nf, g, glog);
    return;
  }
  uint32_t* lds_fo = reinterpret_cast<uint32_t*>(lds);                                      // [nf + 1]
  uint32_t* lds_pre = reinterpret_cast<uint32_t*>(lds + dsp_pre_off());                         // [2 nf]
  uint16_t* lds_ph = reinterpret_cast<uint16_t*>(lds_pre + 2u * kSpanNF);                      // [2 nf]
  uint64_t* lds_wsum = reinterpret_cast<uint64_t*>(lds_ph + 2u * kSpanNF);                     // [4]
  uint32_t* lds_whc = reinterpret_cast<uint32_t*>(lds_wsum + 4);                               // [4]
  uint64_t* lds_lex = reinterpret_cast<uint64_t*>(lds_whc + 4);                                // [256]
  uint16_t* lds_lhc = reinterpret_cast<uint16_t*>(lds_lex + kBlock);                           // [256]
  unsigned char* img = lds + dsp_img_off();
  const uint64_t total = frames_limit<false>(a);
#if RUDP_TOOLS
  if (a.diag & 64u) {  // ablation: the loads only
    const uint32_t nvec = (uint32_t)(run >> 4);
    u32x4 x = make_u32x4(0ull, 0ull);
    for (uint32_t v = tid; v < nvec; v += kBlock) {
      const u32x4 r = load16_guarded(a.frames, A + 16ull * v, total);
      x.x ^= r.x;
    }
    if (x.x == 0x12345678u) a.ok[f0] = 9;
    return;
  }
#endif
  {
    const uint32_t fo_r = tid <= nf ? (uint32_t)(a.frame_off[f0 + tid] - A) : 0u;
    const uint32_t nvec = (uint32_t)(run >> 4);
    u32x4* dst = reinterpret_cast<u32x4*>(img);
    constexpr uint32_t P = 8;
    for (uint32_t v0 = tid; v0 < nvec; v0 += P * kBlock) {
      u32x4 r[P];
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * kBlock;
        if (v < nvec) r[u] = load16_guarded(a.frames, A + 16ull * v, total);
      }
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t v = v0 + u * kBlock;
        if (v < nvec) dst[v] = r[u];
      }
    }
    if (tid <= nf) lds_fo[tid] = fo_r;
  }
  __syncthreads();
  const u32x4* img16 = reinterpret_cast<const u32x4*>(img);
  const uint32_t nvec = (uint32_t)(run >> 4);
  // Lane tid sums chunks [tid kc, (tid + 1) kc) of the run, whatever frames
  // they hold (the lanes cover one chunk past the run, so every boundary, at
  // most 16 nvec, lies in some lane's chunks; kc odd: the 16 lanes of an LDS
  // pass read 16 different bank groups).  U8: it also counts bytes >= 0x80.
  const uint32_t kc = (nvec / kBlock + 1u) | 1u;
  const uint32_t c_begin = tid * kc;
  const uint32_t c_end = c_begin + kc < nvec ? c_begin + kc : nvec;
  auto hcount = [](const u32x4& w) {
    return (uint32_t)(__builtin_popcount(w.x & 0x80808080u) + __builtin_popcount(w.y & 0x80808080u) +
                      __builtin_popcount(w.z & 0x80808080u) + __builtin_popcount(w.w & 0x80808080u));
  };
  uint32_t acc = 0, hc = 0;  // even | odd << 16 byte sums (each at most kc * 2040), high bytes
#if RUDP_TOOLS
  const uint32_t c_stop = (a.diag & 16u) ? c_begin : c_end;  // ablation: no sums
#else
  const uint32_t c_stop = c_end;
#endif
  for (uint32_t c0 = c_begin; c0 < c_stop; c0 += 4u) {
    u32x4 w[4];
#pragma unroll
    for (uint32_t u = 0; u < 4u; ++u) w[u] = c0 + u < c_stop ? img16[c0 + u] : make_u32x4(0ull, 0ull);
#pragma unroll
    for (uint32_t u = 0; u < 4u; ++u) {
      acc += eo_sum(lo64(w[u]), hi64(w[u]));
      if (U8) hc += hcount(w[u]);
    }
  }
  // each lane's exclusive prefix within its wave, and the four wave totals
  {
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    uint32_t se = acc & 0xFFFFu, so = acc >> 16, sh = hc;
    for (uint32_t d = 1; d < 64u; d <<= 1) {
      const uint32_t te = (uint32_t)__shfl_up((int)se, d, 64), to = (uint32_t)__shfl_up((int)so, d, 64);
      const uint32_t th = U8 ? (uint32_t)__shfl_up((int)sh, d, 64) : 0u;
      if (lane >= d) {
        se += te;
        so += to;
        sh += th;
      }
    }
    if (lane == 63u) {
      lds_wsum[wave] = (uint64_t)se | ((uint64_t)so << 32);
      if (U8) lds_whc[wave] = sh;
    }
    lds_lex[tid] = (uint64_t)(se - (acc & 0xFFFFu)) | ((uint64_t)(so - (acc >> 16)) << 32);
    if (U8) lds_lhc[tid] = (uint16_t)(sh - hc);  // (at most 63 * 16 kc)
  }
  __syncthreads();
  // Boundary b = tid: payload start of frame b / 2 (even b) or its end (odd
  // b).  The run's sums before it = its lane's prefix + that lane's chunks up
  // to it (at most kc reads, issued four at a time), weighted by the frame's
  // start parity (even offsets are high bytes iff the frame starts even).
  if (tid < 2u * nf) {
    const uint32_t i = tid >> 1, fs = lds_fo[i], fe = lds_fo[i + 1u];
    const uint32_t x = (tid & 1u) ? fe : (fs + (uint32_t)H < fe ? fs + (uint32_t)H : fe);
    const uint32_t cx = x >> 4, L = cx / kc;
    uint32_t loc = 0, lh = 0;
    for (uint32_t c0 = L * kc; c0 <= cx; c0 += 4u) {
      u32x4 w[4];
#pragma unroll
      for (uint32_t u = 0; u < 4u; ++u) {
        const uint32_t c = c0 + u;
        w[u] = c <= cx && c < nvec ? img16[c] : make_u32x4(0ull, 0ull);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4u; ++u) {
        const uint32_t c = c0 + u;
        const u32x4 v = c == cx ? keep_bytes(w[u], 0, (int)(x & 15u)) : w[u];
        loc += eo_sum(lo64(v), hi64(v));
        if (U8) lh += hcount(v);
      }
    }
    uint64_t p = lds_lex[L];
    uint32_t ph = U8 ? lds_lhc[L] : 0u;
    for (uint32_t w = 0; w < (L >> 6); ++w) {
      p += lds_wsum[w];
      if (U8) ph += lds_whc[w];
    }
    const uint32_t e = (uint32_t)p + (loc & 0xFFFFu), o = (uint32_t)(p >> 32) + (loc >> 16);
    lds_pre[tid] = (fs & 1u) ? e + (o << 8) : (e << 8) + o;
    if (U8) lds_ph[tid] = (uint16_t)(ph + lh);
  }
  __syncthreads();
  if (U8) {  // frames with a byte >= 0x80 in their payload: the byte checks, G lanes each, from LDS
    const uint32_t* idw = reinterpret_cast<const uint32_t*>(img);  // kVTGuard bytes before it
    for (uint32_t base = 0; base < nf; base += T) {
      const uint32_t i = base + q;
      const bool flagged = i < nf && lds_ph[2u * i + 1u] != lds_ph[2u * i];
      if (__any(flagged)) {
        uint32_t bad = 0;
        if (flagged) {
          const uint32_t fs = lds_fo[i], fe = lds_fo[i + 1u];
          const uint32_t ps = fs + (uint32_t)H < fe ? fs + (uint32_t)H : fe;
          bad = utf8_check_frame(ps, fe, g, G, [&](uint64_t c) { return img16[c]; },
                                 [&](uint64_t x) { return idw[(int64_t)(x >> 2) - 1]; });
        }
        bad = group_or(bad, G);
        if (flagged && g == 0) a.valid[f0 + i] = bad ? 0 : 1;
      }
    }
  }
#if RUDP_TOOLS
  if (a.diag & 32u) return;  // ablation: no leaders' work
#endif
  if (tid < nf) {
    const uint32_t fs = lds_fo[tid], fe = lds_fo[tid + 1u];
    if (U8 && lds_ph[2u * tid + 1u] == lds_ph[2u * tid]) a.valid[f0 + tid] = 1;
    decode_varlen_finish<H>(a, f0 + tid, fe - fs, lds_pre[2u * tid + 1u] - lds_pre[2u * tid],
                            window16_dw(reinterpret_cast<const uint32_t*>(img), fs));
  }
}
#endif  // RUDP_TOOLS

// Strict UTF-8 validation kernels (the checks themselves: utf8_device.hpp).
__global__ void __launch_bounds__(kBlock) validate_utf8_par_kernel(Utf8Args a) {
  if (call_failed(a.status)) return;
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid_p = p < a.n;
  uint32_t bad = 0;
  if (valid_p) {
    uint64_t fo, fe;
    if (a.frame_off) {
      fo = a.frame_off[p];
      fe = a.frame_off[p + 1];
    } else {
      fo = p * (uint64_t)a.F;
      fe = fo + a.F;
    }
    const uint64_t s = fo + a.H;  // payload start
    if (s < fe) bad = utf8_slice(a.frames, s, fe - s, g, kVarLanes);
  }
  for (uint32_t m = kVarLanes >> 1; m > 0; m >>= 1) bad |= __shfl_xor(bad, (int)m, 64);
  if (valid_p && g == 0) a.valid[p] = bad ? 0 : 1;
}

// Vector form of the same check for 16-byte-aligned frame buffers: G = 16
// lanes per frame walk the ALIGNED 16-byte chunks that overlap the payload
// (one dwordx4 each, plus the dword before the chunk for the three
// predecessor bytes), bytes outside [payload start, frame end) count as
// absent (0).  An all-ASCII chunk whose predecessors hold no lead byte is
// valid without the per-byte walk: the common case for text payloads.

__global__ void __launch_bounds__(kBlock) validate_utf8_vec_kernel(Utf8Args a) {
  if (call_failed(a.status)) return;
  constexpr uint32_t U = 4;  // chunks per lane per round (2 and 8, nt loads: no better)
  const uint32_t G = 1u << a.glog;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = threadIdx.x & (G - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> a.glog;
  const bool valid_p = p < a.n;
  uint64_t fo = 0, fe = 0;
  if (valid_p) {
    if (a.frame_off) {
      fo = a.frame_off[p];
      fe = a.frame_off[p + 1];
    } else {
      fo = p * (uint64_t)a.F;
      fe = fo + a.F;
    }
  }
  const uint64_t s = fo + a.H;
  const uint64_t total = a.frame_off ? a.frame_off[a.n] : a.n * (uint64_t)a.F;
  const uint64_t c_lo = s >> 4;
  const uint64_t c_hi = s < fe ? (fe - 1) >> 4 : 0;
  const uint32_t nch = s < fe ? (uint32_t)(c_hi - c_lo + 1) : 0u;
  // the group's round count is uniform across the wave's groups only up to
  // their own nch: every lane runs the shuffles of the longest group's rounds
  uint32_t rounds = (nch + G * U - 1u) / (G * U);
  for (uint32_t m = 32; m > 0; m >>= 1) rounds = max(rounds, (uint32_t)__shfl_xor((int)rounds, (int)m, 64));
  // Rounds of U chunks per lane, all loads issued first.  Lane g takes chunks
  // c_lo + g + G*(u + U*r).  The three bytes before a chunk (the end of chunk
  // c-1) come by shuffle: from lane g-1 in the same round slot, or for g = 0
  // from lane G-1 one slot earlier (the previous round's last slot: `carry`).
  const int src_same = (int)(g > 0 ? lane - 1u : lane);
  const int src_prev = (int)(g == 0 ? lane + G - 1u : lane);
  uint32_t bad = 0, carry = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    u32x4 vv[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = g + G * (u + U * r);
      const uint64_t base = (c_lo + i) << 4;
      vv[u] = make_u32x4(0ull, 0ull);
      if (i < nch) {
        if (base + 16 <= total) {
          vv[u] = *reinterpret_cast<const u32x4*>(a.frames + base);
        } else {  // the batch's last chunk: never read past the buffer
          uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const uint32_t b = base + k < total ? (uint32_t)a.frames[base + k] << (8 * (k & 3)) : 0u;
            if (k < 4) d0 |= b;
            else if (k < 8) d1 |= b;
            else if (k < 12) d2 |= b;
            else d3 |= b;
          }
          vv[u].x = d0;
          vv[u].y = d1;
          vv[u].z = d2;
          vv[u].w = d3;
        }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t same = (uint32_t)__shfl((int)vv[u].w, src_same, 64);
      const uint32_t prev_slot = (uint32_t)__shfl((int)(u > 0 ? vv[u - 1].w : carry), src_prev, 64);
      const uint32_t prev = g > 0 ? same : prev_slot;
      const uint32_t i = g + G * (u + U * r);
      if (i >= nch) continue;
      const uint64_t base = (c_lo + i) << 4;
      const u32x4 v = vv[u];
      // predecessor bytes, zeroed where they fall before the payload start
      uint32_t p3 = (base >= s + 3) ? (prev >> 8) & 0xFFu : 0u;
      uint32_t p2 = (base >= s + 2) ? (prev >> 16) & 0xFFu : 0u;
      uint32_t p1 = (base >= s + 1) ? (prev >> 24) : 0u;
      // the payload's bytes of this chunk (others zeroed: ASCII by construction)
      const int lo_b = (int)((int64_t)s - (int64_t)base), hi_b = (int)((int64_t)fe - (int64_t)base);
      const uint64_t pl = lo64(v) & byte_mask(lo_b, hi_b), ph = hi64(v) & byte_mask(lo_b - 8, hi_b - 8);
      if (((pl | ph) & 0x8080808080808080ull) == 0 && p1 < 0xC0 && p2 < 0xC0 && p3 < 0xC0)
        continue;  // plain ASCII, nothing pending from before (and so nothing at the end)
      if (bad) continue;  // this lane already found an invalid byte
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint64_t x = base + (uint64_t)k;
        if (x < s || x >= fe) continue;
        const uint32_t cb = byte_of(v, k);
        bad |= utf8_byte_ok(cb, p1, p2, p3) ? 0u : 1u;
        p3 = p2;
        p2 = p1;
        p1 = cb;
      }
      if (i + 1 == nch)  // the frame's last chunk: nothing may still be expected
        bad |= utf8_pending(p1, p2, p3) ? 1u : 0u;
    }
    carry = vv[U - 1].w;
  }
  for (uint32_t m = G >> 1; m > 0; m >>= 1) bad |= __shfl_xor(bad, (int)m, 64);
  if (valid_p && g == 0) a.valid[p] = bad ? 0 : 1;
}

// Fixed-stride frames through an LDS tile (frames 16-B aligned, H < F,
// T = 256 / G frames per workgroup with T % 16 == 0, so the tile starts on a
// 16-B boundary): the decode tile kernel's shape.  Phase 1 streams the tile's
// T*F bytes into LDS as one contiguous run (1 KiB per wave-instruction);
// phase 2 gives G lanes to each frame, which read its payload as aligned LDS
// chunks: a chunk whose payload bytes are ASCII with nothing pending from the
// three bytes before it (an aligned LDS dword, no shuffles) is done; any other
// runs the byte checks.  The per-lane, per-frame strided global loads of the
// vector kernel gave 256-B runs per wave-instruction instead.
__global__ void __launch_bounds__(kBlock) validate_utf8_tile_kernel(Utf8Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog, G = 1u << glog, T = kBlock >> glog;
  const uint32_t q = tid >> glog, g = tid & (G - 1u);
  const uint64_t p0 = (uint64_t)(a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x) * T;
  const uint64_t left = a.n - p0;
  const uint32_t Tv = left < T ? (uint32_t)left : T;
  const uint32_t F = a.F, H = a.H;
  const uint64_t total = a.n * (uint64_t)F;
  const uint64_t base = p0 * (uint64_t)F;  // 16-B aligned: T % 16 == 0
  const uint32_t nbytes = Tv * F;
  const uint32_t nvec = (nbytes + 15u) >> 4;
  u32x4* tile = reinterpret_cast<u32x4*>(lds + 16);  // 16 B of guard before the tile
  {
    const uint64_t whole = (total - base) >> 4;
    const uint32_t ndma = whole < nvec ? (uint32_t)whole : nvec;
    const uint32_t lane = tid & 63u;
    const u32x4* src = reinterpret_cast<const u32x4*>(a.frames + base);
    for (uint32_t v0 = tid & ~63u; v0 < ndma; v0 += kBlock)
      if (v0 + lane < ndma)
        __builtin_amdgcn_global_load_lds(
            (const void __attribute__((address_space(1)))*)(src + v0 + lane),
            (void __attribute__((address_space(3)))*)(tile + v0), 16, 0, 2);
    if (ndma < nvec && tid == 0) tile[ndma] = load16_guarded(a.frames, base + 16ull * ndma, total);
  }
  __syncthreads();
  uint32_t bad = 0;
  if (q < Tv) {
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(lds + 16);
    if (G >= 2u && G <= 16u)  // over payload-aligned windows, the bytes before handed on by DPP
      bad = utf8_check_payload_group(F - H, g, G, [&](uint32_t v) { return window16_dw(dw, q * F + H + 16u * v); });
    else
      bad = utf8_check_frame(q * F + H, q * F + F, g, G,  // payload bytes [s, fe) of the tile
                             [&](uint64_t c) { return tile[c]; },
                             [&](uint64_t x) { return dw[(x >> 2) - 1u]; });  // x = 0 reads the guard
  }
  for (uint32_t m = G >> 1; m > 0; m >>= 1) bad |= __shfl_xor(bad, (int)m, 64);
  if (g == 0 && q < Tv) a.valid[p0 + q] = bad ? 0 : 1;
}

// Packed variable-length frames through an LDS tile (frames 16-B aligned;
// hints of 128 B and up): a workgroup owns T = 256 / G consecutive frames,
// one contiguous run [frame_off[p0], frame_off[p0 + T]) streamed into LDS by
// LDS-DMA; the frames' offsets come along.  A run over tile_cap (lengths far
// above the hint) checks its frames straight from HBM instead.
__global__ void __launch_bounds__(kBlock) validate_utf8_vtile_kernel(Utf8Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t glog = a.glog, G = 1u << glog, T = kBlock >> glog;
  const uint32_t q = tid >> glog, g = tid & (G - 1u);
  const uint64_t p0 = (uint64_t)(a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x) * T;
  const uint64_t left = a.n - p0;
  const uint32_t Tv = left < T ? (uint32_t)left : T;
  const uint64_t total = a.frame_off[a.n];
  const uint64_t fo0 = a.frame_off[p0], fo_end = a.frame_off[p0 + Tv];
  if (call_failed(a.status)) return;
  const uint64_t A = fo0 & ~15ull;
  const uint64_t run = ((fo_end + 15u) & ~15ull) - A;
  uint32_t bad = 0;
  if (run > a.tile_cap) {  // uniform over the workgroup: frames straight from HBM
    if (q < Tv)
      bad = utf8_check_frame(a.frame_off[p0 + q] + a.H, a.frame_off[p0 + q + 1], g, G,
                             [&](uint64_t c) { return load16_guarded(a.frames, c << 4, total); },
                             [&](uint64_t x) {
                               return x >= 4 ? *reinterpret_cast<const uint32_t*>(a.frames + x - 4) : 0u;
                             });
  } else {
    uint32_t* lds_fo = reinterpret_cast<uint32_t*>(lds);                    // [T + 1]
    const uint32_t img_off = ((((T + 1u) * 4u) + 15u) & ~15u) + 16u;       // 16 B guard before the run
    u32x4* img = reinterpret_cast<u32x4*>(lds + img_off);
    const uint32_t nvec = (uint32_t)(run >> 4);
    const uint64_t whole = total > A ? (total - A) >> 4 : 0u;
    const uint32_t ndma = whole < nvec ? (uint32_t)whole : nvec;
    const uint32_t lane = tid & 63u;
    const u32x4* src = reinterpret_cast<const u32x4*>(a.frames + A);
    for (uint32_t v0 = tid & ~63u; v0 < ndma; v0 += kBlock)
      if (v0 + lane < ndma)
        __builtin_amdgcn_global_load_lds(
            (const void __attribute__((address_space(1)))*)(src + v0 + lane),
            (void __attribute__((address_space(3)))*)(img + v0), 16, 0, 2);
    if (ndma < nvec && tid == 0) img[ndma] = load16_guarded(a.frames, A + 16ull * ndma, total);
    for (uint32_t i = tid; i <= Tv; i += kBlock) lds_fo[i] = (uint32_t)(a.frame_off[p0 + i] - A);
    __syncthreads();
    if (q < Tv) {
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(lds + img_off);
      const uint32_t ps = lds_fo[q] + a.H, fe = lds_fo[q + 1];
      if (G >= 2u && G <= 16u)  // over payload-aligned windows, the bytes before handed on by DPP
        bad = utf8_check_payload_group(fe > ps ? fe - ps : 0u, g, G,
                                       [&](uint32_t v) { return window16_dw(dw, ps + 16u * v); });
      else
        bad = utf8_check_frame((uint64_t)ps, fe, g, G,
                               [&](uint64_t c) { return img[c]; },
                               [&](uint64_t x) { return dw[(x >> 2) - 1u]; });  // x = 0 reads the guard
    }
  }
  for (uint32_t m = G >> 1; m > 0; m >>= 1) bad |= __shfl_xor(bad, (int)m, 64);
  if (g == 0 && q < Tv) a.valid[p0 + q] = bad ? 0 : 1;
}

// ---- small frames (the reference's 1-character datagrams) ------------------
// Packed payloads with a mean length hint under kSmallHint bytes: frames of
// 5-20 bytes share every aligned 16-B chunk with their neighbours, so the
// per-packet vector kernel writes them bytewise, and the offset scan's last
// pass plus the encode launch re-read the offsets.  Here one kernel per tile
// of T = 256 * FPT packets does the scan's last pass and the framing:
//   loads    the tile's lengths and header table (coalesced), and its packed
//            payload run [fo0 - p0*H, fo_end - (p0+T)*H) into LDS, where fo0 /
//            fo_end are the scan's block bases (passes 1-2 ran over the same
//            tiles);
//   scan     lengths -> tile-relative frame offsets (block scan), written to
//            frame_off with coalesced stores;
//   frames   each thread builds its FPT consecutive frames in an LDS image of
//            the tile's output run (header word + payload bytes, LE16 sums on
//            the way), then the block stores the run as aligned 16-B vectors
//            (only the two edge chunks, shared with the neighbour tiles, bytewise).
// A tile whose run outgrows the LDS budget (a burst far above the hint)
// encodes its packets with the per-packet vector path inside the launch.
constexpr uint32_t kSmallHint = 16;

__host__ __device__ inline uint32_t small_lds_off_seq(uint32_t T) { return ((8u * T + 4u + 15u) & ~15u); }
__host__ __device__ inline uint32_t small_lds_off_pay(uint32_t T) {
  return small_lds_off_seq(T) + ((7u * T + 15u) & ~15u);  // seq u16, ack u16, flags u8, csum u16
}
__host__ __device__ inline uint32_t small_lds_off_out(uint32_t T, uint32_t cap) {
  return small_lds_off_pay(T) + cap + 32u;
}
__host__ __device__ inline uint32_t small_out_cap(uint32_t T, uint32_t cap, uint32_t H) { return cap + T * H + 16u; }

// FUSED: `sums` are the raw pass-1 block sums (with their status bits) and
// every block finds its own base (the sum of the sums before it) and the
// status from all of them -- nb <= kSmallFusedTiles, so that is a few KiB of
// L2 reads per block -- instead of a one-workgroup pass between the two
// launches.  Otherwise `sums` are pass 2's exclusive bases.
// SINGLE (a checked call of packed payloads that is one tile, e.g. a
// recvmmsg batch of <= 1024 datagrams): no pass 1 at all.  The tile's base
// is 0 and its payload run is the whole payload buffer, whose size the call
// states, so the run loads before the scan; the block scan's total then gives
// frame_off[n] and the checks pass 1 would have made.  One launch per call.
// FIXED (a fixed-stride batch, frame_off null): tile t's base is fo_at(t T),
// every length is stride - H; no scan, no offsets written, one launch.
constexpr uint64_t kSmallFusedTiles = 2048;
// FUSED_NIB: FUSED with pass 1's length codes (VarlenArgs::len_code: 2 bits a
// packet at 4 packets a thread, 4 at 2, offsets from the call's length hint;
// the all-ones code reads len[] for that packet): len[] leaves HBM once per
// call instead of twice.
enum SmallMode { kSmallBases = 0, kSmallFused = 1, kSmallSingle = 2, kSmallFixed = 3, kSmallFusedNib = 4 };

template <int H, uint32_t FPT, int MODE>
__global__ void __launch_bounds__(kBlock) encode_varlen_small_kernel(VarlenArgs a, const uint64_t* sums,
                                                                     uint64_t nb, ScanCheck chk) {
  constexpr bool FUSED = MODE == kSmallFused || MODE == kSmallFusedNib, SINGLE = MODE == kSmallSingle,
                 FIXED = MODE == kSmallFixed, NIB = MODE == kSmallFusedNib;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr uint32_t T = kBlock * FPT;
  const uint32_t tid = threadIdx.x;
  const uint32_t cap = a.small_cap;
  uint32_t* s_len = reinterpret_cast<uint32_t*>(lds);        // [T]
  uint32_t* s_off = s_len + T;                               // [T + 1], tile-relative
  uint16_t* s_seq = reinterpret_cast<uint16_t*>(lds + small_lds_off_seq(T));
  uint16_t* s_ack = s_seq + T;
  uint16_t* s_cs = s_ack + T;
  uint8_t* s_flags = reinterpret_cast<uint8_t*>(s_cs + T);
  unsigned char* pay = lds + small_lds_off_pay(T);
  unsigned char* img = lds + small_lds_off_out(T, cap);
  __shared__ uint32_t s_wave32[kBlock / 64];

  const uint64_t tile = a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t p0 = tile * T;
  const uint32_t Tv = a.n - p0 < T ? (uint32_t)(a.n - p0) : T;
  uint64_t fo0, fo_end;
#if RUDP_TOOLS
  const uint64_t t_start = a.trace ? (uint64_t)wall_clock64() : 0ull;  // diagnostics
#endif
  // The tile's lengths and header table (coalesced) go out first: they do not
  // depend on the tile's base, so their round trip overlaps the base's.
  uint32_t lv[FPT], sq[FPT], ak[FPT], fl[FPT];
#pragma unroll
  for (uint32_t j = 0; j < FPT; ++j) {
    const uint32_t q = j * kBlock + tid;
    lv[j] = sq[j] = ak[j] = fl[j] = 0;
    if (q < Tv) {
      lv[j] = FIXED ? (uint32_t)a.stride - (uint32_t)H : NIB ? 0u : a.len[p0 + q];
      sq[j] = a.seq_in[p0 + q];
      ak[j] = a.ack_in[p0 + q];
      fl[j] = a.flags_in[p0 + q];
    }
  }
  uint32_t code = 0;
  if (NIB) code = a.len_code[tile * kBlock + tid];  // (decoded after the base's round trip)
  if (FUSED) {
    __shared__ uint64_t s_pre[kBlock / 64], s_all[kBlock / 64];
    __shared__ uint32_t s_bits;
    if (tid == 0) s_bits = 0;
    uint64_t pre = 0, all = 0;
    uint32_t bits = 0;
    for (uint64_t c = tid; c < nb; c += kBlock) {
      const uint64_t v = sums[c];
      all += v & kSumMask;
      pre += c < tile ? (v & kSumMask) : 0u;
      bits |= (uint32_t)(v >> kSumBitsShift);
    }
    for (int m = 32; m > 0; m >>= 1) {
      pre += __shfl_xor(pre, m, 64);
      all += __shfl_xor(all, m, 64);
    }
    __syncthreads();  // s_bits initialised
    if (bits) atomicOr(&s_bits, bits);
    if ((tid & 63u) == 0) {
      s_pre[tid >> 6] = pre;
      s_all[tid >> 6] = all;
    }
    __syncthreads();
    pre = all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64; ++w) {
      pre += s_pre[w];
      all += s_all[w];
    }
    uint32_t st = s_bits;
    if (chk.status) {
      if (!chk.payload_off && all - a.n * (uint64_t)H != chk.payload_bytes) st |= RUDP_ST_PAYLOAD;
      if (all > chk.frames_cap) st |= RUDP_ST_FRAMES_CAP;
    }
    if (tile == 0 && tid == 0) {
      const_cast<uint64_t*>(a.frame_off)[a.n] = all;
      if (chk.status) *chk.status = st;
    }
    if (chk.status && st) return;  // uniform: every block computes the same status
    fo0 = pre;
    fo_end = pre + (sums[tile] & kSumMask);
  } else if (SINGLE) {
    fo0 = 0;
    fo_end = 0;  // from the scan below
  } else if (FIXED) {
    fo0 = fo_at<true>(a, p0);
    fo_end = fo_at<true>(a, p0 + Tv);
  } else {
    fo0 = sums[tile];
    fo_end = p0 + T < a.n ? sums[tile + 1] : a.frame_off[a.n];
    if (call_failed(a.status)) return;
  }
#if RUDP_TOOLS
  const uint64_t t_base = a.trace ? (uint64_t)wall_clock64() : 0ull;
#endif
  if (NIB) {  // the lengths from pass 1's codes (an all-ones code: len[] for that packet)
    constexpr uint32_t B = 8u / FPT, M = (1u << B) - 1u;
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) {
      const uint32_t q = j * kBlock + tid;
      const uint32_t c = (code >> (B * j)) & M;
      lv[j] = q < Tv ? (c < M ? a.len_code_base + c : a.len[p0 + q]) : 0u;
    }
  }
  const uint64_t po0 = fo0 - p0 * (uint64_t)H + (FIXED ? a.po_delta : 0ull);
  const uint64_t po_end = SINGLE ? chk.payload_bytes : fo_end - (p0 + Tv) * (uint64_t)H + (FIXED ? a.po_delta : 0ull);
  const uint64_t A = po0 & ~15ull, OA = fo0 & ~15ull;
  const uint64_t prun = ((po_end + 15u) & ~15ull) - A;
  uint64_t orun = ((fo_end + 15u) & ~15ull) - OA;
  bool fits = prun <= cap && (SINGLE || orun <= small_out_cap(T, cap, H));

  // ---- loads: the payload run; lengths and header table to LDS -------------
  {
    if (fits) {
      const u32x4* src = reinterpret_cast<const u32x4*>(a.payload + A);
      u32x4* dst = reinterpret_cast<u32x4*>(pay);
      const uint32_t nvec = (uint32_t)(prun >> 4);
      for (uint32_t v0 = tid; v0 < nvec; v0 += 4u * kBlock) {
        u32x4 r[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
          if (v0 + u * kBlock < nvec) r[u] = __builtin_nontemporal_load(src + v0 + u * kBlock);
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
          if (v0 + u * kBlock < nvec) dst[v0 + u * kBlock] = r[u];
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) {
      const uint32_t q = j * kBlock + tid;
      s_len[q] = lv[j];
      s_seq[q] = (uint16_t)sq[j];
      s_ack[q] = (uint16_t)ak[j];
      s_flags[q] = (uint8_t)fl[j];
    }
  }
  __syncthreads();

  // ---- the scan's last pass: tile-relative offsets, frame_off ---------------
  {
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t i = 0; i < FPT; ++i) {
      const uint32_t q = tid * FPT + i;
      mine += q < Tv ? s_len[q] + (uint32_t)H : 0u;
    }
    uint32_t total = 0;  // (at most 256 * FPT * 65542)
    uint32_t run = FIXED ? tid * FPT * (uint32_t)a.stride : block_exclusive_scan32(mine, &total, s_wave32);
#pragma unroll
    for (uint32_t i = 0; i < FPT; ++i) {
      const uint32_t q = tid * FPT + i;
      s_off[q] = run;
      run += q < Tv ? s_len[q] + (uint32_t)H : 0u;
    }
    if (SINGLE) {  // the checks pass 1 would have made, and frame_off[n]
      uint32_t big = 0;
#pragma unroll
      for (uint32_t j = 0; j < FPT; ++j) big |= lv[j] > kMaxPayload ? 1u : 0u;
      uint32_t st = __syncthreads_or((int)big) ? RUDP_ST_LEN : 0u;
      if (total - a.n * (uint64_t)H != chk.payload_bytes) st |= RUDP_ST_PAYLOAD;
      if (total > chk.frames_cap) st |= RUDP_ST_FRAMES_CAP;
      if (tid == 0) {
        const_cast<uint64_t*>(a.frame_off)[a.n] = total;
        if (chk.status) *chk.status = st;
      }
      if (st) return;  // uniform
      fo_end = total;
      orun = ((fo_end + 15u) & ~15ull) - OA;
      fits = fits && orun <= small_out_cap(T, cap, H);
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < FPT && !FIXED; ++j) {
    const uint32_t q = j * kBlock + tid;
    if (q < Tv) const_cast<uint64_t*>(a.frame_off)[p0 + q] = fo0 + s_off[q];
  }
  if (!fits) {  // uniform: per-packet vector path, offsets from LDS
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) {
      const uint32_t q = j * kBlock + tid;
      encode_varlen_packet<H, FIXED>(a, p0 + q, q < Tv, 0u, 0u, q < Tv ? fo0 + s_off[q] : 0ull);
    }
    return;
  }

  // ---- frames into the LDS image of the output run ---------------------------
  // (lane-strided: neighbouring lanes build neighbouring frames, so their LDS
  // byte stores land a frame apart instead of FPT frames apart)
  const uint32_t lead = (uint32_t)(fo0 - OA);   // output bytes before fo0 in the first chunk
  const uint32_t pshift = (uint32_t)(po0 - A);  // LDS offset of payload byte po0
#pragma unroll
  for (uint32_t i = 0; i < FPT; ++i) {
    const uint32_t q = i * kBlock + tid;
    if (q < Tv) {
      const uint32_t Lq = s_len[q], fs = s_off[q];
      const unsigned char* src = pay + pshift + fs - q * (uint32_t)H;
      unsigned char* dst = img + lead + fs;
      uint32_t sum = 0;
      for (uint32_t j = 0; j < Lq; ++j) {
        const uint32_t b = src[j];
        sum += (j & 1u) ? (b << 8) : b;  // LE16 words: payload sits at an odd frame offset
        dst[H + j] = (unsigned char)b;
      }
      const uint32_t sq = s_seq[q], ak = s_ack[q], fl = s_flags[q];
      const uint32_t c = packet_csum(sum, sq, ak, fl);
      const uint64_t h = pack_header<H>(sq, ak, fl, c);
#pragma unroll
      for (int k = 0; k < H; ++k) dst[k] = (unsigned char)(h >> (8 * k));
      s_cs[q] = (uint16_t)c;
    }
  }
  __syncthreads();
  if (a.csum) {
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) {
      const uint32_t q = j * kBlock + tid;
      if (q < Tv) a.csum[p0 + q] = s_cs[q];
    }
  }
  // ---- the output run: aligned 16-B vectors, edge chunks bytewise ------------
  const uint32_t end = (uint32_t)(fo_end - OA);
  const uint32_t nch = (uint32_t)(orun >> 4);
  const u32x4* img16 = reinterpret_cast<const u32x4*>(img);
  unsigned char* out = a.frames + OA;
  for (uint32_t c = tid; c < nch; c += kBlock) {
    const uint32_t X = c << 4;
    if (X >= lead && X + 16u <= end) {
      __builtin_nontemporal_store(img16[c], reinterpret_cast<u32x4*>(out + X));
    } else {
      const uint32_t lo = X > lead ? X : lead, hi = X + 16u < end ? X + 16u : end;
      for (uint32_t b = lo; b < hi; ++b) out[b] = img[b];
    }
  }
#if RUDP_TOOLS
  if (a.trace) {  // diagnostics: {start, base known, end, XCC} per tile (tools/small_timeline.py)
    __syncthreads();
    if (tid == 0) {
      u32x4* rec = reinterpret_cast<u32x4*>(a.trace + 4ull * tile);
      rec[0] = make_u32x4(t_start, t_base);
      rec[1] = make_u32x4((uint64_t)wall_clock64(), __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20));
    }
  }
#endif
}

template <int H, uint32_t FPT>
int launch_small_fpt(const VarlenArgs& args, const uint64_t* sums, uint64_t nb, const ScanCheck& chk,
                     bool fused, hipStream_t stream) {
  constexpr uint32_t T = kBlock * FPT;
  const size_t lds = small_lds_off_out(T, args.small_cap) + small_out_cap(T, args.small_cap, H) + 32u;
  const int mode = sums == nullptr ? kSmallSingle : fused ? (args.len_code ? kSmallFusedNib : kSmallFused) : kSmallBases;
  const void* fn = mode == kSmallSingle ? reinterpret_cast<const void*>(&encode_varlen_small_kernel<H, FPT, kSmallSingle>)
                 : mode == kSmallFusedNib ? reinterpret_cast<const void*>(&encode_varlen_small_kernel<H, FPT, kSmallFusedNib>)
                 : mode == kSmallFused  ? reinterpret_cast<const void*>(&encode_varlen_small_kernel<H, FPT, kSmallFused>)
                                        : reinterpret_cast<const void*>(&encode_varlen_small_kernel<H, FPT, kSmallBases>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  if (mode == kSmallSingle)
    hipLaunchKernelGGL((encode_varlen_small_kernel<H, FPT, kSmallSingle>), dim3(1), dim3(kBlock), lds, stream,
                       args, sums, nb, chk);
  else if (mode == kSmallFusedNib)
    hipLaunchKernelGGL((encode_varlen_small_kernel<H, FPT, kSmallFusedNib>), dim3((uint32_t)nb), dim3(kBlock), lds,
                       stream, args, sums, nb, chk);
  else if (mode == kSmallFused)
    hipLaunchKernelGGL((encode_varlen_small_kernel<H, FPT, kSmallFused>), dim3((uint32_t)nb), dim3(kBlock), lds,
                       stream, args, sums, nb, chk);
  else
    hipLaunchKernelGGL((encode_varlen_small_kernel<H, FPT, kSmallBases>), dim3((uint32_t)nb), dim3(kBlock), lds,
                       stream, args, sums, nb, chk);
  return (int)hipGetLastError();
}

// 2 or 4 packets per thread (the measured choice by hint); 1 and 8 in the tools build's sweeps.
template <int H>
int launch_small_any(const VarlenArgs& args, const uint64_t* sums, uint64_t nb, const ScanCheck& chk, bool fused,
                     hipStream_t stream) {
#if RUDP_TOOLS
  if (args.small_fpt == 1) return launch_small_fpt<H, 1>(args, sums, nb, chk, fused, stream);
  if (args.small_fpt == 8) return launch_small_fpt<H, 8>(args, sums, nb, chk, fused, stream);
#endif
  return args.small_fpt == 2 ? launch_small_fpt<H, 2>(args, sums, nb, chk, fused, stream)
                             : launch_small_fpt<H, 4>(args, sums, nb, chk, fused, stream);
}

template <int H, uint32_t FPT>
int launch_stride_small_fpt(const VarlenArgs& args, hipStream_t stream) {
  constexpr uint32_t T = kBlock * FPT;
  const size_t lds = small_lds_off_out(T, args.small_cap) + small_out_cap(T, args.small_cap, H) + 32u;
  const void* fn = reinterpret_cast<const void*>(&encode_varlen_small_kernel<H, FPT, kSmallFixed>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const uint64_t nb = (args.n + T - 1) / T;
  hipLaunchKernelGGL((encode_varlen_small_kernel<H, FPT, kSmallFixed>), dim3((uint32_t)nb), dim3(kBlock), lds, stream,
                     args, nullptr, nb, ScanCheck{});
  return (int)hipGetLastError();
}

int launch_encode_stride_small(const VarlenArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  if (args.small_fpt == 2)
    return layout == 7 ? launch_stride_small_fpt<7, 2>(args, stream) : launch_stride_small_fpt<5, 2>(args, stream);
  return layout == 7 ? launch_stride_small_fpt<7, 4>(args, stream) : launch_stride_small_fpt<5, 4>(args, stream);
}

// Copy-out of fixed-stride frames that miss the fixed-length decode tile
// (launch_copy_payloads): a workgroup stages the run of its T frames in LDS
// from the aligned-down start (bytes before the caller's first frame are
// staged, never written) and writes the run [p0 L, (p0 + T) L) of `out` as
// aligned 16-B chunks, each gathered from the payloads it covers -- one
// byte-shifted LDS window per payload, one or two per chunk at L >= 16 -- the
// two chunks shared with the neighbour tiles bytewise.
constexpr uint32_t kCopyRun = 32768;  // frame bytes a tile stages (at least one frame)
__global__ void __launch_bounds__(kBlock) copy_payloads_kernel(const unsigned char* frames, uint64_t fo_base,
                                                                uint32_t F, uint32_t H, uint64_t n, uint32_t T,
                                                                unsigned char* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* img = lds + kVTGuard;  // the run, a guard before and after it
  const uint32_t tid = threadIdx.x;
  const uint64_t p0 = (uint64_t)(xcd_tile(blockIdx.x, gridDim.x)) * T;
  const uint32_t Tv = n - p0 < T ? (uint32_t)(n - p0) : T;
  const uint32_t L = F - H;
  const uint64_t fo0 = fo_base + p0 * F, fo_end = fo0 + (uint64_t)Tv * F;
  const uint64_t A = fo0 & ~15ull;
  const uint32_t nvec = (uint32_t)((((fo_end + 15u) & ~15ull) - A) >> 4);
  u32x4* dst = reinterpret_cast<u32x4*>(img);
  for (uint32_t v0 = tid; v0 < nvec; v0 += 4u * kBlock) {
    u32x4 r[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (v0 + u * kBlock < nvec) r[u] = load16_guarded(frames, A + 16ull * (v0 + u * kBlock), fo_end);
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (v0 + u * kBlock < nvec) dst[v0 + u * kBlock] = r[u];
  }
  __syncthreads();
  const uint32_t* lds_dw = reinterpret_cast<const uint32_t*>(lds);
  const uint32_t d0 = kVTGuard + (uint32_t)(fo0 - A) + H;  // LDS offset of the tile's first payload byte
  unsigned char* o = out + p0 * (uint64_t)L;     // the tile's output run [0, nb)
  const uint32_t nb = Tv * L;
  const uint32_t lead = (uint32_t)(-(uintptr_t)o) & 15u;  // bytes before its first aligned chunk
  const uint32_t nch = nb > lead ? (nb - lead + 15u) / 16u + 1u : 1u;  // chunk 0 is the head [0, lead)
  for (uint32_t c = tid; c < nch; c += kBlock) {
    // chunk c covers run bytes [x, x + 16) of which [b_lo, b_hi) are owned
    const int x = c == 0 ? (int)lead - 16 : (int)lead + 16 * (int)(c - 1u);
    const int b_lo = x < 0 ? -x : 0;
    const int b_hi = x + 16 <= (int)nb ? 16 : (int)nb - x;
    if (b_hi <= b_lo) continue;
    uint64_t lo = 0, hi = 0;
    uint32_t y = (uint32_t)(x + b_lo);
    uint32_t q = y / L, j = y - q * L;
    for (int b = b_lo; b < b_hi;) {
      const int take = (int)(L - j) < b_hi - b ? (int)(L - j) : b_hi - b;
      // chunk byte b is payload q's byte j, at LDS offset d0 + q F + j
      const u32x4 w = window16_dw(lds_dw, d0 + q * F + j - (uint32_t)b);  // (>= kVTGuard - 15)
      lo |= lo64(w) & byte_mask(b, b + take);
      hi |= hi64(w) & byte_mask(b - 8, b + take - 8);
      b += take;
      ++q;
      j = 0;
    }
    if (b_lo == 0 && b_hi == 16) {
      __builtin_nontemporal_store(make_u32x4(lo, hi), reinterpret_cast<u32x4*>(o + x));
    } else {
      for (int b = b_lo; b < b_hi; ++b) o[x + b] = (unsigned char)(b < 8 ? lo >> (8 * b) : hi >> (8 * (b - 8)));
    }
  }
}

int launch_copy_payloads(const unsigned char* frames, uint32_t F, uint32_t H, uint64_t n, unsigned char* out,
                         hipStream_t stream) {
  if (n == 0 || F <= H) return 0;
  const uint64_t fmis = reinterpret_cast<uintptr_t>(frames) & 15u;
  uint32_t T = kCopyRun / F;
  if (T < 1u) T = 1u;
  if (T > 4096u) T = 4096u;
  const size_t lds = 2u * kVTGuard + (((size_t)T * F + 31u) & ~size_t(15));
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&copy_payloads_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const uint64_t blocks = (n + T - 1) / T;
  hipLaunchKernelGGL(copy_payloads_kernel, dim3((uint32_t)blocks), dim3(kBlock), lds, stream, frames - fmis, fmis, F,
                     H, n, T, out);
  return (int)hipGetLastError();
}

int launch_encode_varlen_small(const VarlenArgs& args, const ScanCheck& chk, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  const uint32_t fpt = args.small_fpt;
  const uint64_t T = (uint64_t)kBlock * fpt;
  const uint64_t nb = (args.n + T - 1) / T;
  // one tile of a checked call (packed payloads: the small path's only form): one launch, no pass 1
  if (nb == 1 && chk.status && tuning().varlen_small_single)
    return layout == 7 ? launch_small_any<7>(args, nullptr, 1, chk, false, stream)
                       : launch_small_any<5>(args, nullptr, 1, chk, false, stream);
  uint64_t* sums = nullptr;
  hipError_t e = stream_scratch(reinterpret_cast<void**>(&sums), nb * sizeof(uint64_t), stream, kScratchSums);
  if (e != hipSuccess) return (int)e;
  // pass 1, then either the framing kernel finds its own base (two launches)
  // or pass 2 runs between them (three)
  const bool fused = tuning().varlen_small_fused && nb <= kSmallFusedTiles;
  VarlenArgs a = args;
  if (fused && tuning().varlen_small_nib && (fpt == 2u || fpt == 4u)) {
    void* codes = nullptr;  // (the records' slot: the MTU tile's, never used by a small-frame call)
    e = stream_scratch(&codes, nb * kBlock, stream, kScratchRecords);
    if (e != hipSuccess) return (int)e;
    a.len_code = static_cast<const uint8_t*>(codes);
    // codes are offsets from the caller's length hint: 2-bit codes (4 packets a
    // thread) cover hint .. hint + 2, 4-bit ones hint - 7 .. hint + 7
    const uint32_t h = args.len_code_base;
    a.len_code_base = fpt == 4u ? h : (h > 7u ? h - 7u : 0u);
  }
  scan_block_sums(args.len, args.n, (uint32_t)layout, fpt, sums, chk, stream, 0u, 0u, const_cast<uint8_t*>(a.len_code),
                  a.len_code_base);
  if (!fused) scan_block_bases(sums, nb, const_cast<uint64_t*>(args.frame_off), args.n, (uint32_t)layout, chk, stream);
  return layout == 7 ? launch_small_any<7>(a, sums, nb, chk, fused, stream)
                     : launch_small_any<5>(a, sums, nb, chk, fused, stream);
}

// Small-frame decode: a tile of T = 256 * FPT consecutive frames (the
// reference's 6-9 B datagrams) is one contiguous run; its offsets and the run
// stream into LDS, then each lane parses FPT frames (lane-strided, so the
// per-frame outputs leave as coalesced stores), summing a frame's LDS dwords
// by address parity.  A run over the LDS budget decodes per frame (G = 1).
// One frame by one lane, straight from HBM, byte by byte: the checked rule
// on its true offsets (the small-frame tile's frames whose offsets fall
// outside its staged run; rare).
template <int H, bool U8, bool FX>
__device__ __forceinline__ void decode_varlen_frame_lane(const VarlenArgs& a, uint64_t p) {
  const uint64_t fo = fo_at<FX>(a, p), fe = fo_at<FX>(a, p + 1);
  if (fo > fe || fe > frames_limit<FX>(a)) {
    decode_varlen_reject(a, p);
    return;
  }
  const uint64_t F64 = fe - fo;
  const uint32_t F = F64 < 0xFFFFFFFFull ? (uint32_t)F64 : 0xFFFFFFFFu;
  uint64_t acc = 0;
  for (uint64_t j = (uint64_t)H; j < F64; ++j) acc += ((j - H) & 1u) ? (uint32_t)a.frames[fo + j] << 8 : a.frames[fo + j];
  const uint32_t sum = fold_keep(acc);
  uint32_t d[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < 7 && i < F; ++i) d[i >> 2] |= (uint32_t)a.frames[fo + i] << (8 * (i & 3));
  u32x4 h;
  h.x = d[0];
  h.y = d[1];
  h.z = 0;
  h.w = 0;
  if (U8)
    a.valid[p] = F > (uint32_t)H && utf8_check_bytes((uint32_t)H, F, [&](uint32_t i) { return (uint32_t)a.frames[fo + i]; })
                     ? 0 : 1;
  decode_varlen_finish<H>(a, p, F, sum, h);
}

template <int H, uint32_t FPT, bool U8, bool FX>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) decode_varlen_small_kernel(VarlenArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr uint32_t T = kBlock * FPT;
  const uint32_t tid = threadIdx.x;
  uint32_t* s_fo = reinterpret_cast<uint32_t*>(lds);                    // [T + 1]
  unsigned char* img = lds + ((4u * (T + 1u) + 15u) & ~15u);            // the run, then a guard
  const uint64_t p0 = (uint64_t)(a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x) * T;
  const uint32_t Tv = a.n - p0 < T ? (uint32_t)(a.n - p0) : T;
  const uint64_t fo0 = fo_at<FX>(a, p0), fo_end = fo_at<FX>(a, p0 + Tv);
  const uint64_t total = frames_limit<FX>(a);
  const uint64_t A = fo0 & ~15ull;
  const uint64_t run = ((fo_end + 15u) & ~15ull) - A;
  if (fo0 > fo_end || fo_end > total || run > a.small_cap) {  // uniform: per-frame path, two lanes each
#pragma unroll
    for (uint32_t j = 0; j < 2u * FPT; ++j) {  // (the header comes from the pair's two first chunks)
      const uint32_t q = j * (kBlock / 2u) + (tid >> 1);
      decode_varlen_frame<H, U8, U8 ? 4 : 0, FX>(a, p0 + q, q < Tv, tid & 1u, 1u);
    }
    return;
  }
  {
    uint32_t fo_r[FPT], fo_last = 0;
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) {
      const uint32_t q = j * kBlock + tid;
      const uint64_t o = q <= Tv ? fo_at<FX>(a, p0 + q) : A;
      fo_r[j] = o - A <= fo_end - A ? (uint32_t)(o - A) : 0xFFFFFFFFu;  // outside [A, fo_end]
    }
    if (tid == 0) fo_last = (uint32_t)(fo_end - A);
    const uint32_t nvec = (uint32_t)(run >> 4);
    u32x4* dst = reinterpret_cast<u32x4*>(img);
    for (uint32_t v0 = tid; v0 < nvec; v0 += 4u * kBlock) {
      u32x4 r[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (v0 + u * kBlock < nvec) r[u] = load16_guarded(a.frames, A + 16ull * (v0 + u * kBlock), total);
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (v0 + u * kBlock < nvec) dst[v0 + u * kBlock] = r[u];
    }
#pragma unroll
    for (uint32_t j = 0; j < FPT; ++j) s_fo[j * kBlock + tid] = fo_r[j];
    if (tid == 0) s_fo[Tv] = fo_last;
  }
  __syncthreads();
  const uint32_t* dw = reinterpret_cast<const uint32_t*>(img);
  const uint32_t lim = (uint32_t)(fo_end - A);
  uint32_t fallback = 0;  // this lane's frames whose offsets leave the run (see the tile kernel)
#pragma unroll
  for (uint32_t j = 0; j < FPT; ++j) {
    const uint32_t q = j * kBlock + tid;
    if (q >= Tv) continue;
    const uint32_t fs = s_fo[q], fe = s_fo[q + 1];
    if (fs > fe || fe > lim) {  // out of order or outside the run: after the loop, from HBM
      fallback |= 1u << j;
      continue;
    }
    uint32_t ev = 0, od = 0;  // byte sums at even / odd offsets (A is even)
    uint32_t hib = 0;         // U8: high bits of the payload bytes
    const uint32_t ps = fs + (uint32_t)H;
    if (fe > ps) {  // the payload's dwords, the edge ones masked to it
      const uint32_t w0 = ps >> 2, w1 = (fe - 1u) >> 2;
      for (uint32_t w = w0; w <= w1; ++w) {
        uint32_t v = dw[w];
        if (w == w0 || w == w1) {
          const int lo = (int)ps - (int)(4u * w), hi = (int)fe - (int)(4u * w);
          v &= (uint32_t)byte_mask(lo, hi < 4 ? hi : 4);
        }
        if (U8) hib |= v;
        ev = even_bytes_acc(v, ev);
        od = odd_bytes_acc(v, od);
      }
    }
    if (U8) {
      const unsigned char* ib = img;
      a.valid[p0 + q] = (hib & 0x80808080u) && utf8_check_bytes(ps, fe, [&](uint32_t i) { return (uint32_t)ib[i]; })
                            ? 0 : 1;
    }
    const uint32_t sum = (fs & 1u) ? (ev + (od << 8)) : ((ev << 8) + od);
    decode_varlen_finish<H>(a, p0 + q, fe - fs, sum, window16_dw(dw, fs));
  }
#pragma unroll 1
  for (uint32_t j = 0; j < FPT; ++j)  // one lane per such frame, straight from HBM (rare)
    if (fallback & (1u << j)) decode_varlen_frame_lane<H, U8, FX>(a, p0 + j * kBlock + tid);
}

template <int H, uint32_t FPT, bool U8, bool FX>
int launch_decode_small_fpt(const VarlenArgs& args, hipStream_t stream) {
  constexpr uint32_t T = kBlock * FPT;
  const size_t lds = ((4u * (T + 1u) + 15u) & ~15u) + (size_t)args.small_cap + 32u;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_varlen_small_kernel<H, FPT, U8, FX>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const uint64_t blocks = (args.n + T - 1) / T;
  hipLaunchKernelGGL((decode_varlen_small_kernel<H, FPT, U8, FX>), dim3((uint32_t)blocks), dim3(kBlock), lds, stream,
                     args);
  return (int)hipGetLastError();
}

template <int H, bool U8, bool FX>
int launch_decode_small(const VarlenArgs& args, hipStream_t stream) {
#if RUDP_TOOLS  // 4 frames per thread is the measured choice; 1, 2 and 8 for sweeps
  if constexpr (!FX) {
    switch (args.small_fpt) {
      case 1: return launch_decode_small_fpt<H, 1, U8, FX>(args, stream);
      case 2: return launch_decode_small_fpt<H, 2, U8, FX>(args, stream);
      case 8: return launch_decode_small_fpt<H, 8, U8, FX>(args, stream);
      default: break;
    }
  }
#endif
  return launch_decode_small_fpt<H, 4, U8, FX>(args, stream);
}

// Dynamic LDS of one varlen encode tile whose arrays hold Tl packets.
static size_t varlen_tile_lds(uint32_t Tl, uint32_t cap, uint32_t H, uint32_t vhc) {
  size_t b = vt_pay_off(Tl, cap, H, vhc == 2u ? 1u : 0u) + 2u * kVTGuard + cap;
  if (vhc) b = ((b + 15u) & ~size_t(15)) + 32u * Tl;
  return b;
}

// Tiles of the varlen encode kernel (waves-per-SIMD floor W) one CU holds at
// `lds` bytes of dynamic LDS, from the runtime's occupancy calculation (its LDS
// allocation granule and limit, the kernel's registers), cached per (device,
// size): a byte count over 160 KiB misjudged it (1M x 1472 B byte tiles at
// 31.8 KB ran 4 per CU, not 5).  Every launch asks; a thread's last answer is
// kept thread-locally, so only a new size takes the shared map's lock.
template <int H, int W>
static int vt_occupancy(size_t lds) {
  int device = 0;
  (void)hipGetDevice(&device);
  const uint64_t key = ((uint64_t)(uint32_t)device << 40) | (uint64_t)lds;
  thread_local uint64_t last_key = ~0ull;
  thread_local int last_nb = 0;
  if (key == last_key) return last_nb;
  static std::mutex mu;
  static std::map<uint64_t, int> cache;
  int nb = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) {
      nb = it->second;
    } else {
      const void* fn = reinterpret_cast<const void*>(&encode_varlen_tile_kernel<H, W>);
      if (lds > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, (int)kBlock, lds) != hipSuccess || nb < 1)
        nb = (int)((160u * 1024u) / lds);  // (no answer: the plain byte count)
      cache.emplace(key, nb);
    }
  }
  last_key = key;
  last_nb = nb;
  return nb;
}

// The kernel's register budget to match its LDS occupancy: 94 VGPRs (5 waves
// per SIMD) unconstrained, so tiles small enough for 6-7 per CU ask the
// allocator for that many waves (a few spills in the per-packet fallback):
// 1M x 512 B 0.259 -> 0.233 ms (W = 7), x 256 B 0.163 -> 0.153 (W = 6).  At 5
// tiles per CU and fewer it stays unconstrained: spills cost ragged batches
// whose tiles take the fallback (lengths uniform in [0, 2944] at W = 7: 0.80 ->
// 1.00 ms; profiles/r01/sweeps/varlen_waves.json).
template <int H>
static int vt_waves(size_t lds) {
  if (vt_occupancy<H, 7>(lds) >= 7) return 7;
  if (vt_occupancy<H, 6>(lds) >= 6) return 6;
  return 1;
}

template <int H>
static int vt_tiles_per_cu(size_t lds) {
  const int w = vt_waves<H>(lds);
  return w == 7 ? vt_occupancy<H, 7>(lds) : w == 6 ? vt_occupancy<H, 6>(lds) : vt_occupancy<H, 1>(lds);
}

// Byte tiles of bt_slots packets as an alternative to packet tiles of tile_T:
// only for packet tiles of 16 or fewer (hints from 1 KiB: below, ragged
// lengths rarely overflow and byte tiles lost, lengths uniform in [0, 512]
// 0.204 -> 0.248 ms), where their arrays leave the tiles per CU unchanged
// (1M x 512 B: 64 slots would take 7 packet tiles per CU to 6, 8% slower) --
// fewer slots, down to min_slots, when that keeps them so -- and their grid
// is at most 5% larger (the surplus workgroups of the form not taken still
// occupy LDS for a round trip: 4000-B hints, 50% slower).
bool varlen_btile_ok(uint32_t tile_T, uint32_t* bt_slots, uint32_t min_slots, uint32_t cap, uint32_t cap_packet,
                     uint32_t H, uint32_t vhc, uint64_t packet_tiles, uint64_t spans) {
  if (tile_T > 16u) return false;
  auto per_cu = [&](uint32_t Tl, uint32_t c) {
    const size_t lds = varlen_tile_lds(Tl, c, H, vhc);
    return H == 7u ? vt_tiles_per_cu<7>(lds) : vt_tiles_per_cu<5>(lds);
  };
  const int want = per_cu(tile_T, cap_packet);
  uint32_t slots = *bt_slots;
  while (slots > tile_T && slots > min_slots && per_cu(slots, cap) < want) --slots;
  if (per_cu(slots > tile_T ? slots : tile_T, cap) < want) return false;
  *bt_slots = slots;
  return spans * 20u <= packet_tiles * 21u;
}

template <int H, int W, bool FX>
int launch_varlen_tile_w(const VarlenArgs& args, size_t lds, uint64_t blocks, hipStream_t stream) {
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&encode_varlen_tile_kernel<H, W, FX>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((encode_varlen_tile_kernel<H, W, FX>), dim3((uint32_t)blocks), dim3(kBlock), lds, stream, args);
  return (int)hipGetLastError();
}

template <int H, bool FX>
int launch_varlen_tile(const VarlenArgs& in, hipStream_t stream) {
  VarlenArgs args = in;
  uint64_t blocks = (args.n + args.tile_T - 1) / args.tile_T;
  if (args.span_rec && args.span_count > blocks) blocks = args.span_count;
  const uint32_t Tl = args.span_rec && args.bt_slots > args.tile_T ? args.bt_slots : args.tile_T;
  args.tile_Tl = Tl;
  // The coded map costs 1 B more per output chunk.  Where that would leave
  // fewer than 4 tiles per CU (1M x 1024 B: 4 -> 3, 9% slower) the u8 map is
  // used instead (profiles/r01/sweeps/varlen_coded_map.json).
  if (args.vhc == 2u && vt_tiles_per_cu<H>(varlen_tile_lds(Tl, args.tile_cap, H, 2u)) < 4 &&
      vt_tiles_per_cu<H>(varlen_tile_lds(Tl, args.tile_cap, H, 1u)) >= 4)
    args.vhc = 1u;
  size_t lds = vt_pay_off(Tl, args.tile_cap, H, args.vhc == 2u ? 1u : 0u) + 2u * kVTGuard + args.tile_cap;
  if (args.vhc) {  // prebuilt header chunks [Tl][2] x 16 B after the payload run
    lds = (lds + 15u) & ~size_t(15);
    args.hc_off = (uint32_t)lds;
    lds += 32u * Tl;
  }
  // register budget to match the LDS occupancy (vt_waves)
  int w = tuning().varlen_waves;
  if (w < 0) w = vt_waves<H>(lds);
#if RUDP_TOOLS
  if constexpr (!FX)
    if (w == 8) return launch_varlen_tile_w<H, 8, FX>(args, lds, blocks, stream);
#endif
  return w == 6 ? launch_varlen_tile_w<H, 6, FX>(args, lds, blocks, stream)
       : w == 7 ? launch_varlen_tile_w<H, 7, FX>(args, lds, blocks, stream)
                : launch_varlen_tile_w<H, 1, FX>(args, lds, blocks, stream);
}

void varlen_tile_geometry(uint32_t len_hint, uint32_t* T, uint32_t* glog, uint32_t* cap) {
  // About 24 KiB of payload per tile (the fixed-length encode's T = 16 at
  // 1472 B); room for 1.1x the hinted run (varlen_encode_cap_pct) before a
  // tile takes the per-packet path.  Hints above 6 KiB use the per-packet vector kernel (T = 0).
  // 1M x 1472 B with the scan: 0.63 vs 0.77 ms; lengths uniform in
  // [0, 2944]: 0.75 vs 1.04 ms (tools/sweep.py --only varlen_enc).
  const uint32_t h = len_hint;
  *T = 0;
  // Below 16 B the per-packet kernel is as fast (1M one-character datagrams:
  // 0.037 vs 0.038 ms with the scan).
  if (h < 16 || h > 6144) return;
  uint32_t t = 256, lg = 0;
  // Payload bytes per tile at the hint: 24 KiB.  A 32 KiB target above
  // 512-B hints (T = 32 at 1024 B) won while the kernel was VGPR-bound at 5
  // waves (0.47 -> 0.43 ms); with the register budget matched to LDS
  // occupancy, T = 16 (7 tiles per CU) is faster: 1M x 1024 B 0.440 -> 0.407
  // ms (profiles/r01/sweeps/varlen_tile_bytes_r2.json; 32 KiB tiles at
  // 128-512 B measured up to 12% slower, varlen_tile_bytes.json).
  const uint32_t maxT = (uint32_t)tuning().varlen_tile_maxT;
  const uint32_t bytes = tuning().varlen_tile_bytes > 0 ? (uint32_t)tuning().varlen_tile_bytes : 24576u;
  while (t > 4 && (t > maxT || t * h > bytes)) { t >>= 1; ++lg; }
  *T = t;
  *glog = lg;
  *cap = ((t * h * (uint32_t)tuning().varlen_encode_cap_pct / 100u + 256u) + 15u) & ~15u;
  if (*cap < 1024u) *cap = 1024u;
}

int launch_encode_varlen(const VarlenArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  const bool fx = args.frame_off == nullptr;  // a fixed-stride batch (VarlenArgs::stride)
  if (args.tile_T && !args.payload_off && ((reinterpret_cast<uintptr_t>(args.frames) |
                                            reinterpret_cast<uintptr_t>(args.payload)) & 15u) == 0) {
    if (fx) return layout == 7 ? launch_varlen_tile<7, true>(args, stream) : launch_varlen_tile<5, true>(args, stream);
    return layout == 7 ? launch_varlen_tile<7, false>(args, stream) : launch_varlen_tile<5, false>(args, stream);
  }
  if (args.glog != kNoVec && ((reinterpret_cast<uintptr_t>(args.frames) |
                              reinterpret_cast<uintptr_t>(args.payload)) & 15u) == 0) {
    const uint64_t blocks = (args.n + (kBlock >> args.glog) - 1) / (kBlock >> args.glog);
    const void* fn = layout == 7 ? (fx ? reinterpret_cast<const void*>(&encode_varlen_vec_kernel<7, true>)
                                       : reinterpret_cast<const void*>(&encode_varlen_vec_kernel<7, false>))
                                 : (fx ? reinterpret_cast<const void*>(&encode_varlen_vec_kernel<5, true>)
                                       : reinterpret_cast<const void*>(&encode_varlen_vec_kernel<5, false>));
    void* kargs[] = {const_cast<VarlenArgs*>(&args)};
    return (int)hipLaunchKernel(fn, dim3((uint32_t)blocks), dim3(kBlock), kargs, 0, stream);
  }
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  if (layout == 7)
    hipLaunchKernelGGL(encode_varlen_kernel<7>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  else
    hipLaunchKernelGGL(encode_varlen_kernel<5>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

// Every varlen decode form validates the payload's UTF-8 in the same pass when
// args.valid is set (U8): the reference's receive decodes every payload
// (utils/reliableUDP.py:121, get_payload's strict decode at utils/packet.py:73).
template <int H, bool U8, bool FX>
static int launch_decode_varlen_t(const VarlenArgs& args, hipStream_t stream) {
#if RUDP_TOOLS  // byte spans (measured slower; the diagnostics build only)
  if (!FX && args.span_rec) {  // byte spans: the index pass, then one workgroup per span (or per T frames)
    const uint32_t nt = (uint32_t)args.span_count;
    const uint64_t idx_threads = args.n + 2u + nt;
    hipLaunchKernelGGL(decode_span_index_kernel, dim3((uint32_t)((idx_threads + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, stream, args.frame_off, args.n, args.frames_lim, args.span_S, nt,
                       const_cast<SpanRec*>(args.span_rec), const_cast<uint32_t*>(args.span_flag), args.span_epoch);
    const uint32_t T = kBlock >> args.glog;
    const uint64_t frame_blocks = (args.n + T - 1) / T;
    const uint64_t blocks = frame_blocks > nt ? frame_blocks : nt;
    hipLaunchKernelGGL((decode_varlen_span_kernel<H, U8>), dim3((uint32_t)blocks), dim3(kBlock),
                       dsp_lds_bytes(args.tile_cap), stream, args);
    return (int)hipGetLastError();
  }
#endif
  if (args.small_fpt && args.glog != kNoVec && (reinterpret_cast<uintptr_t>(args.frames) & 15u) == 0)
    return launch_decode_small<H, U8, FX>(args, stream);
  if (args.glog != kNoVec && args.tile_cap && (reinterpret_cast<uintptr_t>(args.frames) & 15u) == 0) {
    const uint32_t T = kBlock >> args.glog;
    const size_t lds = dvt_lds_bytes(T, args.tile_cap, args.tile_sums == 2u);
    if (lds <= 65536) {
      const uint64_t blocks = (args.n + T - 1) / T;
      // 76 VGPRs (6 waves per SIMD).  Asking the allocator for 7 or 8 waves
      // spills and was slower at every size (1M x 1479 B 0.265 -> 0.306 ms;
      // profiles/r01/sweeps/varlen_decode_waves.json).
#if RUDP_TOOLS  // chunks read four at a time and two-wave tiles: measured slower
      if constexpr (!FX) {
      if (args.dec_r4) {
        hipLaunchKernelGGL((decode_varlen_tile_kernel<H, U8, kBlock, true>), dim3((uint32_t)blocks), dim3(kBlock),
                           lds, stream, args);
        return (int)hipGetLastError();
      }
      if (args.dec_nt == 128u) {  // two-wave tiles: a tile's LDS waits for the slower of two waves, not four
        const uint64_t b128 = (args.n + (128u >> args.glog) - 1) / (128u >> args.glog);
        hipLaunchKernelGGL((decode_varlen_tile_kernel<H, U8, 128u>), dim3((uint32_t)b128), dim3(128), lds, stream,
                           args);
        return (int)hipGetLastError();
      }
      }
#endif
      // 2-16 lanes a frame with the UTF-8 check: sums and check in one pass
      // (profiles/r06/sweeps/varlen_utf8_fused_ab.json)
      if (U8 && args.glog >= 1u && args.glog <= 4u && args.tile_sums != 2u)
        hipLaunchKernelGGL((decode_varlen_tile_kernel<H, U8, kBlock, false, FX, true>), dim3((uint32_t)blocks),
                           dim3(kBlock), lds, stream, args);
      else
        hipLaunchKernelGGL((decode_varlen_tile_kernel<H, U8, kBlock, false, FX>), dim3((uint32_t)blocks),
                           dim3(kBlock), lds, stream, args);
      return (int)hipGetLastError();
    }
  }
  if (args.glog != kNoVec && (reinterpret_cast<uintptr_t>(args.frames) & 15u) == 0) {
    const uint64_t blocks = (args.n + (kBlock >> args.glog) - 1) / (kBlock >> args.glog);
    hipLaunchKernelGGL((decode_varlen_vec_kernel<H, U8, FX>), dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
    return (int)hipGetLastError();
  }
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  hipLaunchKernelGGL((decode_varlen_kernel<H, U8>), dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

#if RUDP_TOOLS
bool decode_span_fits(uint64_t cap) { return cap < 65536u && dsp_lds_bytes((uint32_t)cap) <= 65536u; }
#endif

int launch_decode_varlen(const VarlenArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  if (args.frame_off == nullptr) {  // a fixed-stride batch (VarlenArgs::stride)
    if (args.valid)
      return layout == 7 ? launch_decode_varlen_t<7, true, true>(args, stream)
                         : launch_decode_varlen_t<5, true, true>(args, stream);
    return layout == 7 ? launch_decode_varlen_t<7, false, true>(args, stream)
                       : launch_decode_varlen_t<5, false, true>(args, stream);
  }
  if (args.valid)
    return layout == 7 ? launch_decode_varlen_t<7, true, false>(args, stream)
                       : launch_decode_varlen_t<5, true, false>(args, stream);
  return layout == 7 ? launch_decode_varlen_t<7, false, false>(args, stream)
                     : launch_decode_varlen_t<5, false, false>(args, stream);
}

int launch_validate_utf8(const Utf8Args& args, hipStream_t stream) {
  if (args.n == 0) return 0;
  const bool aligned = (reinterpret_cast<uintptr_t>(args.frames) & 15u) == 0;
  if (aligned && !args.frame_off && args.F > args.H && tuning().utf8_tile) {
    Utf8Args a = args;
    a.glog = decode_group_log2(args.F - args.H);  // T = 256 / G frames, a multiple of 16
    const uint32_t T = kBlock >> a.glog;
    const size_t lds = (((size_t)T * args.F + 15u) & ~size_t(15)) + 32u;
    if (lds <= 65536) {
      const uint64_t blocks = (args.n + T - 1) / T;
      hipLaunchKernelGGL(validate_utf8_tile_kernel, dim3((uint32_t)blocks), dim3(kBlock), lds, stream, a);
      return (int)hipGetLastError();
    }
  }
  // Hints of 128 B and up (1M x 263 B 0.102 -> 0.079 ms with the byte-sized
  // tiles; profiles/r01/sweeps/varlen_decode_small.json).
  if (aligned && args.frame_off && tuning().utf8_vtile && (args.F >= 128u || tuning().utf8_vtile == 2)) {
    // packed frames through LDS tiles of T = 256 / G frames, 1.1x the hinted run
    Utf8Args a = args;
    const uint32_t chunks = args.F / 16u + 1u;
    uint32_t lg = 1;
    const uint32_t run = (uint32_t)tuning().utf8_vtile_bytes;
    if (run) {  // the most frames (G >= 2) whose LDS budget stays within `run` bytes
      while (lg < 4 && (uint64_t)(256u >> lg) * args.F * (uint64_t)tuning().utf8_vtile_cap_pct / 100u > run) ++lg;
    } else {    // two+ 16-byte chunks per lane
      while (lg < 4 && (4u << lg) <= chunks) ++lg;
    }
    a.glog = lg;
    const uint32_t T = kBlock >> lg;
    const uint64_t cap = (((uint64_t)T * args.F * (uint64_t)tuning().utf8_vtile_cap_pct / 100u + 256u) + 15u) & ~15ull;
    if (cap <= 49152u) {
      a.tile_cap = (uint32_t)cap;
      const size_t lds = ((((T + 1u) * 4u) + 15u) & ~15u) + 16u + cap + 32u;
      const uint64_t blocks = (args.n + T - 1) / T;
      hipLaunchKernelGGL(validate_utf8_vtile_kernel, dim3((uint32_t)blocks), dim3(kBlock), lds, stream, a);
      return (int)hipGetLastError();
    }
  }
  if (aligned) {
    // lanes per frame from the (typical) frame length: two+ 16-byte chunks per lane
    Utf8Args a = args;
    const uint32_t chunks = args.F / 16u + 1u;
    uint32_t lg = 0;
    while (lg < 4 && (4u << lg) <= chunks) ++lg;
    a.glog = lg;
    const uint64_t blocks = ((args.n << lg) + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(validate_utf8_vec_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, a);
    return (int)hipGetLastError();
  }
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(validate_utf8_par_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

#if RUDP_TOOLS
// The round-1 scan by hipcub (tools build, sweeps only): no device-side checks, no span starts.
static int scan_frame_offsets_hipcub(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                                     hipStream_t stream) {
  hipcub::CountingInputIterator<uint64_t> idx(0);
  hipcub::TransformInputIterator<uint64_t, FrameLen, hipcub::CountingInputIterator<uint64_t>> it(
      idx, FrameLen{d_len, H});
  size_t temp = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, temp, it, d_frame_off + 1, (int)n, stream);
  if (e != hipSuccess) return (int)e;
  void* d_temp = nullptr;
  if ((e = stream_alloc(&d_temp, temp ? temp : 1, stream)) != hipSuccess) return (int)e;
  e = hipcub::DeviceScan::InclusiveSum(d_temp, temp, it, d_frame_off + 1, (int)n, stream);
  hipError_t e2 = hipMemsetAsync(d_frame_off, 0, sizeof(uint64_t), stream);
  hipError_t e3 = stream_free(d_temp, stream);
  if (e != hipSuccess) return (int)e;
  if (e2 != hipSuccess) return (int)e2;
  return (int)e3;
}
#endif

// frame_off[0..n] = exclusive scan of len[i] + H, frame_off[n] = total bytes.
int scan_frame_offsets(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                       const ScanCheck& chk, hipStream_t stream, const SpanStarts& spans) {
#if RUDP_TOOLS
  // the device-side checks and the span starts live in the three-pass scan only
  if (tuning().varlen_scan != 1 && !chk.status && !spans.rec)
    return scan_frame_offsets_hipcub(d_len, n, H, d_frame_off, stream);
#endif
  return scan_frame_offsets_3pass(d_len, n, H, d_frame_off, chk, stream, spans);
}

}  // namespace rudp
