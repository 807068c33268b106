// Batched frame + checksum (encode) kernels for gfx950.
//
// Replaces the per-packet encode of the reference, utils/reliableUDP.py:53-61:
//   Packet() (utils/packet.py:13-16) -> set_header_field seq/ack/syn/fin
//   (:43-57) -> set_payload (:60-65) -> to_byte (:76-81)
// plus the build-defined RFC 1071 checksum.
//
// Payloads that are a multiple of 16 B (and 16-B aligned buffers): one workgroup per TILE of T packets
// (a power of two, 4..256; 16 at L >= 512).  The frame stride L+H is odd, so
// for T < 16 a tile's output range starts and ends mid-chunk; the two shared
// chunks are written bytewise by their owners.
//   phase 1  the tile's payload is one contiguous run: it streams into an
//            LDS tile by LDS-DMA (global_load_lds_dwordx4 nt, 1 KiB per
//            wave-instruction; register staging in the tools build's sweeps).  For
//            tiles up to 16 KiB the leaders' header-table loads go out first.
//   sums     G = 256/T lanes per packet sum its LE u16 halves out of LDS; a
//            shfl_xor butterfly combines them; the leader writes the 5/7-byte
//            header word (with checksum) and, for T % 16 == 0, prebuilds the
//            packet's 1-2 header chunks in LDS.
//   phase 2  output-stationary: each lane owns aligned 16 B output chunks
//            (dealt from the tile's first 64-B boundary): a pure-payload chunk
//            is one byte-shifted LDS window, a header chunk one aligned LDS
//            read of the prebuilt chunk (the general form assembles any chunk
//            from two windows and the header words); one dwordx4 nt store.
// HBM traffic = read L + 5 (payload + header table) and write L + H per
// packet, each byte exactly once (PMC: 1.011x at L = 1472).
#include "codec_device.hpp"
#include "internal.hpp"

namespace RUDP_NS {

constexpr int kLdsGuard = 16;  // bytes before the payload tile (negative offsets)

template <bool NT>
__device__ __forceinline__ u32x4 load16(const u32x4* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

template <bool NT>
__device__ __forceinline__ void store16(u32x4 v, u32x4* p) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Writes the one or two header chunks of the packet whose payload starts at
// output offset P.
template <int H>
__device__ __forceinline__ void store_header_chunks(unsigned char* out, uint64_t P, uint64_t h,
                                                    u32x4 tail, u32x4 head) {
  const uint64_t X0 = (P - H) & ~15ull, X1 = (P + 15u) & ~15ull;
  for (uint64_t X = X0; X < X1; X += 16)
    __builtin_nontemporal_store(header_chunk<H>(X, P, h, tail, head), reinterpret_cast<u32x4*>(out + X));
}

// Phase 2 of the encode tile:
// output-stationary aligned 16 B chunks assembled from the LDS payload tile
// and header words.
template <int H, bool NTS, int BLOCK>
__device__ __forceinline__ void encode_phase2(const EncodeTileArgs& a, const unsigned char* lds_pay,
                                              const uint64_t* lds_hdr, uint64_t p0, uint32_t Tv,
                                              uint32_t tid) {
  const uint32_t L = a.L;
  // The tile owns output bytes [p0*F, (p0+Tv)*F).  Chunks are aligned to the
  // global address; when T*F is not a multiple of 16 (T < 16) the tile's first
  // and last chunk are shared with its neighbours and only the owned bytes
  // are written (bytewise, two partial chunks per tile).
  const uint32_t F = L + H;
  const uint32_t nbytes = Tv * F;
  unsigned char* out = a.frames + p0 * (uint64_t)F;
  const uint32_t lead = (uint32_t)(-(uintptr_t)out) & 15u;  // bytes before the first aligned chunk
  const uint32_t nfull = nbytes > lead ? (nbytes - lead) >> 4 : 0u;
  // Full chunks are dealt from the first 64-B boundary on (the 0-3 chunks
  // before it go last), so each wave's 1 KiB store covers whole 64-B sectors
  // instead of splitting one at each end with the next wave.
  uint32_t npre = a.out_align64 ? ((uint32_t)(-(uintptr_t)out) & 63u) >> 4 : 0u;
  if (npre > nfull) npre = nfull;
  const uint32_t* pay_dw = reinterpret_cast<const uint32_t*>(lds_pay);
  // unit k < nfull: full chunk i = (k + npre) mod nfull at tile offset
  // lead + 16i; the two units after that are the partial head [0, lead) and
  // tail [lead + 16*nfull, nbytes).
  for (uint32_t k = tid; k < nfull + 2u; k += BLOCK) {
    uint32_t x, lo_b, hi_b;  // tile offset of chunk byte 0; owned byte range [lo_b, hi_b)
    if (k < nfull) {
      const uint32_t i = k + npre < nfull ? k + npre : k + npre - nfull;
      x = lead + 16u * i; lo_b = 0; hi_b = 16;
    } else if (k == nfull) {
      x = 0; lo_b = 0; hi_b = lead < nbytes ? lead : nbytes;
    } else {
      x = lead + 16u * nfull; lo_b = 0; hi_b = nbytes > x ? nbytes - x : 0u;
    }
    if (hi_b <= lo_b) continue;
    const uint32_t qq = (uint32_t)(((uint64_t)x * a.invF) >> 32);  // x / F
    const uint32_t r = x - qq * F;           // frame position of chunk byte 0
    const int kA0 = r < (uint32_t)H ? H - (int)r : 0;  // first payload byte of qq
    const int kend = (int)(F - r);           // first byte of packet qq+1
    // LDS offset (from lds_pay) of byte 0 if it were payload of qq.
    const uint32_t sA = kLdsGuard + qq * L + r - H;
    const u32x4 A = window16_dw(pay_dw, sA);
    uint64_t lo = lo64(A) & byte_mask(kA0, kend);
    uint64_t hi = hi64(A) & byte_mask(kA0 - 8, kend - 8);
    if (kA0 > 0) lo |= lds_hdr[qq] >> (8 * r);
    if (kend < 16) {
      const u32x4 B = window16_dw(pay_dw, sA - H);
      lo |= lo64(B) & byte_mask(kend + H, 16);
      hi |= hi64(B) & byte_mask(kend + H - 8, 8);
      const uint64_t h1 = lds_hdr[qq + 1];
      if (kend < 8) {
        lo |= h1 << (8 * kend);
        if (kend > 0) hi |= h1 >> (64 - 8 * kend);
      } else {
        hi |= h1 << (8 * (kend - 8));
      }
    }
    const u32x4 v = make_u32x4(lo, hi);
    if (hi_b == 16u) {
      store16<NTS>(v, reinterpret_cast<u32x4*>(out + x));
    } else {
      uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b)
        if (b < hi_b) out[x + b] = (unsigned char)(d[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// Phase 2 with prebuilt header chunks (T % 16 == 0, so the tile starts on a
// 16-B boundary).  A chunk is either pure payload of one packet (frame
// positions [r, r + 16) inside [H, F)) — one byte-shifted LDS window — or one
// of the 1-2 chunks over a header, which the packet's leader built in the sum
// pass (lds_hc[2q + slot]).  Stores stay one 1 KiB run per wave-instruction.
template <int H, bool NTS, int BLOCK>
__device__ __forceinline__ void encode_phase2_hc(const EncodeTileArgs& a, const unsigned char* lds_pay,
                                                 const u32x4* lds_hc, uint64_t p0, uint32_t Tv,
                                                 uint32_t tid) {
  const uint32_t L = a.L, F = L + H;
  const uint32_t nbytes = Tv * F;
  unsigned char* out = a.frames + p0 * (uint64_t)F;
  const uint32_t nfull = nbytes >> 4;
  const uint32_t nall = (nbytes + 15u) >> 4;
  uint32_t npre = a.out_align64 ? ((uint32_t)(-(uintptr_t)out) & 63u) >> 4 : 0u;
  if (npre > nfull) npre = nfull;
  const uint32_t* pay_dw = reinterpret_cast<const uint32_t*>(lds_pay);
  for (uint32_t k = tid; k < nall; k += BLOCK) {
    const uint32_t i = k < nfull ? (k + npre < nfull ? k + npre : k + npre - nfull) : k;
    const uint32_t x = 16u * i;
    const uint32_t qq = (uint32_t)(((uint64_t)x * a.invF) >> 32);  // x / F
    const uint32_t r = x - qq * F;
    const uint32_t ph = r < (uint32_t)H ? qq : qq + 1u;  // packet whose header the chunk holds
    u32x4 v;
    if ((r >= (uint32_t)H && r + 16u <= F) || ph >= Tv) {
      v = window16_dw(pay_dw, kLdsGuard + qq * L + r - H);
    } else {
      v = lds_hc[2u * ph + ((x - ((ph * F) & ~15u)) >> 4)];
    }
    if (i < nfull) {
      store16<NTS>(v, reinterpret_cast<u32x4*>(out + x));
    } else {  // the batch's last bytes
      const uint32_t d[4] = {v.x, v.y, v.z, v.w};
      for (uint32_t b = 0; b < nbytes - x; ++b) out[x + b] = (unsigned char)(d[b >> 2] >> (8 * (b & 3)));
    }
  }
}

template <int H, bool NTL, bool NTS, int P1, int BLOCK = kBlock, bool DMA = false>
__global__ void __launch_bounds__(BLOCK) encode_tile_kernel(EncodeTileArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  uint32_t tile = blockIdx.x;
  if (a.xcd_swizzle) tile = xcd_tile(tile, a.num_tiles);  // each XCD streams its own slice
  uint64_t* lds_hdr = reinterpret_cast<uint64_t*>(lds);  // [T + 1]
  unsigned char* lds_pay = lds + a.hdr_bytes;            // guard + T*L + tail guard

  const uint32_t tid = threadIdx.x;
  const uint32_t L = a.L;
  const uint32_t T = a.T;
  const uint64_t p0 = (uint64_t)tile * T;
  // a.glog is lanes-per-packet for 256-thread groups; wider (narrower) groups
  // give each packet more (fewer) lanes.  The launcher keeps T <= BLOCK.
  constexpr int kLogBlock = BLOCK == 64 ? 6 : BLOCK == 128 ? 7 : BLOCK == 512 ? 9 : BLOCK == 1024 ? 10 : 8;
  const uint32_t glog = (uint32_t)((int)a.glog + kLogBlock - 8);
  const uint32_t G = 1u << glog;
  const uint64_t left = a.n - p0;
  const uint32_t Tv = left < T ? (uint32_t)left : T;
#if RUDP_TOOLS
  const uint64_t t_start = a.trace ? (uint64_t)wall_clock64() : 0ull;
  uint64_t t_loaded = 0, t_summed = 0;
#endif

  // ---- phase 1: payload -> LDS, per-packet LE16 sums --------------------
  const uint32_t q = tid >> glog;
  const uint32_t g = tid & (G - 1u);
  const uint32_t V = L >> 4;  // 16 B vectors per packet
  // Header-table loads can go out before the payload stream, so their latency
  // overlaps phase 1 instead of adding a round trip after the barrier.
  uint32_t t_seq = 1u, t_ack = 2u, t_flags = 3u;
  const bool dma_tab = DMA && a.early_table == 2u && Tv == T;  // uniform
  if (a.early_table == 1u && g == 0 && q < Tv) {
    t_seq = a.seq[p0 + q];
    t_ack = a.ack[p0 + q];
    t_flags = a.flags[p0 + q];
  }
  uint32_t sum = 0;
  {
    // The tile's payload is one contiguous run: stream it like a copy (lane t
    // takes vectors t, t+256, ...: every wave-instruction reads 1 KiB
    // contiguous), then sum each packet back out of LDS.
    const u32x4* src = reinterpret_cast<const u32x4*>(a.payload + p0 * (uint64_t)L);
    u32x4* dst = reinterpret_cast<u32x4*>(lds_pay + kLdsGuard);
    const uint32_t nvec = Tv * V;
    if (DMA) {
      // LDS-DMA (global_load_lds_dwordx4): each wave-instruction moves 1 KiB
      // from HBM straight into the tile, lane-linear, no VGPR round trip.
      if (dma_tab && tid < 5u) {  // the tile's table: seq 2 x 16 B, ack 2 x 16 B, flags 16 B
        const unsigned char* g_src = tid < 2u ? reinterpret_cast<const unsigned char*>(a.seq + p0) + 16u * tid
                                   : tid < 4u ? reinterpret_cast<const unsigned char*>(a.ack + p0) + 16u * (tid - 2u)
                                              : reinterpret_cast<const unsigned char*>(a.flags + p0);
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g_src,
                                         (void __attribute__((address_space(3)))*)(lds + a.tab_off), 16, 0,
                                         NTL ? 2 : 0);
      }
      const uint32_t wbase = tid & ~63u;
      for (uint32_t v0 = wbase; v0 < nvec; v0 += BLOCK) {
        if (v0 + (tid & 63u) < nvec)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1)))*)(src + v0 + (tid & 63u)),
              (void __attribute__((address_space(3)))*)(dst + v0), 16, 0, NTL ? 2 : 0);
      }
    }
    for (uint32_t v0 = tid; !DMA && v0 < nvec; v0 += (uint32_t)P1 * BLOCK) {
      u32x4 r[P1];
#pragma unroll
      for (int u = 0; u < P1; ++u) {
        const uint32_t v = v0 + (uint32_t)u * BLOCK;
        if (v < nvec) r[u] = load16<NTL>(src + v);
      }
#pragma unroll
      for (int u = 0; u < P1; ++u) {
        const uint32_t v = v0 + (uint32_t)u * BLOCK;
        if (v < nvec) dst[v] = r[u];
      }
    }
    __syncthreads();
#if RUDP_TOOLS
    if (a.trace && tid == 0) t_loaded = (uint64_t)wall_clock64();
#endif
    if (q < Tv) {
      const u32x4* mine = dst + q * V;
      for (uint32_t v = g; v < V; v += G) sum += le16_sum(mine[v]);
    }
  }
  sum = group_sum(sum, G);
  if (g == 0 && q < Tv) {
    const uint64_t p = p0 + q;
    const bool late = a.early_table != 1u && !dma_tab;
    uint32_t s = late ? a.seq[p] : t_seq, k = late ? a.ack[p] : t_ack, f = late ? a.flags[p] : t_flags;
    if (dma_tab) {
      const unsigned char* tb = lds + a.tab_off;
      s = reinterpret_cast<const uint16_t*>(tb)[q];
      k = reinterpret_cast<const uint16_t*>(tb + 32)[q];
      f = tb[64 + q];
    }
    const uint32_t c = packet_csum(sum, s, k, f);
    const uint64_t h = pack_header<H>(s, k, f, c);
    lds_hdr[q] = h;
    if (a.csum) a.csum[p] = (uint16_t)c;
    if (a.hchunk) {  // this packet's 1-2 header chunks, for encode_phase2_hc
      const u32x4* img = reinterpret_cast<const u32x4*>(lds_pay + kLdsGuard);
      const uint32_t P = q * (L + H) + H;
      u32x4* hc = reinterpret_cast<u32x4*>(lds + a.hc_off) + 2u * q;
      const uint32_t X0 = (P - H) & ~15u, X1 = (P + 15u) & ~15u;
      const u32x4 tail = img[q * V - 1u], head = img[q * V];
      if (a.hc_scratch) {
        // [previous payload's last 16 | header | first 16 payload bytes] laid
        // out in 48 B of LDS with compile-time shifts; each chunk is then one
        // byte-shifted window (no variable-shift funnels).
        constexpr uint32_t b = (uint32_t)H & 3u, sl = 8u * b, sr = 32u - 8u * b;
        uint32_t* scr = reinterpret_cast<uint32_t*>(lds + a.scr_off) + 12u * q;
        reinterpret_cast<u32x4*>(scr)[0] = tail;
        u32x4 w1, w2;
        w1.x = (uint32_t)h;
        w1.y = ((uint32_t)(h >> 32) & ((1u << sl) - 1u)) | (head.x << sl);
        w1.z = (head.x >> sr) | (head.y << sl);
        w1.w = (head.y >> sr) | (head.z << sl);
        w2.x = (head.z >> sr) | (head.w << sl);
        w2.y = head.w >> sr;
        w2.z = 0u;
        w2.w = 0u;
        reinterpret_cast<u32x4*>(scr)[1] = w1;
        reinterpret_cast<u32x4*>(scr)[2] = w2;
        for (uint32_t X = X0; X < X1; X += 16)
          hc[(X - X0) >> 4] = window16_dw(scr, 16u + X - (P - H));
      } else {
        for (uint32_t X = X0; X < X1; X += 16)
          hc[(X - X0) >> 4] = header_chunk<H>(X, P, h, tail, head);
      }
    }
  }
  __syncthreads();
#if RUDP_TOOLS
  if (a.trace && tid == 0) t_summed = (uint64_t)wall_clock64();
#endif

  if (a.hchunk)
    encode_phase2_hc<H, NTS, BLOCK>(a, lds_pay, reinterpret_cast<const u32x4*>(lds + a.hc_off), p0, Tv, tid);
  else
    encode_phase2<H, NTS, BLOCK>(a, lds_pay, lds_hdr, p0, Tv, tid);
#if RUDP_TOOLS
  if (a.trace) {  // diagnostics: the tile's timeline (100 MHz wall clock), XCD and CU
    __syncthreads();
    if (tid == 0) {
      const uint64_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID[3:0]
      u32x4* rec = reinterpret_cast<u32x4*>(a.trace + 6ull * tile);
      const uint64_t t_end = (uint64_t)wall_clock64();
      rec[0] = make_u32x4(t_start, t_end);
      rec[1] = make_u32x4(xcc, (uint64_t)__smid());
      rec[2] = make_u32x4(t_loaded, t_summed);  // phase-1 loads landed, sums + headers done
    }
  }
#endif
}

template <int H, bool NTL, bool NTS, int P1, int BLOCK = kBlock, bool DMA = false>
int launch_tile(const EncodeTileArgs& args, hipStream_t stream) {
  const uint64_t blocks = args.num_tiles;
  size_t lds = args.hdr_bytes + kLdsGuard + (size_t)args.T * args.L + 32;
  int per_cu = tuning().encode_blocks_per_cu;
  // Auto: cap resident tiles per CU by tile payload, so the concurrent HBM
  // footprint stays near 70-120 KiB per CU: 5 above 14 KiB (1M x 1472 B
  // 0.504 vs 0.516 ms at 6; x 1024 B 0.357 vs 0.370 ms natural), 6 above
  // 10 KiB (x 768 B 0.259 vs 0.270 ms natural), natural below (x 512 B
  // 0.176 vs 0.181 at 7).  (profiles/r01/sweeps/encode_percu_lds_dma.json;
  // before LDS-DMA phase 1 and early table loads, 16 KiB tiles preferred
  // natural occupancy.)
  if (per_cu < 0) {
    const size_t bytes = (size_t)args.T * args.L;
    per_cu = bytes > 14336 ? 5 : bytes > 10240 ? 6 : 0;
  }
  if (per_cu > 0) {  // reserve LDS to cap resident workgroups per CU
    const size_t want = ((size_t)(160 * 1024) / (size_t)per_cu) & ~size_t(15);
    if (want > lds) lds = want;
  }
  const void* fn = reinterpret_cast<const void*>(&encode_tile_kernel<H, NTL, NTS, P1, BLOCK, DMA>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((encode_tile_kernel<H, NTL, NTS, P1, BLOCK, DMA>), dim3((uint32_t)blocks), dim3(BLOCK), lds,
                     stream, args);
  return (int)hipGetLastError();
}

#if RUDP_TOOLS
template <int H, int P1>
int launch_tile_nt(const EncodeTileArgs& args, hipStream_t stream) {
  const Tuning& t = tuning();
  if (t.encode_nt_load && t.encode_nt_store) return launch_tile<H, true, true, P1>(args, stream);
  if (t.encode_nt_load) return launch_tile<H, true, false, P1>(args, stream);
  if (t.encode_nt_store) return launch_tile<H, false, true, P1>(args, stream);
  return launch_tile<H, false, false, P1>(args, stream);
}

// The tools build's sweep forms: register-staged phase 1 (P1 loads in flight
// per lane), temporal loads or stores, 64- to 1024-thread workgroups.
template <int H>
int launch_tile_policy(const EncodeTileArgs& args, hipStream_t stream) {
  const int p1 = tuning().encode_p1;
  int block = tuning().encode_block;
  // A packet's lanes must sit in one wave (the shfl_xor reduction): wider
  // blocks give each packet (256/T)*(block/256) lanes, so keep that <= 64.
  if (block > 256 && (uint64_t)(256u / args.T) * (uint32_t)(block / 256) > 64u) block = 256;
  const Tuning& t = tuning();
  if (t.encode_dma && block == 512) return launch_tile<H, true, true, 8, 512, true>(args, stream);
  if (t.encode_dma && block == 128 && args.T <= 128) return launch_tile<H, true, true, 8, 128, true>(args, stream);
  if (t.encode_dma && block == 256) {
    if (t.encode_nt_load && t.encode_nt_store) return launch_tile<H, true, true, 8, kBlock, true>(args, stream);
    if (t.encode_nt_load) return launch_tile<H, true, false, 8, kBlock, true>(args, stream);
    if (t.encode_nt_store) return launch_tile<H, false, true, 8, kBlock, true>(args, stream);
    return launch_tile<H, false, false, 8, kBlock, true>(args, stream);
  }
  if (block == 64 && args.T <= 64) return launch_tile<H, true, true, 8, 64>(args, stream);
  if (block == 128 && args.T <= 128) return launch_tile<H, true, true, 8, 128>(args, stream);
  if (block == 512) return launch_tile<H, true, true, 8, 512>(args, stream);
  if (block == 1024) return launch_tile<H, true, true, 8, 1024>(args, stream);
  if (p1 == 2) return launch_tile_nt<H, 2>(args, stream);
  if (p1 == 4) return launch_tile_nt<H, 4>(args, stream);
  return launch_tile_nt<H, 8>(args, stream);
}
#else
// The measured form: LDS-DMA phase 1, non-temporal loads and stores,
// 256-thread workgroups (profiles/r01/sweeps/encode_dma*.json, encode_block_sizes.json).
template <int H>
int launch_tile_policy(const EncodeTileArgs& args, hipStream_t stream) {
  return launch_tile<H, true, true, 8, kBlock, true>(args, stream);
}
#endif


int launch_encode(const EncodeTileArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  return layout == 7 ? launch_tile_policy<7>(args, stream) : launch_tile_policy<5>(args, stream);
}

}  // namespace rudp
