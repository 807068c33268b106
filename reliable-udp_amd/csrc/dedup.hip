// Batched retransmission detection.
//
// The reference proxy keeps its last Proxy.MAX_MEMORY = 500 packets in a list
// (proxy.py:17, :92-94) and counts a datagram as retransmitted when
// `packet in self.packets` (proxy.py:90): up to 500 Packet.__eq__ calls, each
// comparing two get_hex() strings (utils/packet.py:83-86), ~54 us apiece at
// 1472 B.  Over a batch in arrival order this is
//     dup[i] = 1  iff  frame i == some frame j, max(0, i - window) <= j < i
// with == meaning equal get_hex(): equal bytes, except that an empty datagram
// parses as the 40-bit zero header (utils/packet.py:16), i.e. equals 00 00 00 00 00.
//
//   pass 1  hash: G lanes per frame (1 for the reference's 6-9 B datagrams,
//           up to 8 from 256-B frames), h = sum over bytes of
//           mix64(position << 8 | byte) (order-sensitive, associative, so the
//           lanes can split the frame), plus the length.
//   pass 2  window: each workgroup stages the hashes of its 256 frames and the
//           `window` frames before them in LDS and chains them into an LDS
//           hash table (bucket heads by atomic exchange); each frame walks its
//           bucket's chain for an entry inside its window with an equal hash
//           and confirms the hit byte by byte (exact, never a probabilistic
//           answer).  Expected O(1) per frame instead of `window` compares.
//           The scan form (every frame compares its whole window) stays
//           behind rudpx_tune key 32 = 0.
//
// Small frames (the reference's 6-9 B datagrams; mean length up to
// kDedupSmallLen, window up to kDedupSmallWin) take one launch instead:
// dedup_small_kernel.  A workgroup owns T = 256 * FPT consecutive frames and
// stages their offsets and bytes, and those of the `window` frames before
// them, in LDS (one contiguous run, coalesced; the halo is its neighbour
// workgroup's run, an L2 hit under the XCD-contiguous tile order), hashes all
// of them from LDS (32-bit, an invalid frame hashes to 0), chains them into
// an LDS table and confirms every hit from LDS.  No hash scratch in HBM and
// each offset read once: the round-3 two-pass chain moved 3.8x the algorithmic
// bytes (8-B hashes written, then re-read per workgroup with their halo).
#include <type_traits>

#include "codec_device.hpp"

#include "internal.hpp"

namespace RUDP_NS {

constexpr uint32_t kDedupLanes = 8;
constexpr uint32_t kMaxWindow = 4096;

__device__ __forceinline__ uint64_t dmix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// The bytes Packet(frame).get_hex() spells: the frame, or 5 zero bytes when it
// is empty.  False (and an empty span) for a checked call's frame whose offsets
// are decreasing or past the buffer: none of its bytes is read.
__device__ __forceinline__ bool frame_span(const DedupArgs& a, uint64_t i, uint64_t* off, uint32_t* len) {
  if (a.frame_off) {
    const uint64_t fo = a.frame_off[i], fe = a.frame_off[i + 1];
    if (a.lim_checked && (fo > fe || fe > a.frames_lim)) {
      *off = 0;
      *len = 0;
      return false;
    }
    *off = fo;
    *len = (uint32_t)(fe - fo);
  } else {
    *off = i * (uint64_t)a.F;
    *len = a.F;
  }
  return true;
}

__device__ __forceinline__ uint32_t canon_byte(const DedupArgs& a, uint64_t off, uint32_t len, uint32_t k) {
  return len ? a.frames[off + k] : 0u;
}

__global__ void __launch_bounds__(kBlock) dedup_hash_kernel(DedupArgs a) {
  const uint32_t G = 1u << a.glog;
  const uint32_t g = threadIdx.x & (G - 1u);
  const uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> a.glog;
  const bool valid = i < a.n;
  uint64_t h = 0;
  uint32_t len = 0;
  if (valid) {
    uint64_t off;
    const bool ok = frame_span(a, i, &off, &len);
    const uint32_t clen = len ? len : 5u;
    for (uint32_t k = g; ok && k < clen; k += G)
      h += dmix(((uint64_t)k << 8) | canon_byte(a, off, len, k));
    if (g == 0) h += dmix(0xFFFFFFFF00000000ull | clen);
  }
  for (uint32_t m = G >> 1; m > 0; m >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)h, (int)m, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(h >> 32), (int)m, 64);
    h += ((uint64_t)hi << 32) | lo;
  }
  if (valid && g == 0) a.hash[i] = h;
}

__device__ bool frames_equal(const DedupArgs& a, uint64_t i, uint64_t j) {
  uint64_t oi, oj;
  uint32_t li, lj;
  if (!frame_span(a, i, &oi, &li) || !frame_span(a, j, &oj, &lj)) return false;
  const uint32_t ci = li ? li : 5u, cj = lj ? lj : 5u;
  if (ci != cj) return false;
  // 16 bytes of each frame per step, all loads issued before the compares
  for (uint32_t k0 = 0; k0 < ci; k0 += 16) {
    uint32_t diff = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
      if (k0 + k < ci) diff |= canon_byte(a, oi, li, k0 + k) ^ canon_byte(a, oj, lj, k0 + k);
    if (diff) return false;
  }
  return true;
}

__global__ void __launch_bounds__(kBlock) dedup_window_kernel(DedupArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint64_t* lh = reinterpret_cast<uint64_t*>(lds_raw);  // [window + kBlock]
  const uint64_t first = (uint64_t)blockIdx.x * kBlock;
  const uint64_t lo = first > a.window ? first - a.window : 0;
  const uint64_t hi = first + kBlock < a.n ? first + kBlock : a.n;
  for (uint64_t j = lo + threadIdx.x; j < hi; j += kBlock) lh[j - lo] = a.hash[j];
  __syncthreads();
  const uint64_t i = first + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t h = lh[i - lo];
  const uint64_t j0 = i > a.window ? i - a.window : 0;
  uint8_t dup = 0;
  for (uint64_t j = j0; j < i; ++j) {
    if (lh[j - lo] == h && frames_equal(a, i, j)) {
      dup = 1;
      break;
    }
  }
  uint64_t o;
  uint32_t l;
  a.dup[i] = frame_span(a, i, &o, &l) ? dup : (uint8_t)RUDP_DUP_BAD_OFFSETS;
}

// Table form of pass 2: LDS = hashes [cnt] u64, chain links [cnt] i32, bucket
// heads [nb] i32 (nb a power of two, about 2x cnt).
__global__ void __launch_bounds__(kBlock) dedup_table_kernel(DedupArgs a, uint32_t nb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const uint64_t first = (uint64_t)blockIdx.x * kBlock;
  const uint64_t lo = first > a.window ? first - a.window : 0;
  const uint64_t hi = first + kBlock < a.n ? first + kBlock : a.n;
  const uint32_t cnt = (uint32_t)(hi - lo);
  const uint32_t cap = a.window + kBlock;
  uint64_t* lh = reinterpret_cast<uint64_t*>(lds_raw);  // [cap]
  int* nxt = reinterpret_cast<int*>(lh + cap);          // [cap]
  int* head = nxt + cap;                                 // [nb]
  for (uint32_t b = threadIdx.x; b < nb; b += kBlock) head[b] = -1;
  for (uint32_t e = threadIdx.x; e < cnt; e += kBlock) lh[e] = a.hash[lo + e];
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < cnt; e += kBlock) {
    const uint64_t h = lh[e];
    nxt[e] = atomicExch(&head[(uint32_t)(h ^ (h >> 32)) & (nb - 1u)], (int)e);
  }
  __syncthreads();
  const uint64_t i = first + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t ei = (uint32_t)(i - lo);
  const uint32_t emin = (uint32_t)((i > a.window ? i - a.window : 0) - lo);
  const uint64_t h = lh[ei];
  uint8_t dup = 0;
  for (int e = head[(uint32_t)(h ^ (h >> 32)) & (nb - 1u)]; e >= 0; e = nxt[e]) {
    const uint32_t u = (uint32_t)e;
    if (u >= emin && u < ei && lh[u] == h && frames_equal(a, i, lo + u)) {
      dup = 1;
      break;
    }
  }
  uint64_t o;
  uint32_t l;
  a.dup[i] = frame_span(a, i, &o, &l) ? dup : (uint8_t)RUDP_DUP_BAD_OFFSETS;
}

// ---- small frames: one launch -------------------------------------------------
constexpr uint32_t kDedupSmallWin = 1024;  // most window the one-launch form stages
constexpr uint32_t kDedupSmallLen = 16;    // mean frame length (bytes) it is used up to

// 32-bit hash of a frame's canonical bytes (FNV-1a, then the murmur3 finalizer
// with the length): equal frames hash equal; 0 is kept for invalid frames.
template <class ByteF>
__device__ __forceinline__ uint32_t small_hash(uint32_t len, ByteF byte) {
  const uint32_t cl = len ? len : 5u;
  uint32_t h = 0x811C9DC5u;
  for (uint32_t k = 0; k < cl; ++k) h = (h ^ (len ? byte(k) : 0u)) * 0x01000193u;
  h ^= cl * 0x9E3779B1u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h ? h : 1u;
}

// The tile's work once its entries' spans are known: `span(e, &off, &len)`
// gives entry e's bytes (false: offsets rejected, equal to nothing) and
// `byte(off, k)` one of them; entries [0, C) are frames lo .. lo + C - 1, the
// tile's own frames entries [own0, C).
template <class SpanF, class ByteF>
__device__ __forceinline__ void dedup_tile(const DedupArgs& a, uint64_t lo, uint32_t C, uint32_t own0,
                                           uint32_t* lh, int16_t* nxt, int* head, uint32_t nb, SpanF span,
                                           ByteF byte) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t b = tid; b < nb; b += kBlock) head[b] = -1;
  for (uint32_t e = tid; e < C; e += kBlock) {
    uint64_t off;
    uint32_t len;
    lh[e] = span(e, &off, &len) ? small_hash(len, [&](uint32_t k) { return byte(off, k); }) : 0u;
  }
  __syncthreads();
  for (uint32_t e = tid; e < C; e += kBlock)
    if (lh[e]) nxt[e] = (int16_t)atomicExch(&head[lh[e] & (nb - 1u)], (int)e);
  __syncthreads();
  for (uint32_t e = own0 + tid; e < C; e += kBlock) {  // lane-strided: coalesced flags
    const uint64_t i = lo + e;
    const uint32_t h = lh[e];
    uint8_t dup = RUDP_DUP_BAD_OFFSETS;
    if (h) {
      dup = 0;
      const uint32_t emin = (uint32_t)((i > a.window ? i - a.window : 0) - lo);
      uint64_t oi;
      uint32_t li;
      span(e, &oi, &li);
      const uint32_t ci = li ? li : 5u;
      for (int c = head[h & (nb - 1u)]; c >= 0 && !dup; c = nxt[c]) {
        const uint32_t u = (uint32_t)c;
        if (u < emin || u >= e || lh[u] != h) continue;
        uint64_t ou;
        uint32_t lu;
        span(u, &ou, &lu);
        if ((lu ? lu : 5u) != ci) continue;
        uint32_t diff = 0;
        for (uint32_t k = 0; k < ci && !diff; ++k)
          diff = (li ? byte(oi, k) : 0u) ^ (lu ? byte(ou, k) : 0u);
        dup = diff ? 0 : 1;
      }
    }
    a.dup[i] = dup;
  }
}

// LDS of the one-launch form: offsets u32 [cmax + 1] | hashes u32 [cmax] |
// chain links i16 [cmax] | bucket heads i32 [nb] | the run [cap].
__host__ __device__ inline uint32_t dedup_small_lds(uint32_t cmax, uint32_t nb, uint32_t cap) {
  return 4u * ((cmax + 1u + 3u) & ~3u) + 4u * cmax + 2u * ((cmax + 1u) & ~1u) + 4u * nb + cap;
}

// Offsets and run vectors a thread stages (loads all issued before any is used).
constexpr uint32_t kDedupOffPer = 9;    // (T + kDedupSmallWin + 1) / kBlock, FPT = 4
constexpr uint32_t kDedupVecPer = 11;   // the largest budget / 16 / kBlock

template <uint32_t FPT>
__global__ void __launch_bounds__(kBlock) dedup_small_kernel(DedupArgs a, uint32_t nb, uint32_t cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr uint32_t T = kBlock * FPT;
  static_assert(T + kDedupSmallWin + 1 <= kDedupOffPer * kBlock, "offsets per thread");
  const uint32_t W = a.window;
  const uint32_t tid = threadIdx.x;
  const uint64_t p0 = (uint64_t)xcd_tile(blockIdx.x, gridDim.x) * T;
  const uint64_t p1 = p0 + T < a.n ? p0 + T : a.n;
  const uint64_t lo = p0 > W ? p0 - W : 0;
  const uint32_t C = (uint32_t)(p1 - lo), own0 = (uint32_t)(p0 - lo);
  const uint32_t cmax = T + W;
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds_raw);                 // [cmax + 1]
  uint32_t* lh = s_off + ((cmax + 1u + 3u) & ~3u);                        // [cmax]
  int16_t* nxt = reinterpret_cast<int16_t*>(lh + cmax);                  // [cmax]
  int* head = reinterpret_cast<int*>(nxt + ((cmax + 1u) & ~1u));         // [nb]
  unsigned char* img = reinterpret_cast<unsigned char*>(head + nb);      // the run [cap]
  // first round trip: the tile's offsets, and its outer two (every lane) for the run
  uint64_t o[kDedupOffPer];
#pragma unroll
  for (uint32_t j = 0; j < kDedupOffPer; ++j) {
    const uint32_t e = j * kBlock + tid;
    o[j] = e <= C ? a.frame_off[lo + e] : 0;
  }
  const uint64_t lim = a.lim_checked ? a.frames_lim : a.frame_off[a.n];
  const uint64_t f_lo = a.frame_off[lo], f_hi = a.frame_off[p1];
  const uint64_t A = f_lo & ~15ull;
  const uint64_t run = ((f_hi + 15u) & ~15ull) - A;
  // The tile's run is staged when its outer offsets are in order, inside the
  // buffer and within budget, and every inner offset falls inside it (else a
  // frame could be valid yet reach outside the run): otherwise the same work
  // straight from HBM.
  bool staged = f_lo <= f_hi && f_hi <= lim && run <= cap;
  uint32_t outside = 0;
  if (staged) {
    // second round trip: the run, every vector load issued before the offsets are stored
    const uint32_t nvec = (uint32_t)(run >> 4);
    const uint64_t whole = lim > A ? (lim - A) >> 4 : 0;
    u32x4 r[kDedupVecPer];
#pragma unroll
    for (uint32_t j = 0; j < kDedupVecPer; ++j) {
      const uint32_t v = j * kBlock + tid;
      if (v < nvec)
        r[j] = v < whole ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.frames + A) + v)
                         : load16_guarded(a.frames, A + 16ull * v, lim);
    }
#pragma unroll
    for (uint32_t j = 0; j < kDedupOffPer; ++j) {
      const uint32_t e = j * kBlock + tid;
      if (e <= C) {
        const bool in = o[j] >= f_lo && o[j] <= f_hi;
        outside |= in ? 0u : 1u;
        s_off[e] = in ? (uint32_t)(o[j] - A) : 0u;
      }
    }
    u32x4* dst = reinterpret_cast<u32x4*>(img);
#pragma unroll
    for (uint32_t j = 0; j < kDedupVecPer; ++j) {
      const uint32_t v = j * kBlock + tid;
      if (v < nvec) dst[v] = r[j];
    }
  }
  staged = !__syncthreads_or((int)(!staged || outside));
  if (staged) {
    const uint32_t rlim = (uint32_t)(f_hi - A);
    dedup_tile(
        a, lo, C, own0, lh, nxt, head, nb,
        [&](uint32_t e, uint64_t* off, uint32_t* len) {
          const uint32_t fs = s_off[e], fe = s_off[e + 1];
          *off = fs;
          *len = fe - fs;
          return fs <= fe && fe <= rlim;  // (inner offsets in order: the checked rule)
        },
        [&](uint64_t off, uint32_t k) { return (uint32_t)img[off + k]; });
  } else {
    dedup_tile(
        a, lo, C, own0, lh, nxt, head, nb,
        [&](uint32_t e, uint64_t* off, uint32_t* len) {
          // (an unchecked caller's offsets are valid by contract; checking them
          // anyway keeps a bad one from reading past the buffer)
          const uint64_t fo = a.frame_off[lo + e], fe = a.frame_off[lo + e + 1];
          const bool ok = fo <= fe && fe <= lim;
          *off = ok ? fo : 0;
          *len = ok ? (uint32_t)(fe - fo) : 0u;
          return ok;
        },
        [&](uint64_t off, uint32_t k) { return (uint32_t)a.frames[off + k]; });
  }
}

int launch_dedup(const DedupArgs& args, hipStream_t stream) {
  if (args.n == 0) return 0;
  if (args.small_cap) {
    auto launch = [&](auto fpt) -> int {
      constexpr uint32_t FPT = decltype(fpt)::value, T = kBlock * FPT;
      const uint32_t cmax = T + args.window;
      uint32_t nb = 256;  // buckets: chains of 1-2 entries
      while (2u * nb < cmax) nb <<= 1;
      const size_t lds = dedup_small_lds(cmax, nb, args.small_cap);
      if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dedup_small_kernel<FPT>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
      }
      const uint64_t blocks = (args.n + T - 1) / T;
      hipLaunchKernelGGL((dedup_small_kernel<FPT>), dim3((uint32_t)blocks), dim3(kBlock), lds, stream, args, nb,
                         args.small_cap);
      return (int)hipGetLastError();
    };
    // 1024-frame tiles; 512 (rudpx_tune 70 = 2) for the A/B
    if (tuning().dedup_small_fpt == 2) return launch(std::integral_constant<uint32_t, 2>{});
    return launch(std::integral_constant<uint32_t, 4>{});
  }
  const uint64_t hblocks = ((args.n << args.glog) + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(dedup_hash_kernel, dim3((uint32_t)hblocks), dim3(kBlock), 0, stream, args);
  const uint64_t wblocks = (args.n + kBlock - 1) / kBlock;
  if (tuning().dedup_table) {
    const uint32_t cap = args.window + kBlock;
    uint32_t nb = 256;
    while (nb < 2u * cap && nb < 4096u) nb <<= 1;
    const size_t lds = (size_t)cap * (sizeof(uint64_t) + sizeof(int)) + (size_t)nb * sizeof(int);
    if (lds > 65536) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dedup_table_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(dedup_table_kernel, dim3((uint32_t)wblocks), dim3(kBlock), lds, stream, args, nb);
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)(args.window + kBlock) * sizeof(uint64_t);
  hipLaunchKernelGGL(dedup_window_kernel, dim3((uint32_t)wblocks), dim3(kBlock), lds, stream, args);
  return (int)hipGetLastError();
}

uint32_t dedup_max_window() { return kMaxWindow; }

// Retransmission counts of a batch by side: counts[side[i]] += (dup[i] == 1)
// (proxy.py:90-91: client_/server_retransmitted).  Per block in LDS, then one
// atomic per side per block.
__global__ void __launch_bounds__(kBlock) dedup_count_kernel(const uint8_t* dup, const uint8_t* side, uint64_t n,
                                                             unsigned long long* counts) {
  __shared__ unsigned int s_c[2];
  if (threadIdx.x < 2) s_c[threadIdx.x] = 0;
  __syncthreads();
  unsigned int c0 = 0, c1 = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const unsigned int d = dup[i] == 1 ? 1u : 0u;
    if (side && side[i]) c1 += d;
    else c0 += d;
  }
  for (int m = 32; m > 0; m >>= 1) {
    c0 += (unsigned int)__shfl_xor((int)c0, m, 64);
    c1 += (unsigned int)__shfl_xor((int)c1, m, 64);
  }
  if ((threadIdx.x & 63u) == 0) {
    if (c0) atomicAdd(&s_c[0], c0);
    if (c1) atomicAdd(&s_c[1], c1);
  }
  __syncthreads();
  if (threadIdx.x < 2 && s_c[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)s_c[threadIdx.x]);
}

int launch_dedup_count(const uint8_t* dup, const uint8_t* side, uint64_t n, uint64_t* counts, hipStream_t stream) {
  if (n == 0) return 0;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(dedup_count_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, dup, side, n,
                     reinterpret_cast<unsigned long long*>(counts));
  return (int)hipGetLastError();
}

uint32_t dedup_small_cap(uint32_t mean_len, uint32_t window) {
  if (!tuning().dedup_small || !tuning().dedup_table || window > kDedupSmallWin || mean_len > kDedupSmallLen)
    return 0;
  // the tile's and its window's frames at 1.25x the mean length (a burst past it
  // takes the same work from HBM inside the launch)
  const uint64_t C = (uint64_t)kBlock * 4u + window;
  const uint64_t cap = (C * (mean_len ? mean_len : 1u) * 5u / 4u + 256u + 15u) & ~15ull;
  return cap <= 16ull * kDedupVecPer * kBlock ? (uint32_t)cap : 0u;
}

}  // namespace rudp
