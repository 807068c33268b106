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
#include "codec_device.hpp"
#include "internal.hpp"

namespace rudp {

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

int launch_dedup(const DedupArgs& args, hipStream_t stream) {
  if (args.n == 0) return 0;
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

}  // namespace rudp
