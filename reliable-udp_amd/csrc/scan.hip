// Frame offsets of a variable-length batch: frame_off[i] = sum_{j<i} (len[j] + H),
// frame_off[n] = total bytes (the varlen layout).
//
// Reduce-then-scan in three launches, no temporary allocation beyond one u64
// per 2048 packets:
//   1. block sums of len + H over 2048-packet blocks (coalesced loads);
//   2. one workgroup turns the block sums into exclusive block bases in place
//      and writes frame_off[n];
//   3. each block rescans its lengths through LDS from its base and writes
//      frame_off[] with coalesced stores.
// Replaces hipcub::DeviceScan (17 us for 1M lengths including its state
// init; this form: see DESIGN.md §3 varlen).
//
// With a ScanCheck the same passes validate the batch on the device (the
// sync-free entry points): pass 1 flags lengths over 65535 and gathered
// payloads outside the payload buffer in the top bits of its block sum, pass 2
// checks the packed payload size and the frame buffer's capacity against the
// total and writes the status word every later kernel of the call reads.
#include "codec_device.hpp"
#include "internal.hpp"
#include "scan_device.hpp"

namespace RUDP_NS {

constexpr uint32_t kScanItems = 8;                     // per thread
constexpr uint32_t kScanBlockItems = kBlock * kScanItems;  // 2048 per block


// ITEMS packets per thread: a block sums kBlock * ITEMS lengths (8 for the
// offset scan; the small-frame encode uses its own tile size).
// With over_T (a power of two <= 64): the block's packet tiles of over_T
// consecutive packets -- over_T consecutive lanes of one load -- whose length
// sum + 30 (a bound on their 16-B aligned payload run) exceeds over_cap are
// counted into bits 44-55 of the sum (at most 2048 tiles per block).
// With codes (ITEMS 2 or 4, the small-frame encode's pass): every thread also
// stores its ITEMS lengths in one byte, codes[block * kBlock + thread], as
// 8 / ITEMS-bit offsets from code_base (the all-ones code: any other length,
// read len[] again), so the framing kernel, which takes the same packets per
// thread, reads 1 B per ITEMS packets instead of 4 B per packet.
template <uint32_t ITEMS>
__global__ void __launch_bounds__(kBlock) scan_block_sums_kernel(const uint32_t* len, uint64_t n,
                                                                 uint32_t H, uint64_t* sums,
                                                                 ScanCheck chk, uint32_t over_T,
                                                                 uint32_t over_cap, uint8_t* codes,
                                                                 uint32_t code_base) {
  __shared__ uint64_t s_wave[kBlock / 64];
  __shared__ uint32_t s_bits, s_over;
  if (threadIdx.x == 0) s_bits = s_over = 0;
  const uint64_t base = (uint64_t)blockIdx.x * (kBlock * ITEMS);
  uint64_t acc = 0;
  uint32_t bits = 0, over = 0, code = 0;
#pragma unroll
  for (uint32_t j = 0; j < ITEMS; ++j) {
    const uint64_t i = base + j * kBlock + threadIdx.x;
    const uint32_t l = i < n ? len[i] : 0u;
    if (ITEMS == 2 || ITEMS == 4) {
      constexpr uint32_t B = 8u / ITEMS, M = (1u << B) - 1u;
      const uint32_t c = l - code_base;  // (below the base: wraps high, the escape)
      code |= (c < M ? c : M) << (B * j);
    }
    if (i < n) {
      acc += (uint64_t)l + H;
      if (chk.status) {
        if (l > kMaxPayload) bits |= RUDP_ST_LEN;
        if (chk.payload_off) {
          const uint64_t o = chk.payload_off[i];
          // o + l <= payload_bytes without overflow (o is read as u64: a negative int64 is huge)
          if (o > chk.payload_bytes || (uint64_t)l > chk.payload_bytes - o) bits |= RUDP_ST_PAYLOAD;
        }
      }
    }
    if (over_T) {  // (uniform; lengths clamped: any over 65535 fails the call anyway)
      const uint32_t ts = group_sum(l < 0x10000u ? l : 0x10000u, over_T);
      const bool o = (threadIdx.x & (over_T - 1u)) == 0 && i < n && ts + 30u > over_cap;
      over += (uint32_t)__popcll(__ballot(o));
    }
  }
  if ((ITEMS == 2 || ITEMS == 4) && codes) codes[(uint64_t)blockIdx.x * kBlock + threadIdx.x] = (uint8_t)code;
  acc = wave_sum64(acc);
  __syncthreads();  // s_bits, s_over initialised
  if (bits) atomicOr(&s_bits, bits);
  if ((threadIdx.x & 63u) == 0) {
    s_wave[threadIdx.x >> 6] = acc;
    if (over) atomicAdd(&s_over, over);  // (every lane holds its wave's count)
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w) t += s_wave[w];
    sums[blockIdx.x] = t | ((uint64_t)s_over << kSumCountShift) | ((uint64_t)s_bits << kSumBitsShift);
  }
}

// One workgroup of 1024 threads: sums[b] <- sum_{c<b} sums[c]; frame_off[n] <- total;
// with a ScanCheck, the call's status word.
// With ctl: the varlen tile form, *ctl = 1 (byte tiles) when pass 1 counted at
// least min_over likely overflowing packet tiles, else 0.
__global__ void __launch_bounds__(1024) scan_block_bases_kernel(uint64_t* sums, uint64_t nb,
                                                               uint64_t* frame_off, uint64_t n,
                                                               uint32_t H, ScanCheck chk, uint32_t* ctl,
                                                               uint32_t min_over) {
  __shared__ uint64_t s_wave[1024 / 64];
  __shared__ uint32_t s_bits, s_over;
  if (threadIdx.x == 0) s_bits = s_over = 0;
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint64_t mine = 0;
  uint32_t bits = 0, over = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t v = sums[i];
    mine += v & kSumMask;
    over += (uint32_t)(v >> kSumCountShift) & 0xFFFu;
    bits |= (uint32_t)(v >> kSumBitsShift);
  }
  uint64_t total = 0;
  uint64_t run = block_exclusive_scan(mine, &total, s_wave);  // (its barriers order s_bits, s_over)
  if (bits) atomicOr(&s_bits, bits);
  if (over) atomicAdd(&s_over, over);
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t v = sums[i] & kSumMask;
    sums[i] = run;
    run += v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (ctl) *ctl = s_over >= min_over ? 1u : 0u;
    frame_off[n] = total;
    if (chk.status) {
      uint32_t st = s_bits;
      if (!chk.payload_off && total - n * (uint64_t)H != chk.payload_bytes) st |= RUDP_ST_PAYLOAD;
      if (total > chk.frames_cap) st |= RUDP_ST_FRAMES_CAP;
      *chk.status = st;
    }
  }
}

// With spans.rec: the varlen tile kernel's records in the form pass 2 chose
// (*spans.ctl).  Byte tiles: the packed payload splits into spans of S bytes,
// and span t's record is {frame_off[p], p} for p the first packet whose payload
// starts at or after t*S (n for spans after the last packet's start), t = 0 ..
// spans.count.  Packet tiles: tile k's record is {frame_off[k T], k T}, k = 0
// .. ptiles (the last {total, n}).  Tile k of nt goes to record index
// k + floor(k (grid - nt) / nt), so the grid's workgroups the form does not
// need are spread evenly (over the XCDs too); a skipped index repeats the
// next tile's record, which makes its workgroup's tile empty.
__global__ void __launch_bounds__(kBlock) scan_apply_kernel(const uint32_t* len, uint64_t n, uint32_t H,
                                                            const uint64_t* bases, uint64_t* frame_off,
                                                            SpanStarts spans) {
  __shared__ uint32_t s_len[kScanBlockItems];
  __shared__ uint64_t s_off[kScanBlockItems];
  __shared__ uint32_t s_wave32[kBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlockItems;
  // coalesced load of the block's lengths, then each thread takes 8 in a row
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; ++j) {
    const uint32_t k = j * kBlock + threadIdx.x;
    s_len[k] = base + k < n ? len[base + k] + H : 0u;
  }
  __syncthreads();
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; ++j) mine += s_len[threadIdx.x * kScanItems + j];
  uint32_t total = 0;  // (at most kScanBlockItems * (65535 + H) for lengths that passed pass 1)
  uint64_t run = bases[blockIdx.x] + block_exclusive_scan32(mine, &total, s_wave32);
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; ++j) {
    const uint32_t k = threadIdx.x * kScanItems + j;
    s_off[k] = run;
    run += s_len[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; ++j) {
    const uint32_t k = j * kBlock + threadIdx.x;
    if (base + k < n) frame_off[base + k] = s_off[k];
  }
  if (spans.rec) {
    const uint64_t G = spans.grid;
    auto put = [&](uint64_t k, uint64_t nt, SpanRec r) {
      const uint64_t e = G - nt;
      const uint64_t ri = e ? k + k * e / nt : k;
      const uint64_t r0 = k == 0 ? 0 : (e ? (k - 1) + (k - 1) * e / nt : k - 1) + 1;
      for (uint64_t x = r0; x <= ri; ++x) spans.rec[x] = r;
    };
    if (*spans.ctl) {  // byte tiles
      const uint64_t S = spans.bytes, K = spans.count;
      // x / S through the double reciprocal, corrected to the exact quotient
      // (x < 2^53: the estimate is off by at most one); a u64 division per
      // packet cost 10 us on 1M packets
      const double inv = 1.0 / (double)S;
      auto div_s = [&](uint64_t x) {
        uint64_t d = (uint64_t)((double)x * inv);
        if (d * S > x) --d;
        if ((d + 1u) * S <= x) ++d;
        return d;
      };
#pragma unroll
      for (uint32_t j = 0; j < kScanItems; ++j) {
        const uint32_t k = j * kBlock + threadIdx.x;
        const uint64_t p = base + k;
        if (p >= n) continue;
        const uint64_t po = s_off[k] - p * H;  // packed payload offset of packet p
        uint64_t lo = 0;
        if (p > 0) {
          const uint64_t prev_len = k > 0 ? s_len[k - 1] - H : len[p - 1];
          lo = div_s(po - prev_len) + 1;  // spans after the one the previous packet starts in
        }
        const uint64_t qpo = div_s(po);
        const uint64_t hi = qpo < K ? qpo : K;
        for (uint64_t t = lo; t <= hi; ++t) put(t, K, SpanRec{s_off[k], (uint32_t)p, 0u});
        if (p == n - 1)
          for (uint64_t t = (qpo + 1 > lo ? qpo + 1 : lo); t <= K; ++t)
            put(t, K, SpanRec{s_off[k] + s_len[k], (uint32_t)n, 0u});
      }
    } else {  // packet tiles of spans.tile_T packets (a power of two dividing the block)
      const uint32_t T = spans.tile_T, tiles = kScanBlockItems / T;
      for (uint32_t i = threadIdx.x; i < tiles; i += kBlock) {
        const uint64_t p = base + (uint64_t)i * T;
        if (p < n) put(p / T, spans.ptiles, SpanRec{s_off[i * T], (uint32_t)p, 0u});
      }
      if (threadIdx.x == 0 && base + kScanBlockItems >= n) {  // the last block: the end record
        const uint32_t kl = (uint32_t)(n - 1 - base);
        put(spans.ptiles, spans.ptiles, SpanRec{s_off[kl] + s_len[kl], (uint32_t)n, 0u});
      }
    }
  }
}

void scan_block_sums(const uint32_t* d_len, uint64_t n, uint32_t H, uint32_t items, uint64_t* sums,
                     const ScanCheck& chk, hipStream_t stream, uint32_t over_T, uint32_t over_cap, uint8_t* codes,
                     uint32_t code_base) {
  const uint64_t nb = (n + kBlock * items - 1) / (kBlock * items);
  const dim3 grid((uint32_t)nb), block(kBlock);
  switch (items) {
    case 1: hipLaunchKernelGGL(scan_block_sums_kernel<1>, grid, block, 0, stream, d_len, n, H, sums, chk, 0u, 0u,
                               nullptr, 0u); break;
    case 2: hipLaunchKernelGGL(scan_block_sums_kernel<2>, grid, block, 0, stream, d_len, n, H, sums, chk, 0u, 0u,
                               codes, code_base); break;
    case 4: hipLaunchKernelGGL(scan_block_sums_kernel<4>, grid, block, 0, stream, d_len, n, H, sums, chk, 0u, 0u,
                               codes, code_base); break;
    default: hipLaunchKernelGGL(scan_block_sums_kernel<8>, grid, block, 0, stream, d_len, n, H, sums, chk, over_T,
                                over_cap, nullptr, 0u);
  }
}

void scan_block_bases(uint64_t* sums, uint64_t nb, uint64_t* d_frame_off, uint64_t n, uint32_t H,
                      const ScanCheck& chk, hipStream_t stream, uint32_t* ctl, uint32_t min_over) {
  hipLaunchKernelGGL(scan_block_bases_kernel, dim3(1), dim3(1024), 0, stream, sums, nb, d_frame_off, n, H, chk,
                     ctl, min_over);
}

int scan_frame_offsets_3pass(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                             const ScanCheck& chk, hipStream_t stream, const SpanStarts& spans) {
  const uint64_t nb = (n + kScanBlockItems - 1) / kScanBlockItems;
  uint64_t* sums = nullptr;
  hipError_t e = stream_scratch(reinterpret_cast<void**>(&sums), nb * sizeof(uint64_t), stream, kScratchSums);
  if (e != hipSuccess) return (int)e;
  scan_block_sums(d_len, n, H, kScanItems, sums, chk, stream, spans.rec ? spans.tile_T : 0u, spans.tile_cap);
  scan_block_bases(sums, nb, d_frame_off, n, H, chk, stream, spans.rec ? spans.ctl : nullptr, spans.min_over);
  hipLaunchKernelGGL(scan_apply_kernel, dim3((uint32_t)nb), dim3(kBlock), 0, stream, d_len, n, H, sums,
                     d_frame_off, spans);
  return (int)hipGetLastError();
}

}  // namespace rudp
