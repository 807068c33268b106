// Block-wide scan shared by the offset scan (scan.hip) and the small-frame
// varlen encode, which folds the scan's last pass into its own tile (varlen.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec_device.hpp"  // RUDP_NS

namespace RUDP_NS {

// Status bits of a block live above bit 56 of its pass-1 block sum (a sum of
// at most 2048 x (2^32 - 1 + 7) fits in 44 bits); bits 44-55 hold the
// varlen tile kernel's count of likely overflowing packet tiles (SpanStarts).
constexpr int kSumBitsShift = 56;
constexpr int kSumCountShift = 44;
constexpr uint64_t kSumMask = (1ull << kSumCountShift) - 1ull;

// Exclusive scan of one u64 per thread over the block (all threads call it).
__device__ inline uint64_t block_exclusive_scan(uint64_t x, uint64_t* total, uint64_t* s_wave) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  uint64_t incl = x;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t w = 0; w < nwaves; ++w) {
    const uint64_t v = s_wave[w];
    before += w < wave ? v : 0;
    all += v;
  }
  __syncthreads();  // s_wave may be reused by the caller
  *total = all;
  return before + incl - x;
}

}  // namespace rudp
