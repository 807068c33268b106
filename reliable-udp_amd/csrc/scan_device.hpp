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

// The same for values whose block total fits 32 bits (lengths of at most a
// few thousand packets): the wave's scan by DPP row shifts (1, 2, 4, 8 within
// each row of 16 lanes) and the three lower rows' totals read by
// v_readlane, instead of six dependent 64-bit shuffle steps.
__device__ __forceinline__ uint32_t wave_inclusive_scan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
  const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
  const uint32_t t2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
  const uint32_t row = (threadIdx.x & 63u) >> 4;
  return x + (row >= 1u ? t0 : 0u) + (row >= 2u ? t1 : 0u) + (row >= 3u ? t2 : 0u);
}
__device__ inline uint32_t block_exclusive_scan32(uint32_t x, uint32_t* total, uint32_t* s_wave) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const uint32_t incl = wave_inclusive_scan32(x);
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (uint32_t w = 0; w < nwaves; ++w) {
    const uint32_t v = s_wave[w];
    before += w < wave ? v : 0u;
    all += v;
  }
  __syncthreads();  // s_wave may be reused by the caller
  *total = all;
  return before + incl - x;
}

}  // namespace rudp
