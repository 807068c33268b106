// Non-ABI experiment hooks of the tools build (librudp_tools.so, RUDP_TOOLS=1;
// not declared in include/rudp.h, not in librudp.so): launch-policy knobs for
// kernel sweeps, tile timelines, wall-clock stamps, and plain streaming copies
// that measure the device-to-device bandwidth ceiling next to the codec
// (SURVEY.md §8d).
#include <atomic>

#include "codec_device.hpp"
#include "internal.hpp"

#if RUDP_TOOLS
namespace RUDP_NS {

Tuning& tuning() {
  static Tuning t;
  return t;
}

// dwordx4 grid-stride copy: the HBM ceiling a byte-moving kernel can reach.
__global__ void __launch_bounds__(kBlock) copy_kernel(const u32x4* __restrict__ src,
                                                      u32x4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * kBlock)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// Each thread moves VPT vectors: all loads first, then all stores.
template <int VPT, int POLICY>
__global__ void __launch_bounds__(kBlock) copy_vpt_kernel(const u32x4* __restrict__ src,
                                                          u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t base = (uint64_t)blockIdx.x * kBlock * VPT + threadIdx.x;
  u32x4 v[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const uint64_t i = base + (uint64_t)k * kBlock;
    if (i < n16) v[k] = POLICY ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const uint64_t i = base + (uint64_t)k * kBlock;
    if (i < n16) {
      if (POLICY) __builtin_nontemporal_store(v[k], dst + i);
      else dst[i] = v[k];
    }
  }
}

template <int VPT, int POLICY>
int launch_copy_vpt(const void* src, void* dst, uint64_t n16, hipStream_t s) {
  const uint64_t blocks = (n16 + (uint64_t)kBlock * VPT - 1) / ((uint64_t)kBlock * VPT);
  hipLaunchKernelGGL((copy_vpt_kernel<VPT, POLICY>), dim3((uint32_t)blocks), dim3(kBlock), 0, s,
                     (const u32x4*)src, (u32x4*)dst, n16);
  return (int)hipGetLastError();
}

// Diagnostic: the encode kernel's memory pattern with no compute.  A block
// streams a contiguous tile of `tile16` vectors into LDS (lane t: t, t+256,
// ...), barriers, and streams it back out contiguously from LDS.
__global__ void __launch_bounds__(kBlock) copy_tile_kernel(const u32x4* __restrict__ src,
                                                           u32x4* __restrict__ dst, uint64_t n16,
                                                           uint32_t tile16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  u32x4* t = reinterpret_cast<u32x4*>(lds);
  const uint64_t base = (uint64_t)blockIdx.x * tile16;
  const uint32_t m = (uint32_t)((n16 - base) < tile16 ? (n16 - base) : tile16);
  for (uint32_t v0 = threadIdx.x; v0 < m; v0 += 8u * kBlock) {
    u32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t v = v0 + (uint32_t)u * kBlock;
      if (v < m) r[u] = __builtin_nontemporal_load(src + base + v);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t v = v0 + (uint32_t)u * kBlock;
      if (v < m) t[v] = r[u];
    }
  }
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < m; v += kBlock) __builtin_nontemporal_store(t[v], dst + base + v);
}

// Diagnostic: persistent tiled copy with the next tile's loads in flight
// while the current tile drains from LDS (tile16 <= 8 * 256).
__global__ void __launch_bounds__(kBlock) copy_tile_pipe_kernel(const u32x4* __restrict__ src,
                                                                u32x4* __restrict__ dst,
                                                                uint64_t n16, uint32_t tile16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  u32x4* t = reinterpret_cast<u32x4*>(lds);
  const uint64_t ntiles = (n16 + tile16 - 1) / tile16;
  uint64_t tile = blockIdx.x;
  u32x4 r[8];
  auto fetch = [&](uint64_t tl) {
    const uint64_t base = tl * tile16;
    const uint32_t m = (uint32_t)((n16 - base) < tile16 ? (n16 - base) : tile16);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t v = threadIdx.x + (uint32_t)u * kBlock;
      if (v < m) r[u] = __builtin_nontemporal_load(src + base + v);
    }
  };
  if (tile < ntiles) fetch(tile);
  while (tile < ntiles) {
    const uint64_t base = tile * tile16;
    const uint32_t m = (uint32_t)((n16 - base) < tile16 ? (n16 - base) : tile16);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t v = threadIdx.x + (uint32_t)u * kBlock;
      if (v < m) t[v] = r[u];
    }
    __syncthreads();
    const uint64_t next = tile + gridDim.x;
    if (next < ntiles) fetch(next);
    for (uint32_t v = threadIdx.x; v < m; v += kBlock) __builtin_nontemporal_store(t[v], dst + base + v);
    __syncthreads();
    tile = next;
  }
}


// Diagnostic: tiled copy staged by LDS-DMA (global_load_lds_dwordx4).  PIPE:
// persistent blocks with two LDS buffers; the next tile's DMA is in flight
// while the current tile drains from LDS to HBM.
__device__ __forceinline__ void dma_tile(const u32x4* src, u32x4* buf, uint32_t m) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t v0 = threadIdx.x & ~63u; v0 < m; v0 += kBlock)
    if (v0 + lane < m)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src + v0 + lane),
                                       (void __attribute__((address_space(3)))*)(buf + v0), 16, 0, 2);
}

template <bool PIPE>
__global__ void __launch_bounds__(kBlock) copy_tile_dma_kernel(const u32x4* __restrict__ src,
                                                               u32x4* __restrict__ dst, uint64_t n16,
                                                               uint32_t tile16) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  u32x4* t = reinterpret_cast<u32x4*>(lds);
  const uint64_t ntiles = (n16 + tile16 - 1) / tile16;
  uint64_t tile = blockIdx.x;
  const uint64_t stride = PIPE ? gridDim.x : ntiles;
  uint32_t buf = 0;
  auto count = [&](uint64_t tl) {
    const uint64_t base = tl * tile16;
    return (uint32_t)((n16 - base) < tile16 ? (n16 - base) : tile16);
  };
  if (tile < ntiles) dma_tile(src + tile * tile16, t, count(tile));
  while (tile < ntiles) {
    __syncthreads();  // vmcnt(0): this tile's DMA has landed; the other buffer is free
    const uint64_t next = tile + stride;
    if (next < ntiles) dma_tile(src + next * tile16, t + (buf ^ 1u) * tile16, count(next));
    const uint32_t m = count(tile);
    const u32x4* b = t + buf * tile16;
    for (uint32_t v = threadIdx.x; v < m; v += kBlock)
      __builtin_nontemporal_store(b[v], dst + tile * tile16 + v);
    tile = next;
    buf ^= 1u;
  }
}

// Diagnostics: one lane writes the 100 MHz wall clock (a vector store), so a
// tool can stamp the stream before and after a launch.
__global__ void stamp_kernel(uint64_t* dst) {
  if (threadIdx.x == 0) {
    const uint64_t t = (uint64_t)wall_clock64();
    *reinterpret_cast<u32x4*>(dst) = u32x4{(uint32_t)t, (uint32_t)(t >> 32), 0u, 0u};
  }
}

}  // namespace rudp

extern "C" {

// Persistent pipelined tiled copy (diagnostic): `blocks` workgroups.
RUDP_API int rudpx_copy_tile_pipe(const void* src, void* dst, uint64_t n16, uint32_t tile16, uint32_t blocks,
                         uint32_t lds_bytes, void* stream) {
  if (tile16 == 0 || tile16 > 8u * RUDP_NS::kBlock || blocks == 0) return -22;
  size_t lds = (size_t)tile16 * 16;
  if (lds_bytes > lds) lds = lds_bytes;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&RUDP_NS::copy_tile_pipe_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(RUDP_NS::copy_tile_pipe_kernel, dim3(blocks), dim3(RUDP_NS::kBlock), lds,
                     (hipStream_t)stream, (const RUDP_NS::u32x4*)src, (RUDP_NS::u32x4*)dst, n16, tile16);
  return (int)hipGetLastError();
}

// LDS-DMA tiled copy (diagnostic).  pipe = 0: one tile per block; pipe = 1:
// `blocks` persistent blocks, double-buffered.  lds_bytes >= 2*tile16*16 sets occupancy.
RUDP_API int rudpx_copy_tile_dma(const void* src, void* dst, uint64_t n16, uint32_t tile16, uint32_t blocks,
                        uint32_t lds_bytes, int pipe, void* stream) {
  if (tile16 == 0 || tile16 > 4096u) return -22;
  const uint64_t ntiles = (n16 + tile16 - 1) / tile16;
  size_t lds = (size_t)tile16 * 16 * (pipe ? 2 : 1);
  if (lds_bytes > lds) lds = lds_bytes;
  const void* fn = pipe ? reinterpret_cast<const void*>(&RUDP_NS::copy_tile_dma_kernel<true>)
                        : reinterpret_cast<const void*>(&RUDP_NS::copy_tile_dma_kernel<false>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  const uint32_t grid = pipe ? (uint32_t)(blocks < ntiles ? blocks : ntiles) : (uint32_t)ntiles;
  if (pipe)
    hipLaunchKernelGGL(RUDP_NS::copy_tile_dma_kernel<true>, dim3(grid), dim3(RUDP_NS::kBlock), lds,
                       (hipStream_t)stream, (const RUDP_NS::u32x4*)src, (RUDP_NS::u32x4*)dst, n16, tile16);
  else
    hipLaunchKernelGGL(RUDP_NS::copy_tile_dma_kernel<false>, dim3(grid), dim3(RUDP_NS::kBlock), lds,
                       (hipStream_t)stream, (const RUDP_NS::u32x4*)src, (RUDP_NS::u32x4*)dst, n16, tile16);
  return (int)hipGetLastError();
}

// LDS-staged tile copy (diagnostic); lds_bytes >= tile16*16 sets occupancy.
RUDP_API int rudpx_copy_tile(const void* src, void* dst, uint64_t n16, uint32_t tile16, uint32_t lds_bytes,
                    void* stream) {
  const uint64_t blocks = (n16 + tile16 - 1) / tile16;
  size_t lds = (size_t)tile16 * 16;
  if (lds_bytes > lds) lds = lds_bytes;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&RUDP_NS::copy_tile_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(RUDP_NS::copy_tile_kernel, dim3((uint32_t)blocks), dim3(RUDP_NS::kBlock), lds,
                     (hipStream_t)stream, (const RUDP_NS::u32x4*)src, (RUDP_NS::u32x4*)dst, n16, tile16);
  return (int)hipGetLastError();
}

// Copy with VPT (1, 2, 4, 8, 16) vectors per thread, loads before stores;
// policy 1 = non-temporal, 0 = default.
RUDP_API int rudpx_copy_vpt(const void* src, void* dst, uint64_t n16, int vpt, int policy, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  using namespace RUDP_NS;
  switch (vpt * 2 + (policy ? 1 : 0)) {
    case 2: return launch_copy_vpt<1, 0>(src, dst, n16, s);
    case 3: return launch_copy_vpt<1, 1>(src, dst, n16, s);
    case 4: return launch_copy_vpt<2, 0>(src, dst, n16, s);
    case 5: return launch_copy_vpt<2, 1>(src, dst, n16, s);
    case 8: return launch_copy_vpt<4, 0>(src, dst, n16, s);
    case 9: return launch_copy_vpt<4, 1>(src, dst, n16, s);
    case 16: return launch_copy_vpt<8, 0>(src, dst, n16, s);
    case 17: return launch_copy_vpt<8, 1>(src, dst, n16, s);
    case 32: return launch_copy_vpt<16, 0>(src, dst, n16, s);
    case 33: return launch_copy_vpt<16, 1>(src, dst, n16, s);
    default: return -22;
  }
}

// key 0: encode non-temporal loads (0/1); 1: non-temporal stores (0/1);
// 2: packets per encode tile (power of two 16..256, 0 = auto); 3: encode phase-1
// loads in flight per lane (2, 4, 8); 4: decode-verify log2 lanes per packet
// (1..4, -1 = auto); 5: XCD-contiguous tile order; 6: encode tiles per CU cap;
// (7: per-packet phase-1 loads, lost to the contiguous stream, removed); 8: host pipeline
// slots; 9: host pipeline MiB per slot; 10: encode tile workgroup size;
// 11: copy-out decode through an LDS tile; 12: verify-only decode through an LDS tile;
// (13: encode stage ablation, removed with its kernel branches); 14: varlen vector kernels; 15: varlen lanes log2;
// 16: varlen encode through LDS tiles (packed payloads); 17: most packets per
// varlen tile; 18: varlen tile payload bytes at the hint; 20: register-streamed
// encode; 21: its packets per workgroup (0 auto); 22: its load rounds in flight;
// 23: output wave stores start on 64-B sector boundaries; 24: varlen frame
// offsets by the three-pass scan (1) or hipcub (0); 25: encode phase 1 by LDS-DMA;
// 26: encode by fixed output spans; 27: span bytes per workgroup; (28: decode and
// varlen-encode phase 1 by LDS-DMA, measured no faster and removed); 29: encode phase 2 with prebuilt header chunks;
// 30: encode header-table loads before phase 1; 31: fixed-stride UTF-8 validation
// through LDS tiles; 32: dedup window pass by LDS hash table; 33: varlen decode
// through LDS tiles; 34: decode tile outputs staged in LDS; (35: varlen encode tile
// stage ablation, removed); 36: varlen encode tile prebuilt header chunks;
// 37: encode header chunks through an LDS scratch; 38: varlen decode tile LDS budget (%);
// 39: varlen encode tile LDS budget (%); 40: decode tiles per CU cap; 41: packed-frame
// UTF-8 validation through LDS tiles; 42: its LDS budget (%); 43: varlen tile
// offsets before phase 1; 44: varlen encode tile waves per SIMD; 45: packed UTF-8
// tile bytes; 46: small-frame varlen encode below this hint (0 = off); 47: its
// packets per thread; 48: fixed-length encode packets per launch (0 = one launch);
// 49: XCD-contiguous tile order in the decode / varlen / UTF-8 tile kernels;
// 50: small-frame encode finds its tile bases itself (no pass-2 launch);
// 51: varlen byte tiles (0 never, 1 when the scan counts overflowing packet tiles, 2 always);
// 52: varlen tile sum pass (2 from 128-B block sums, 0 chunk by chunk);
// 62: packed small-frame dedup in one launch (dedup_small_kernel; 0: two passes);
// 63: varlen decode tile frame sums from 128-B block sums (0: chunk by chunk);
// 64: a checked small-frame encode of one tile in one launch (no pass 1);
// 71: *_host pipeline: least chunks for a batch over 4 MiB (copy / kernel overlap).
// 73: *_host varlen decode: per-frame outputs stored by the kernels into pinned host arrays (1) or copied (0).
// 74: small-frame varlen encode: pass 1's length codes for the framing kernel (1) or len[] again (0).
// 75: *_host varlen calls of small frames in pinned memory: one zero-copy launch (1) or the slot pipeline (0).
// (72: a first-round stagger of half the fused decode tiles' workgroups (s_sleep),
// 0.539 -> 0.540-0.543 ms on multi-byte text, ASCII 0.229 -> 0.231-0.233: removed;
// profiles/r05/sweeps/utf8_decode_stagger.json.)
// (54: chunked / rotated XCD orders, measured within 2% and removed;
// profiles/r02/headline/xcd_orders.json.)
// (55, 56: a small-tile launch tail, and 57: persistent workgroups looping over the tiles,
// for the 64-B encode: tail within +-2%, persistent 1-30% slower; removed;
// profiles/r03/sweeps/encode64_*.json, encode_persistent_256_1024_1472.json.)
// (58: phase-2 LDS windows from aligned ds_read_b128 pairs: 20x fewer bank conflicts, same
// kernel time; removed; profiles/r03/sq_counters_encode_tiles.json.)
// Returns the old value.
RUDP_API int rudpx_tune(int key, int value) {
  RUDP_NS::Tuning& t = RUDP_NS::tuning();
  std::atomic<int>* slot = key == 0 ? &t.encode_nt_load : key == 1 ? &t.encode_nt_store
            : key == 2 ? &t.encode_tile : key == 3 ? &t.encode_p1
            : key == 4 ? &t.decode_glog : key == 5 ? &t.encode_xcd_swizzle
            : key == 6 ? &t.encode_blocks_per_cu
            : key == 8 ? &t.host_slots : key == 9 ? &t.host_stage_mb
            : key == 10 ? &t.encode_block : key == 11 ? &t.decode_copy_tile
            : key == 12 ? &t.decode_verify_tile : key == 14 ? &t.varlen_vec : key == 15 ? &t.varlen_glog
            : key == 16 ? &t.varlen_tile : key == 17 ? &t.varlen_tile_maxT
            : key == 18 ? &t.varlen_tile_bytes : key == 23 ? &t.out_align64 : key == 24 ? &t.varlen_scan : key == 25 ? &t.encode_dma
            : key == 29 ? &t.encode_hchunk
            : key == 30 ? &t.encode_early_table
            : key == 31 ? &t.utf8_tile
            : key == 32 ? &t.dedup_table
            : key == 33 ? &t.varlen_decode_tile
            : key == 34 ? &t.decode_stage_out
            : key == 36 ? &t.varlen_hchunk
            : key == 37 ? &t.encode_hc_scratch
            : key == 38 ? &t.varlen_decode_cap_pct
            : key == 39 ? &t.varlen_encode_cap_pct
            : key == 40 ? &t.decode_blocks_per_cu
            : key == 41 ? &t.utf8_vtile
            : key == 42 ? &t.utf8_vtile_cap_pct
            : key == 43 ? &t.varlen_early_fo
            : key == 44 ? &t.varlen_waves
            : key == 45 ? &t.utf8_vtile_bytes
            : key == 46 ? &t.varlen_small
            : key == 47 ? &t.varlen_small_fpt
            : key == 48 ? &t.encode_launch_packets
            : key == 49 ? &t.tile_xcd
            : key == 50 ? &t.varlen_small_fused
            : key == 51 ? &t.varlen_btile
            : key == 52 ? &t.varlen_tile_sums
            : key == 59 ? &t.varlen_span_bytes
            : key == 61 ? &t.varlen_diag
            : key == 62 ? &t.dedup_small
            : key == 63 ? &t.varlen_decode_blocks
            : key == 64 ? &t.varlen_small_single
            : key == 65 ? &t.varlen_decode_span
            : key == 66 ? &t.varlen_decode_span_bytes
            : key == 67 ? &t.varlen_map_bal
            : key == 68 ? &t.varlen_decode_nt
            : key == 69 ? &t.varlen_decode_r4
            : key == 70 ? &t.dedup_small_fpt
            : key == 71 ? &t.host_min_chunks
            : key == 73 ? &t.host_direct_out
            : key == 74 ? &t.varlen_small_nib
            : key == 75 ? &t.host_zero_copy : nullptr;
  if (!slot) return -22;
  return slot->exchange(value);
}

// Diagnostics: while `buf` is non-null, every fixed-length encode tile writes
// {start, end (100 MHz wall clock), XCC id, CU id, phase-1 loads landed, sums
// done} as 6 u64 at buf[6 * tile], and every small-frame encode tile {start,
// base known, end, XCC id} at buf[4 * tile].  Not thread-safe; tools only.
RUDP_API int rudpx_encode_trace(uint64_t* buf) {
  RUDP_NS::tuning().encode_trace.store(buf);
  return 0;
}

// Writes the wall clock at dst[0] (dst 16-B aligned) when the stream gets there.
RUDP_API int rudpx_stamp(uint64_t* dst, void* stream) {
  hipLaunchKernelGGL(RUDP_NS::stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst);
  return (int)hipGetLastError();
}

// Copy n16 16-byte vectors (both pointers 16-byte aligned) with `blocks` workgroups.
RUDP_API int rudpx_copy(const void* src, void* dst, uint64_t n16, uint32_t blocks, void* stream) {
  hipLaunchKernelGGL(RUDP_NS::copy_kernel, dim3(blocks), dim3(RUDP_NS::kBlock), 0, (hipStream_t)stream,
                     (const RUDP_NS::u32x4*)src, (RUDP_NS::u32x4*)dst, n16);
  return (int)hipGetLastError();
}

// The library's call-temporary footprint on `device`: out[0] = bytes in use in
// its stream-ordered pool (hipMemPoolAttrUsedMemCurrent), out[1] = scratch
// sets held (one per stream that made a call needing temporaries).
RUDP_API int rudpx_scratch_stats(int device, uint64_t* out) {
  out[1] = (uint64_t)RUDP_NS::scratch_sets(device);
  return (int)RUDP_NS::pool_used_bytes(device, &out[0]);
}

}  // extern "C"
#endif  // RUDP_TOOLS
