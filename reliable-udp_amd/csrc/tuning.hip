// Non-ABI experiment hooks (not declared in include/rudp.h): launch-policy
// knobs for kernel sweeps, and a plain streaming copy used to measure the
// device-to-device bandwidth ceiling next to the codec.
#include <atomic>

#include "codec_device.hpp"
#include "internal.hpp"

namespace rudp {

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

}  // namespace rudp

extern "C" {

// key 0: encode non-temporal loads (0/1); 1: non-temporal stores (0/1);
// 2: packets per encode tile (power of two 16..256, 0 = auto); 3: encode phase-2
// unroll (1, 2); 4: decode-verify log2 lanes per packet (1..4, -1 = auto).
// Returns the old value.
int rudpx_tune(int key, int value) {
  rudp::Tuning& t = rudp::tuning();
  int* slot = key == 0 ? &t.encode_nt_load : key == 1 ? &t.encode_nt_store
            : key == 2 ? &t.encode_tile : key == 3 ? &t.encode_unroll
            : key == 4 ? &t.decode_glog : key == 5 ? &t.encode_xcd_swizzle : nullptr;
  if (!slot) return -22;
  const int old = *slot;
  *slot = value;
  return old;
}

// Copy n16 16-byte vectors (both pointers 16-byte aligned) with `blocks` workgroups.
int rudpx_copy(const void* src, void* dst, uint64_t n16, uint32_t blocks, void* stream) {
  hipLaunchKernelGGL(rudp::copy_kernel, dim3(blocks), dim3(rudp::kBlock), 0, (hipStream_t)stream,
                     (const rudp::u32x4*)src, (rudp::u32x4*)dst, n16);
  return (int)hipGetLastError();
}

}  // extern "C"
