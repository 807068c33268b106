// Deterministic synthetic packet batches, generated on the device.
//
// Counter-based splitmix64: every value is a pure
// function of (seed, global packet index), so a shard generated on GPU g from
// first_index = g*N/G is bit-identical to the same slice of the unsharded
// batch, and the CPU restatement in oracle/synth.py reproduces it exactly.
//   seq     = (isn + i) mod 2^16, isn = 1 + stream(k0, 0) mod 5000
//             (mirrors utils/reliableUDP.py:41 randint(1, 5000) and :54)
//   ack     = stream(k1, i) mod 2^16
//   flags   = {00,80,20,A0,40,60}[hi32(stream(k2, i)) * 6 >> 32]
//             (the flag bytes seen on the wire)
//   payload = little-endian bytes of stream(k3, i*W + w), W = ceil(L/8),
//             masked to 7 bits for ASCII batches (str API, utils/packet.py:63)
#include "codec_device.hpp"
#include "internal.hpp"

namespace RUDP_NS {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t stream64(uint64_t key, uint64_t ctr) {
  return mix64(key + (ctr + 1ull) * 0x9E3779B97F4A7C15ull);
}

__global__ void __launch_bounds__(kBlock) synth_header_kernel(SynthArgs a) {
  // {00,80,20,A0,40,60} packed little-endian: entry k = byte k.
  constexpr uint64_t kFlags = 0x6040A0208000ull;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < a.n;
       i += (uint64_t)gridDim.x * kBlock) {
    const uint64_t gi = a.first + i;
    a.seq[i] = (uint16_t)((a.isn + gi) & 0xFFFFu);
    a.ack[i] = (uint16_t)(stream64(a.key_ack, gi) & 0xFFFFu);
    const uint64_t hi = stream64(a.key_flags, gi) >> 32;
    a.flags[i] = (uint8_t)(kFlags >> (8 * ((hi * 6ull) >> 32)));
  }
}

__global__ void __launch_bounds__(kBlock) synth_payload_kernel(SynthArgs a) {
  const uint32_t L = a.L;
  const uint64_t W = (L + 7u) / 8u;
  const uint64_t total = a.n * W;
  const uint64_t mask = a.ascii ? 0x7F7F7F7F7F7F7F7Full : ~0ull;
  const bool whole = (L % 8u) == 0 && (reinterpret_cast<uintptr_t>(a.payload) % 8u) == 0;
  for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * kBlock) {
    const uint64_t i = t / W;
    const uint64_t w = t - i * W;
    const uint64_t x = stream64(a.key_payload, (a.first + i) * W + w) & mask;
    if (whole) {
      reinterpret_cast<uint64_t*>(a.payload)[t] = x;
    } else {
      unsigned char* dst = a.payload + i * (uint64_t)L + 8u * w;
      const uint32_t nb = (L - 8u * (uint32_t)w) < 8u ? (L - 8u * (uint32_t)w) : 8u;
      for (uint32_t b = 0; b < nb; ++b) dst[b] = (unsigned char)(x >> (8 * b));
    }
  }
}

int launch_synth(const SynthArgs& args, hipStream_t stream) {
  if (args.n == 0) return 0;
  const uint32_t grid = 256u * 16u;
  hipLaunchKernelGGL(synth_header_kernel, dim3(grid), dim3(kBlock), 0, stream, args);
  if (args.L > 0)
    hipLaunchKernelGGL(synth_payload_kernel, dim3(grid), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

}  // namespace rudp
