// Variable-length batches and strict UTF-8 validation.
//
// The reference's real traffic is 5-9 byte frames: one character of UTF-8
// payload per datagram (utils/reliableUDP.py:11, :60).  A varlen batch is the
// header table plus len[N] (+ optional payload_off[N]) over one payload
// buffer.  Frame offsets are the exclusive scan of len[i] + H (hipcub), so the
// frames come out packed back to back exactly as N calls of Packet.to_byte()
// would be concatenated.
//
// Kernels are byte-granular with G = 8 lanes per packet: right for the tiny
// frames this path exists for; the fixed-length tile kernels stay the path
// for MTU-sized batches.
#include <hipcub/hipcub.hpp>

#include "codec_device.hpp"
#include "internal.hpp"

namespace rudp {

constexpr uint32_t kVarLanes = 8;

struct FrameLen {
  const uint32_t* len;
  uint32_t H;
  __host__ __device__ uint64_t operator()(uint64_t i) const { return (uint64_t)len[i] + H; }
};

template <int H>
__global__ void __launch_bounds__(kBlock) encode_varlen_kernel(VarlenArgs a) {
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid = p < a.n;
  uint32_t sum = 0;
  uint64_t fo = 0;
  if (valid) {
    const uint32_t L = a.len[p];
    fo = a.frame_off[p];
    const uint64_t po = a.payload_off ? a.payload_off[p] : fo - p * (uint64_t)H;
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

template <int H>
__global__ void __launch_bounds__(kBlock) decode_varlen_kernel(VarlenArgs a) {
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid = p < a.n;
  uint32_t sum = 0, F = 0;
  uint64_t fo = 0;
  if (valid) {
    fo = a.frame_off[p];
    F = (uint32_t)(a.frame_off[p + 1] - fo);
    for (uint32_t j = (uint32_t)H + g; j < F; j += kVarLanes) {
      const uint32_t b = a.frames[fo + j];
      sum += ((j - H) & 1u) ? (b << 8) : b;
    }
  }
  for (uint32_t m = kVarLanes >> 1; m > 0; m >>= 1) sum += __shfl_xor(sum, (int)m, 64);
  if (valid && g == 0) {
    uint32_t b[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < 7; ++i)
      if (i < F) b[i] = a.frames[fo + i];
    uint32_t seq = (b[0] << 8) | b[1], ack = (b[2] << 8) | b[3];
    if (F < (uint32_t)H) {  // short frame: fields truncated as utils/packet.py:31 slices them
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

// Strict UTF-8 (RFC 3629, as CPython's bytes.decode() accepts it, i.e. what
// utils/packet.py:73 enforces): no overlongs (C0, C1, E0 80-9F, F0 80-8F), no
// surrogates (ED A0-BF), nothing above U+10FFFF (F4 90+, F5-FF), no stray or
// missing continuation bytes.  Byte-parallel: every byte is judged from itself and the three bytes before it, so the
// payload splits over G lanes with no carried state (the approach of SIMD
// UTF-8 validators): byte c at payload index i, with p1 p2 p3 the bytes at
// i-1, i-2, i-3 (0 before the payload start):
//   c is a continuation byte  <=>  p1 is a 2/3/4-byte lead, or p2 a 3/4-byte
//                                  lead, or p3 a 4-byte lead ("expected")
//   C0 C1 F5..FF never appear; after E0 / ED / F0 / F4 the next byte lies in
//   A0-BF / 80-9F / 90-BF / 80-8F; and nothing is still expected at the end.
__device__ __forceinline__ uint32_t utf8_need(uint32_t b) {  // continuation bytes a lead asks for
  return b >= 0xF0 ? 3u : b >= 0xE0 ? 2u : b >= 0xC0 ? 1u : 0u;
}

__device__ __forceinline__ bool utf8_byte_ok(uint32_t c, uint32_t p1, uint32_t p2, uint32_t p3) {
  const bool cont = (c & 0xC0u) == 0x80u;
  const bool expected = utf8_need(p1) >= 1 || utf8_need(p2) >= 2 || utf8_need(p3) >= 3;
  // p1..p3 that are themselves continuation bytes ask for nothing (need() of 80-BF is 0)
  if (cont != expected) return false;
  if (c == 0xC0 || c == 0xC1 || c >= 0xF5) return false;
  if (p1 == 0xE0 && c < 0xA0) return false;
  if (p1 == 0xED && c > 0x9F) return false;
  if (p1 == 0xF0 && c < 0x90) return false;
  if (p1 == 0xF4 && c > 0x8F) return false;
  return true;
}

__global__ void __launch_bounds__(kBlock) validate_utf8_par_kernel(Utf8Args a) {
  const uint32_t g = threadIdx.x & (kVarLanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kVarLanes;
  const bool valid_p = p < a.n;
  uint32_t bad = 0;
  uint64_t fo = 0, fe = 0;
  if (valid_p) {
    if (a.frame_off) {
      fo = a.frame_off[p];
      fe = a.frame_off[p + 1];
    } else {
      fo = p * (uint64_t)a.F;
      fe = fo + a.F;
    }
    const uint64_t s = fo + a.H;  // payload start
    if (s < fe) {
      const uint64_t len = fe - s;
      // lane g judges a contiguous slice of ceil(len / G) bytes
      const uint64_t per = (len + kVarLanes - 1) / kVarLanes;
      const uint64_t b0 = g * per, b1 = b0 + per < len ? b0 + per : len;
      uint32_t p3 = b0 >= 3 ? a.frames[s + b0 - 3] : 0u;
      uint32_t p2 = b0 >= 2 ? a.frames[s + b0 - 2] : 0u;
      uint32_t p1 = b0 >= 1 ? a.frames[s + b0 - 1] : 0u;
      for (uint64_t i = b0; i < b1; ++i) {
        const uint32_t c = a.frames[s + i];
        bad |= utf8_byte_ok(c, p1, p2, p3) ? 0u : 1u;
        p3 = p2;
        p2 = p1;
        p1 = c;
      }
      if (b1 == len && b0 < b1) {  // last slice: nothing may still be expected
        bad |= (utf8_need(p1) >= 1 || utf8_need(p2) >= 2 || utf8_need(p3) >= 3) ? 1u : 0u;
      }
    }
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
constexpr uint32_t kUtf8Lanes = 16;

__device__ __forceinline__ uint32_t byte_of(u32x4 v, int k) {
  const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
  return (w >> (8 * (k & 3))) & 0xFFu;
}

__global__ void __launch_bounds__(kBlock) validate_utf8_vec_kernel(Utf8Args a) {
  const uint32_t g = threadIdx.x & (kUtf8Lanes - 1u);
  const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / kUtf8Lanes;
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
    const uint64_t s = fo + a.H;
    const uint64_t total = a.frame_off ? a.frame_off[a.n] : a.n * (uint64_t)a.F;
    if (s < fe) {
      const uint64_t c_lo = s >> 4, c_hi = (fe - 1) >> 4;
      for (uint64_t c = c_lo + g; c <= c_hi; c += kUtf8Lanes) {
        const uint64_t base = c << 4;
        u32x4 v;
        if (base + 16 <= total) {
          v = *reinterpret_cast<const u32x4*>(a.frames + base);
        } else {  // the batch's last chunk: never read past the buffer
          uint32_t d[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (base + k < total) d[k >> 2] |= (uint32_t)a.frames[base + k] << (8 * (k & 3));
          v.x = d[0];
          v.y = d[1];
          v.z = d[2];
          v.w = d[3];
        }
        const uint32_t prev = base >= 4 && base > s ? *reinterpret_cast<const uint32_t*>(a.frames + base - 4) : 0u;
        // predecessor bytes, zeroed where they fall before the payload start
        uint32_t p3 = (base >= s + 3) ? (prev >> 8) & 0xFFu : 0u;
        uint32_t p2 = (base >= s + 2) ? (prev >> 16) & 0xFFu : 0u;
        uint32_t p1 = (base >= s + 1) ? (prev >> 24) : 0u;
        const bool interior = base >= s && base + 16 <= fe;
        if (interior && ((v.x | v.y | v.z | v.w) & 0x80808080u) == 0 && p1 < 0xC0 && p2 < 0xC0 &&
            p3 < 0xC0)
          continue;  // plain ASCII, nothing pending from before
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
        if (c == c_hi)  // the frame's last chunk: nothing may still be expected
          bad |= (utf8_need(p1) >= 1 || utf8_need(p2) >= 2 || utf8_need(p3) >= 3) ? 1u : 0u;
      }
    }
  }
  for (uint32_t m = kUtf8Lanes >> 1; m > 0; m >>= 1) bad |= __shfl_xor(bad, (int)m, 64);
  if (valid_p && g == 0) a.valid[p] = bad ? 0 : 1;
}

int launch_encode_varlen(const VarlenArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  if (layout == 7)
    hipLaunchKernelGGL(encode_varlen_kernel<7>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  else
    hipLaunchKernelGGL(encode_varlen_kernel<5>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

int launch_decode_varlen(const VarlenArgs& args, int layout, hipStream_t stream) {
  if (args.n == 0) return 0;
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  if (layout == 7)
    hipLaunchKernelGGL(decode_varlen_kernel<7>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  else
    hipLaunchKernelGGL(decode_varlen_kernel<5>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

int launch_validate_utf8(const Utf8Args& args, hipStream_t stream) {
  if (args.n == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(args.frames) & 15u) == 0) {
    const uint64_t blocks = (args.n * kUtf8Lanes + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(validate_utf8_vec_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
    return (int)hipGetLastError();
  }
  const uint64_t blocks = (args.n * kVarLanes + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(validate_utf8_par_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, args);
  return (int)hipGetLastError();
}

// frame_off[0..n] = exclusive scan of len[i] + H, frame_off[n] = total bytes.
int scan_frame_offsets(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                       hipStream_t stream) {
  hipcub::CountingInputIterator<uint64_t> idx(0);
  hipcub::TransformInputIterator<uint64_t, FrameLen, hipcub::CountingInputIterator<uint64_t>> it(
      idx, FrameLen{d_len, H});
  size_t temp = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, temp, it, d_frame_off + 1, (int)n, stream);
  if (e != hipSuccess) return (int)e;
  void* d_temp = nullptr;
  if ((e = hipMallocAsync(&d_temp, temp ? temp : 1, stream)) != hipSuccess) return (int)e;
  e = hipcub::DeviceScan::InclusiveSum(d_temp, temp, it, d_frame_off + 1, (int)n, stream);
  hipError_t e2 = hipMemsetAsync(d_frame_off, 0, sizeof(uint64_t), stream);
  hipError_t e3 = hipFreeAsync(d_temp, stream);
  if (e != hipSuccess) return (int)e;
  if (e2 != hipSuccess) return (int)e2;
  return (int)e3;
}

}  // namespace rudp
