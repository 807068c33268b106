// Device-side argument checks for the variable-length entry points.
//
// The Python layer needs, before it can size the frame buffer and launch the
// varlen encode, the bounds of the batch: min / max / sum of len[] (and the
// extent of payload_off[]); before a varlen decode, that frame_off[] is
// non-decreasing.  Done with torch ops that was 5-6 reductions and ~55 us per
// call at 1M packets (round-1 probe tools/varlen_overhead.py, in git history) against a 37 us encode; here
// it is a grid-stride pass with per-block partials and one combining block
// that writes the result straight to pinned host memory: 20 us per call with
// the sync (a single launch whose last block combines measured 34 us).
#include <mutex>
#include <vector>

#include "codec_device.hpp"
#include "internal.hpp"

namespace RUDP_NS {

constexpr uint32_t kBoundsBlocks = 256;

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  for (int m = 32; m > 0; m >>= 1) {
    const uint64_t o = __shfl_xor(v, m, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  for (int m = 32; m > 0; m >>= 1) {
    const uint64_t o = __shfl_xor(v, m, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
  for (int m = 32; m > 0; m >>= 1) {
    const int64_t o = __shfl_xor(v, m, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
  for (int m = 32; m > 0; m >>= 1) {
    const int64_t o = __shfl_xor(v, m, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Block-wide combine of one Bounds per thread into out (thread 0 writes).
__device__ void block_combine(Bounds b, Bounds* out) {
  __shared__ Bounds s[kBlock / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  b.min_len = wave_min_u64(b.min_len);
  b.max_len = wave_max_u64(b.max_len);
  b.sum_len = wave_sum_u64(b.sum_len);
  b.min_off = wave_min_i64(b.min_off);
  b.max_end = wave_max_i64(b.max_end);
  b.n_decreasing = wave_sum_u64(b.n_decreasing);
  if (lane == 0) s[wave] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    Bounds r = s[0];
    for (uint32_t w = 1; w < kBlock / 64; ++w) {
      r.min_len = s[w].min_len < r.min_len ? s[w].min_len : r.min_len;
      r.max_len = s[w].max_len > r.max_len ? s[w].max_len : r.max_len;
      r.sum_len += s[w].sum_len;
      r.min_off = s[w].min_off < r.min_off ? s[w].min_off : r.min_off;
      r.max_end = s[w].max_end > r.max_end ? s[w].max_end : r.max_end;
      r.n_decreasing += s[w].n_decreasing;
    }
    *out = r;
  }
}

__device__ __forceinline__ Bounds bounds_identity() {
  Bounds b;
  b.min_len = ~0ull;
  b.max_len = 0;
  b.sum_len = 0;
  b.min_off = INT64_MAX;
  b.max_end = INT64_MIN;
  b.n_decreasing = 0;
  return b;
}

// len[] as u32 (a negative int32 length reads as > 65535 and is rejected the same way).
__global__ void __launch_bounds__(kBlock) len_bounds_kernel(const uint32_t* len, const int64_t* off,
                                                            uint64_t n, Bounds* partial) {
  Bounds b = bounds_identity();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint64_t l = len[i];
    b.min_len = l < b.min_len ? l : b.min_len;
    b.max_len = l > b.max_len ? l : b.max_len;
    b.sum_len += l;
    if (off) {
      const int64_t o = off[i];
      b.min_off = o < b.min_off ? o : b.min_off;
      b.max_end = o + (int64_t)l > b.max_end ? o + (int64_t)l : b.max_end;
    }
  }
  block_combine(b, partial + blockIdx.x);
}

// Pairs (frame_off[i], frame_off[i+1]) for i < n that decrease; min and max
// over all n+1 offsets go into min_off / max_end.
__global__ void __launch_bounds__(kBlock) off_bounds_kernel(const int64_t* off, uint64_t n,
                                                            Bounds* partial) {
  Bounds b = bounds_identity();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i <= n; i += stride) {
    const int64_t o = off[i];
    b.min_off = o < b.min_off ? o : b.min_off;
    b.max_end = o > b.max_end ? o : b.max_end;
    if (i < n && off[i + 1] < o) ++b.n_decreasing;
  }
  block_combine(b, partial + blockIdx.x);
}

__global__ void __launch_bounds__(kBlock) bounds_final_kernel(const Bounds* partial, uint32_t nparts,
                                                              Bounds* out) {
  Bounds b = bounds_identity();
  for (uint32_t i = threadIdx.x; i < nparts; i += kBlock) {
    const Bounds p = partial[i];
    b.min_len = p.min_len < b.min_len ? p.min_len : b.min_len;
    b.max_len = p.max_len > b.max_len ? p.max_len : b.max_len;
    b.sum_len += p.sum_len;
    b.min_off = p.min_off < b.min_off ? p.min_off : b.min_off;
    b.max_end = p.max_end > b.max_end ? p.max_end : b.max_end;
    b.n_decreasing += p.n_decreasing;
  }
  block_combine(b, out);
}

// Scratch for one call: the block partials on the device and the result in
// mapped pinned memory the combining block writes (no copy call).  Kept in a
// mutex-guarded per-device free list: a call takes a slot and gives it back
// when it returns (it is synchronous), so slots are bounded by the peak number
// of concurrent callers and are reused, never freed.
struct BoundsScratch {
  Bounds* d_partial = nullptr;   // [kBoundsBlocks] block partials
  Bounds* h_result = nullptr;
  int device = 0;
};

std::mutex g_bounds_mu;
std::vector<std::vector<BoundsScratch*>> g_bounds_free;

BoundsScratch* bounds_acquire(int device) {
  {
    std::lock_guard<std::mutex> lk(g_bounds_mu);
    if ((int)g_bounds_free.size() <= device) g_bounds_free.resize(device + 1);
    auto& fl = g_bounds_free[device];
    if (!fl.empty()) {
      BoundsScratch* s = fl.back();
      fl.pop_back();
      return s;
    }
  }
  BoundsScratch* s = new BoundsScratch();
  s->device = device;
  if (hipMalloc(reinterpret_cast<void**>(&s->d_partial), sizeof(Bounds) * kBoundsBlocks) != hipSuccess) {
    delete s;
    return nullptr;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&s->h_result), sizeof(Bounds), hipHostMallocMapped) !=
      hipSuccess) {
    (void)hipFree(s->d_partial);
    delete s;
    return nullptr;
  }
  return s;
}

void bounds_release(BoundsScratch* s) {
  std::lock_guard<std::mutex> lk(g_bounds_mu);
  g_bounds_free[s->device].push_back(s);
}

// Runs the pass on `stream` (the current device's) and returns the result in
// *host (synchronous).
int compute_bounds(const uint32_t* len, const int64_t* off, uint64_t n, bool offsets_only,
                   Bounds* host, hipStream_t stream) {
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return (int)e;
  BoundsScratch* s = bounds_acquire(device);
  if (!s) return (int)hipErrorOutOfMemory;
  struct Release {
    BoundsScratch* s;
    ~Release() { bounds_release(s); }
  } release{s};
  const uint64_t items = offsets_only ? n + 1 : n;
  uint64_t want = (items + kBlock * 8 - 1) / (kBlock * 8);  // >= 8 items per thread
  const uint32_t blocks = (uint32_t)(want < 1 ? 1 : want > kBoundsBlocks ? kBoundsBlocks : want);
  Bounds* h_dev = nullptr;
  if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&h_dev), s->h_result, 0)) != hipSuccess)
    return (int)e;
  if (offsets_only)
    hipLaunchKernelGGL(off_bounds_kernel, dim3(blocks), dim3(kBlock), 0, stream, off, n, s->d_partial);
  else
    hipLaunchKernelGGL(len_bounds_kernel, dim3(blocks), dim3(kBlock), 0, stream, len, off, n,
                       s->d_partial);
  // one combining block writes the result straight to pinned host memory
  hipLaunchKernelGGL(bounds_final_kernel, dim3(1), dim3(kBlock), 0, stream, s->d_partial, blocks, h_dev);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(stream)) != hipSuccess) return (int)e;
  *host = *s->h_result;
  return 0;
}

// ---- sync-free offset check -------------------------------------------------
// frame_off[0..n] non-decreasing and inside [0, frames_bytes] (read as u64, so
// a negative offset is out of range).  Block partials, then one block writes
// the status word: no zero-initialisation, no host round trip.
__global__ void __launch_bounds__(kBlock) off_check_kernel(const uint64_t* off, uint64_t n,
                                                           uint64_t frames_bytes, uint32_t* partial) {
  uint32_t bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i <= n; i += stride) {
    const uint64_t o = off[i];
    if (o > frames_bytes || (i < n && off[i + 1] < o)) bad = 1;
  }
  bad = (uint32_t)__syncthreads_or((int)bad);
  if (threadIdx.x == 0) partial[blockIdx.x] = bad;
}

__global__ void __launch_bounds__(kBlock) off_check_final_kernel(const uint32_t* partial, uint32_t nparts,
                                                                 uint32_t* status) {
  uint32_t bad = 0;
  for (uint32_t i = threadIdx.x; i < nparts; i += kBlock) bad |= partial[i];
  bad = (uint32_t)__syncthreads_or((int)bad);
  if (threadIdx.x == 0) *status = bad ? RUDP_ST_OFFSETS : 0u;
}

int check_frame_offsets(const uint64_t* d_frame_off, uint64_t n, uint64_t frames_bytes, uint32_t* d_status,
                        hipStream_t stream) {
  uint64_t want = (n + 1 + kBlock * 8 - 1) / (kBlock * 8);
  const uint32_t blocks = (uint32_t)(want < 1 ? 1 : want > kBoundsBlocks ? kBoundsBlocks : want);
  uint32_t* partial = nullptr;
  hipError_t e = stream_scratch(reinterpret_cast<void**>(&partial), blocks * sizeof(uint32_t), stream,
                                kScratchBounds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(off_check_kernel, dim3(blocks), dim3(kBlock), 0, stream, d_frame_off, n, frames_bytes,
                     partial);
  hipLaunchKernelGGL(off_check_final_kernel, dim3(1), dim3(kBlock), 0, stream, partial, blocks, d_status);
  return (int)hipGetLastError();
}

}  // namespace rudp
