// Stream-ordered temporaries (scan block sums, dedup hash scratch) from a
// library-owned memory pool per device.
//
// hipMallocAsync from the default pool returns freed memory to the driver at
// every synchronize (release threshold 0), so a call made after a sync pays a
// fresh mapping: the Python varlen entry points sync once per call for their
// bounds checks, and the 8 MB dedup scratch of a 1M-datagram batch cost about
// 230 us per call that way (detect_retransmissions 462 -> 236 us with this
// pool, tools/dedup_overhead.py).  This pool keeps what it has (threshold =
// max) and leaves the process's default pool alone.
#include <mutex>
#include <vector>

#include "internal.hpp"

namespace rudp {

namespace {
std::mutex g_pool_mu;
std::vector<hipMemPool_t> g_pools;
}  // namespace

static hipMemPool_t pool_for_current_device(hipError_t* err) {
  int device = 0;
  *err = hipGetDevice(&device);
  if (*err != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if ((int)g_pools.size() <= device) g_pools.resize(device + 1, nullptr);
  if (!g_pools[device]) {
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    hipMemPool_t pool = nullptr;
    if ((*err = hipMemPoolCreate(&pool, &props)) != hipSuccess) return nullptr;
    uint64_t keep = ~0ull;
    if ((*err = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep)) != hipSuccess) {
      (void)hipMemPoolDestroy(pool);
      return nullptr;
    }
    g_pools[device] = pool;
  }
  return g_pools[device];
}

hipError_t stream_alloc(void** ptr, size_t bytes, hipStream_t stream) {
  hipError_t e = hipSuccess;
  hipMemPool_t pool = pool_for_current_device(&e);
  if (!pool) return e;
  return hipMallocFromPoolAsync(ptr, bytes ? bytes : 1, pool, stream);
}

hipError_t stream_free(void* ptr, hipStream_t stream) { return hipFreeAsync(ptr, stream); }

// Per-call temporaries without an allocation per call: every host thread
// keeps one buffer per (device, stream, slot), grown when a call needs more
// (the old one freed in stream order).  Only this thread enqueues work on
// its buffers, and only on that stream, so the stream's order protects them:
// a call's kernels run after the previous call's on the same stream.  (A
// destroyed stream's handle is released only after its pending work, so a
// new stream with the same handle finds its buffers idle.)  hipFreeAsync
// cost 3.9 us of host time per call (rocprofv3 --hip-trace, 1M one-character
// datagrams), as long as a kernel launch.
namespace {
struct Scratch {
  int device;
  hipStream_t stream;
  int slot;
  void* ptr;
  size_t cap;
};
thread_local std::vector<Scratch> t_scratch;
}  // namespace

hipError_t stream_scratch(void** ptr, size_t bytes, hipStream_t stream, int slot) {
  int device = 0;
  hipError_t e = hipGetDevice(&device);
  if (e != hipSuccess) return e;
  Scratch* hit = nullptr;
  for (auto& sc : t_scratch)
    if (sc.device == device && sc.stream == stream && sc.slot == slot) hit = &sc;
  if (hit && hit->cap >= bytes) {
    *ptr = hit->ptr;
    return hipSuccess;
  }
  const size_t cap = ((bytes ? bytes : 1) + 65535u) & ~size_t(65535);
  void* p = nullptr;
  if ((e = stream_alloc(&p, cap, stream)) != hipSuccess) return e;
  if (hit) {
    (void)stream_free(hit->ptr, stream);  // after the calls already enqueued on this stream
    hit->ptr = p;
    hit->cap = cap;
  } else {
    t_scratch.push_back(Scratch{device, stream, slot, p, cap});
  }
  *ptr = p;
  return hipSuccess;
}

}  // namespace rudp
