// Stream-ordered temporaries (scan block sums, dedup hash scratch) from a
// library-owned memory pool per device.
//
// hipMallocAsync from the default pool returns freed memory to the driver at
// every synchronize (release threshold 0), so a call made after a sync pays a
// fresh mapping: the Python varlen entry points sync once per call for their
// bounds checks, and the 8 MB dedup scratch of a 1M-datagram batch cost about
// 230 us per call that way (detect_retransmissions 462 -> 236 us with this
// pool, round-2 probe tools/dedup_overhead.py, in git history).  This pool keeps what it has (threshold =
// max) and leaves the process's default pool alone.
#include <algorithm>
#include <mutex>
#include <vector>

#include "internal.hpp"

namespace RUDP_NS {

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

// Per-call temporaries without an allocation per call: one scratch set per
// (device, stream), shared by every host thread, with one buffer per slot
// grown when a call needs more (the old one freed in stream order).  A call
// holds its set's mutex (ScratchCall) from its first scratch request until
// its last kernel is enqueued, so the kernels of calls on one stream never
// interleave on it and the stream's order protects the buffers: a call's
// kernels run after the previous call's.  Nothing is owned by a host thread,
// so threads that come and go (a thread per request, a worker pool that
// recycles its workers: proxy.py:127, :154) leave nothing behind.  (A
// destroyed stream's handle is released only after its pending work, so a new
// stream with the same handle finds the set idle.)  At most kMaxSets sets per
// device.  Once a device has that many, every call records an event behind
// its work as it ends, and a call on a new stream takes the least recently
// used set that has such an event, making its own stream wait for that event
// (hipStreamWaitEvent: stream order, no host wait, no query and no
// device-wide synchronize -- none of which the runtime allows while another
// thread holds a global-mode graph capture -- and no lock held across a
// wait); when no set has one (a set idle since before the device filled) the
// call gets uncached temporaries (allocated and freed in stream order, as
// under capture), so a caller that makes a stream per call keeps a bounded
// footprint and never reuses a buffer still in use.  A buffer grown past
// kKeepBytes is given back when its call ends.  While the stream is being captured into
// a graph the call's temporaries are allocated and freed inside the capture
// (stream_alloc / stream_free), never cached.  hipFreeAsync cost 3.9 us of
// host time per call (rocprofv3 --hip-trace, 1M one-character datagrams), as
// long as a kernel launch, which is why a call does not allocate.
namespace {
constexpr int kSlots = 4;
constexpr size_t kMaxSets = 64;
constexpr size_t kKeepBytes = size_t(64) << 20;

struct DeviceSets;

struct ScratchSet {
  std::mutex mu;  // held by the ScratchCall that enqueues work on these buffers
  DeviceSets* owner = nullptr;
  hipStream_t stream = nullptr;
  uint64_t last_use = 0;
  void* ptr[kSlots] = {};
  size_t cap[kSlots] = {};
  hipEvent_t done = nullptr;  // recorded behind the last call's work (once the device is full)
  bool done_valid = false;    // done marks the end of everything enqueued on these buffers
};

struct DeviceSets {
  std::mutex mu;
  std::vector<ScratchSet*> sets;  // never deleted: a set is re-keyed, not freed
  uint64_t clock = 0;
  std::atomic<bool> full{false};  // kMaxSets reached: calls record their end events
};

std::mutex g_sets_mu;
std::vector<DeviceSets*> g_sets;

DeviceSets* device_sets(int device) {
  std::lock_guard<std::mutex> lk(g_sets_mu);
  if ((int)g_sets.size() <= device) g_sets.resize(device + 1, nullptr);
  if (!g_sets[device]) g_sets[device] = new DeviceSets();  // lives for the process
  return g_sets[device];
}

thread_local ScratchCall* t_call = nullptr;  // the call this thread is making, if any
}  // namespace

// The set of (device, stream), locked for the caller: found, made (up to
// kMaxSets), or the least recently used set that is provably idle, re-keyed;
// nullptr when there is none (the call then uses uncached temporaries).
static ScratchSet* lock_set(int device, hipStream_t stream) {
  DeviceSets* ds = device_sets(device);
  for (;;) {
    ScratchSet* set = nullptr;
    {
      std::lock_guard<std::mutex> lk(ds->mu);
      for (ScratchSet* s : ds->sets)
        if (s->stream == stream) set = s;
      if (!set && ds->sets.size() < kMaxSets) {
        set = new ScratchSet();
        set->owner = ds;
        set->stream = stream;
        ds->sets.push_back(set);
        if (ds->sets.size() == kMaxSets) ds->full.store(true);
      }
      if (!set) {
        // past kMaxSets streams: sets in least recently used order, the first
        // with no call enqueueing (try_lock) whose last call's work is done
        std::vector<ScratchSet*> order(ds->sets);
        std::sort(order.begin(), order.end(),
                  [](const ScratchSet* a, const ScratchSet* b) { return a->last_use < b->last_use; });
        for (ScratchSet* s : order) {
          // (done_valid is read only under the set's own lock, which its
          // writer, ~ScratchCall, holds)
          if (!s->mu.try_lock()) continue;
          // the new stream waits, in stream order, for everything enqueued on
          // these buffers (no host wait, no query: neither is allowed while
          // another thread holds a global-mode graph capture)
          if (s->done_valid && hipStreamWaitEvent(stream, s->done, 0) == hipSuccess) {
            s->stream = stream;
            s->done_valid = false;
            s->last_use = ++ds->clock;
            return s;  // locked
          }
          s->mu.unlock();
        }
        return nullptr;  // none with a known end: uncached temporaries for this call
      }
      set->last_use = ++ds->clock;
    }
    set->mu.lock();
    if (set->stream == stream) return set;
    set->mu.unlock();  // re-keyed by an eviction between the lookup and the lock: look again
  }
}

ScratchCall::ScratchCall(hipStream_t stream) : stream_(stream) {
  if (t_call) return;  // nested in a call already holding its set (same thread)
  if (hipGetDevice(&device_) != hipSuccess) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  capture_ = stream && hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
  t_call = this;
  outer_ = true;
  if (!capture_) set_ = lock_set(device_, stream);
}

ScratchCall::~ScratchCall() {
  if (!outer_) return;
  t_call = nullptr;
  for (int i = 0; i < nfree_; ++i) (void)stream_free(free_[i], stream_);  // capture: inside the graph
  if (!set_) return;
  ScratchSet* set = static_cast<ScratchSet*>(set_);
  for (int k = 0; k < kSlots; ++k) {
    if (set->cap[k] > kKeepBytes) {  // a one-off giant call does not pin its scratch
      (void)stream_free(set->ptr[k], stream_);
      set->ptr[k] = nullptr;
      set->cap[k] = 0;
    }
  }
  // once sets may be taken by other streams, mark where this call's work ends
  set->done_valid = false;
  if (set->owner->full.load(std::memory_order_relaxed)) {
    if (!set->done && hipEventCreateWithFlags(&set->done, hipEventDisableTiming) != hipSuccess) set->done = nullptr;
    set->done_valid = set->done && hipEventRecord(set->done, stream_) == hipSuccess;
  }
  set->mu.unlock();
}

hipError_t stream_scratch(void** ptr, size_t bytes, hipStream_t stream, int slot) {
  ScratchCall* call = t_call;
  if (!call || call->stream_ != stream || slot < 0 || slot >= kSlots) return hipErrorInvalidValue;
  const size_t cap = ((bytes ? bytes : 1) + 65535u) & ~size_t(65535);
  if (call->capture_ || !call->set_) {
    if (call->nfree_ >= ScratchCall::kMaxFree) return hipErrorInvalidValue;
    hipError_t e = stream_alloc(ptr, cap, stream);
    if (e == hipSuccess) call->free_[call->nfree_++] = *ptr;
    return e;
  }
  ScratchSet* set = static_cast<ScratchSet*>(call->set_);
  if (set->cap[slot] >= bytes && set->ptr[slot]) {
    *ptr = set->ptr[slot];
    return hipSuccess;
  }
  void* p = nullptr;
  hipError_t e = stream_alloc(&p, cap, stream);
  if (e != hipSuccess) return e;
  if (set->ptr[slot]) (void)stream_free(set->ptr[slot], stream);  // after the calls already enqueued
  set->ptr[slot] = p;
  set->cap[slot] = cap;
  *ptr = p;
  return hipSuccess;
}

size_t scratch_sets(int device) {
  DeviceSets* ds = device_sets(device);
  std::lock_guard<std::mutex> lk(ds->mu);
  return ds->sets.size();
}

hipError_t pool_used_bytes(int device, uint64_t* used) {
  *used = 0;
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if ((int)g_pools.size() > device) pool = g_pools[device];
  }
  if (!pool) return hipSuccess;
  return hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, used);
}

}  // namespace rudp
