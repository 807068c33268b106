// C ABI of librudp (include/rudp.h): argument checking, path selection,
// kernel launch, and the host-staged pipeline of the *_host variants.
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <deque>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "../../include/rudp.h"
#include "internal.hpp"

namespace RUDP_NS {
int decode_varlen(const uint8_t* d_frames, const uint64_t* d_frame_off, uint32_t len_hint, uint64_t n,
                  const uint16_t* d_csum_in, uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags,
                  uint8_t* d_ok, uint16_t* d_csum_out, uint8_t* d_payload_out, int layout,
                  int device, void* hip_stream, bool checked = false, uint32_t* status_out = nullptr,
                  uint64_t frames_lim = 0, uint8_t* d_valid = nullptr, bool fixed_stride = false);
namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(RUDP_EHIP_BASE - (int)e, "%s: %s (hipError %d)", what, hipGetErrorString(e), (int)e);
}

#define RUDP_HIP(call)                              \
  do {                                              \
    hipError_t e_ = (call);                         \
    if (e_ != hipSuccess) return hip_fail(e_, #call); \
  } while (0)

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Host memory the device can store to at the same address (pinned by
// hipHostMalloc / hipHostRegister, e.g. torch's pinned allocator): the *_host
// decode's kernels then write their per-frame outputs straight into the
// caller's arrays over PCIe, with no device copy and no D2H copy per chunk.
// Null is "nothing to write" and counts as visible; pageable memory is not.
bool device_writable_host(const void* p) {
  if (!p) return true;
  hipPointerAttribute_t attr{};
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // (pageable memory: the query's error is not the caller's)
    return false;
  }
  return attr.type == hipMemoryTypeHost && attr.devicePointer == p;
}

uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t stream64(uint64_t key, uint64_t ctr) { return mix64(key + (ctr + 1ull) * 0x9E3779B97F4A7C15ull); }

bool encode_tile_ok(uint32_t L, const void* payload, const void* frames) {
  return L >= 16 && L % 16 == 0 && L <= kTileMaxPayload && aligned16(payload) && aligned16(frames);
}

bool decode_vec_ok(uint32_t F, int layout, const void* frames, const void* payload_out) {
  if (F < (uint32_t)layout + 16) return false;
  const uint32_t L = F - (uint32_t)layout;
  return L % 16 == 0 && aligned16(frames) && (payload_out == nullptr || aligned16(payload_out));
}

int check_device(int device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (device < 0 || device >= count)
    return fail(RUDP_EINVAL, "device %d out of range (%d HIP devices)", device, count);
  e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  return 0;
}

// Makes `device` the calling thread's HIP device for one entry point and
// gives the caller its own device back on return: a caller such as torch
// keeps its current device, whatever device a batch names.
class DeviceScope {
 public:
  DeviceScope() = default;
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
  ~DeviceScope() {
    if (prev_ >= 0 && prev_ != cur_) (void)hipSetDevice(prev_);
  }
  int set(int device) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    const int rc = check_device(device);
    if (rc == 0) cur_ = device;
    return rc;
  }

 private:
  int prev_ = -1, cur_ = -1;
};

EncodeTileArgs make_encode_args(const rudp_batch* in, uint8_t* frames, uint16_t* csum, int layout) {
  EncodeTileArgs a{};
  a.payload = in->payload;
  a.seq = in->seq;
  a.ack = in->ack;
  a.flags = in->flags;
  a.frames = frames;
  a.csum = csum;
  a.n = in->n;
  a.L = in->payload_len;
  const uint32_t F = a.L + (uint32_t)layout;
  if (encode_tile_ok(a.L, in->payload, frames)) {
    encode_tile_geometry(a.L, &a.T, &a.glog);
    a.hdr_bytes = ((a.T + 1u) * 8u + 15u) & ~15u;
    // Header-table loads: before phase 1 for tiles of at most 16 KiB; above
    // (automatic) or with early = 2, the tile's 80 table bytes go by LDS-DMA
    // with the payload (T = 16, 16-B aligned arrays): 1M x 1472 B 0.5126 ->
    // 0.5086 and 0.5102 -> 0.5069 ms on two boxes, where the leaders' loads
    // after phase 1 were a dependent round trip inside the sum phase
    // (profiles/r02/headline/tile_phases.json, table_dma*.json).
    const int early = tuning().encode_early_table;
    a.early_table = (early == 1 || (early < 0 && a.T * a.L <= 16384u)) ? 1u : 0u;
    if ((early == 2 || (early < 0 && a.T * a.L > 16384u)) && a.T == 16u && aligned16(in->seq) &&
        aligned16(in->ack) && aligned16(in->flags)) {
      a.early_table = 2;  // the tile's 80 table bytes ride the payload's LDS-DMA stream
      a.tab_off = a.hdr_bytes;
      a.hdr_bytes += 80u;
    }
    if (tuning().encode_hchunk && a.T % 16u == 0) {
      a.hchunk = 1;
      a.hc_off = a.hdr_bytes;
      a.hdr_bytes += (a.T + 1u) * 32u;
      const int scr = tuning().encode_hc_scratch;
      if (scr == 1 || (scr < 0 && a.T * a.L <= 16384u)) {
        a.hc_scratch = 1;
        a.scr_off = a.hdr_bytes;
        a.hdr_bytes += a.T * 48u;
      }
    }
    a.invF = ((1ull << 32) + F - 1ull) / F;
    a.num_tiles = (uint32_t)((a.n + a.T - 1) / a.T);
    // XCD-contiguous tiles from 512-B payloads: 1M x 1472 B 0.519 -> 0.513 ms,
    // x 512 B 0.177 -> 0.173, 16M x 1472 B 8.64 -> 7.70 ms; x 256 B equal, x 64 B
    // 0.0259 -> 0.0279 (profiles/r02/sweeps/encode_xcd.json, launch_split.json)
    const int xs = tuning().encode_xcd_swizzle;
    a.xcd_swizzle = (xs == 1 || (xs < 0 && a.L >= 512u)) ? 1u : 0u;
#if RUDP_TOOLS
    a.trace = tuning().encode_trace.load();
#endif
    const int al = tuning().out_align64;
    // Fixed-length encode deals wave stores from the first 64-B boundary at
    // every tile size (since LDS-DMA phase 1 and the header-chunk phase 2 it
    // measured equal or 0.4-1.3% faster from 64 to 1472 B;
    // profiles/r01/sweeps/align64_after_dma.json).
    a.out_align64 = al != 0 ? 1u : 0u;
  }
  return a;
}

int validate_batch(const rudp_batch* in, const void* frames, int layout) {
  if (!in) return fail(RUDP_EINVAL, "rudp_encode: batch is NULL");
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (in->len || in->payload_off)
    return fail(RUDP_ENOTSUP, "variable-length batch: use rudp_encode_varlen");
  if (in->payload_len > kMaxPayload)
    return fail(RUDP_EINVAL, "payload_len %u exceeds %u", in->payload_len, kMaxPayload);
  if (in->n == 0) return 0;
  if (!in->seq || !in->ack || !in->flags || !frames || (in->payload_len && !in->payload))
    return fail(RUDP_EINVAL, "rudp_encode: NULL buffer for a non-empty batch");
  return 0;
}

int validate_decode(const void* frames, const void* frame_off, uint32_t frame_len, uint64_t n,
                    const void* seq, const void* ack, const void* flags, const void* ok,
                    int layout) {
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (frame_off)
    return fail(RUDP_ENOTSUP, "per-frame offsets are not supported by the host-staged decode");
  if (frame_len > kMaxPayload + (uint32_t)layout)
    return fail(RUDP_EINVAL, "frame_len %u exceeds %u", frame_len, kMaxPayload + (uint32_t)layout);
  if (n == 0) return 0;
  if ((frame_len && !frames) || !seq || !ack || !flags || !ok)
    return fail(RUDP_EINVAL, "rudp_decode: NULL buffer for a non-empty batch");
  return 0;
}

// ---- host-staged pipeline for the *_host variants ---------------------------
// Chunks of the batch cycle through S device slots.  Three streams, one per
// engine: H2D copies, kernels, D2H copies; events chain chunk k's three steps
// and hold a slot until its D2H has drained.  So the H2D of chunk k+1, the
// kernel of chunk k and the D2H of chunk k-1 run at the same time.
constexpr int kMaxSlots = 8;

struct Pipeline {
  std::mutex mu;
  bool init = false;
  hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
  hipEvent_t in_ready[kMaxSlots], out_ready[kMaxSlots], slot_free[kMaxSlots];
  void* dbuf[kMaxSlots] = {};
  uint32_t* d_status = nullptr;  // a call's device status, ORed over its chunks
  uint32_t* h_status = nullptr;  // (pinned) its copy after the call
  size_t bytes = 0;
  int slots = 0;
};

std::mutex g_pipe_mu;
std::vector<Pipeline*> g_pipe;

Pipeline* pipeline_for(int device) {
  std::lock_guard<std::mutex> lk(g_pipe_mu);
  if ((int)g_pipe.size() <= device) g_pipe.resize(device + 1, nullptr);
  if (!g_pipe[device]) g_pipe[device] = new Pipeline();  // lives for the process
  return g_pipe[device];
}

int pipeline_init(Pipeline* pp) {
  if (!pp->init) {
    RUDP_HIP(hipStreamCreateWithFlags(&pp->h2d, hipStreamNonBlocking));
    RUDP_HIP(hipStreamCreateWithFlags(&pp->comp, hipStreamNonBlocking));
    RUDP_HIP(hipStreamCreateWithFlags(&pp->d2h, hipStreamNonBlocking));
    for (int i = 0; i < kMaxSlots; ++i) {
      RUDP_HIP(hipEventCreateWithFlags(&pp->in_ready[i], hipEventDisableTiming));
      RUDP_HIP(hipEventCreateWithFlags(&pp->out_ready[i], hipEventDisableTiming));
      RUDP_HIP(hipEventCreateWithFlags(&pp->slot_free[i], hipEventDisableTiming));
    }
    RUDP_HIP(hipMalloc(reinterpret_cast<void**>(&pp->d_status), 256));
    RUDP_HIP(hipHostMalloc(reinterpret_cast<void**>(&pp->h_status), 256, hipHostMallocDefault));
    pp->init = true;
  }
  return 0;
}

int pipeline_reserve(Pipeline* pp, int slots, size_t bytes) {
  if (int rc = pipeline_init(pp)) return rc;
  if (pp->bytes >= bytes && pp->slots >= slots) return 0;
  for (int i = 0; i < kMaxSlots; ++i) {
    if (pp->dbuf[i]) RUDP_HIP(hipFree(pp->dbuf[i]));
    pp->dbuf[i] = nullptr;
  }
  pp->bytes = 0;
  pp->slots = 0;
  for (int i = 0; i < slots; ++i) {
    hipError_t e = hipMalloc(&pp->dbuf[i], bytes);
    if (e != hipSuccess) return fail(RUDP_ENOMEM, "staging hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  }
  pp->bytes = bytes;
  pp->slots = slots;
  return 0;
}

size_t up256(size_t x) { return (x + 255u) & ~size_t(255); }

size_t stage_bytes() {
  const int mb = tuning().host_stage_mb;
  return (size_t)(mb > 0 ? mb : 32) << 20;
}

// Packets per chunk for a given per-packet staging footprint: a slot's worth,
// and for a batch over 4 MiB at most 1/host_min_chunks of it, so that even a
// batch of small frames has copies in both directions overlapping a kernel.
uint64_t chunk_packets(uint64_t n, uint64_t bytes_per_packet) {
  const uint64_t bpp = bytes_per_packet ? bytes_per_packet : 1;
  uint64_t cn = stage_bytes() / bpp;
  const int kc = tuning().host_min_chunks;
  const uint64_t k = (uint64_t)(kc > 1 ? kc : 1);
  if (n * bpp > (4u << 20) && k > 1) {
    const uint64_t part = (n + k - 1) / k;
    if (part < cn) cn = part;
  }
  if (cn < 64) cn = 64;
  return cn > n ? n : cn;
}

int pipeline_slots() {
  const int s = tuning().host_slots;
  return s < 2 ? 2 : s > kMaxSlots ? kMaxSlots : s;
}

// The host passes over a batch's offsets / lengths that plan its chunks run on
// the caller's thread, ahead of the chunk's copies (for one-character frames a
// scalar pass took as long as the chunk's copies): built for AVX-512 and AVX2
// as well, picked at load time by the CPU.
void offsets_range(const uint64_t* o, uint64_t cnt, uint64_t lim, uint64_t* plo, uint64_t* phi);
void lengths_sum_max(const uint32_t* l, uint64_t m, uint64_t* psum, uint32_t* pmax);
#if !defined(__HIP_DEVICE_COMPILE__)
// least and greatest of o[0, cnt) at or below lim (lo = ~0, hi = 0 when none is)
__attribute__((target_clones("avx512f", "avx2", "default"))) void offsets_range(const uint64_t* o, uint64_t cnt,
                                                                              uint64_t lim, uint64_t* plo,
                                                                              uint64_t* phi) {
  uint64_t lo = ~0ull, hi = 0;
  for (uint64_t i = 0; i < cnt; ++i) {
    const uint64_t x = o[i];
    const bool in = x <= lim;
    const uint64_t a = in ? x : ~0ull, b = in ? x : 0;
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  *plo = lo;
  *phi = hi;
}

__attribute__((target_clones("avx512f", "avx2", "default"))) void lengths_sum_max(const uint32_t* l, uint64_t m,
                                                                                uint64_t* psum, uint32_t* pmax) {
  uint64_t sum = 0;
  uint32_t mx = 0;
  for (uint64_t i = 0; i < m; ++i) {
    sum += l[i];
    mx = l[i] > mx ? l[i] : mx;
  }
  *psum = sum;
  *pmax = mx;
}
#endif

// Drive chunks through the pipeline: `plan(p0)` returns the packets of the
// chunk that starts at packet p0 (> 0, or a negative error code), and the
// three callbacks enqueue that chunk's work on the stream they are given (all
// four run on this thread, one chunk at a time, so a plan's extra state lives
// until the chunk's callbacks have run).  Returns only after all three streams
// have drained, on success and on every error path: earlier chunks' copies
// into the caller's host arrays must not outlive the call (the caller may
// free those arrays as soon as it returns).
template <class PLAN, class H2D, class KERN, class D2H>
int run_pipeline_planned(Pipeline* pp, uint64_t n, PLAN plan, H2D h2d, KERN kern, D2H d2h) {
  const int S = pp->slots;
  auto enqueue = [&]() -> int {
    for (uint64_t p0 = 0, k = 0; p0 < n; ++k) {
      const int64_t mm = plan(p0);
      if (mm <= 0) return mm < 0 ? (int)mm : fail(RUDP_EINVAL, "pipeline: empty chunk");
      const uint64_t m = (uint64_t)mm;
      const int s = (int)(k % (uint64_t)S);
      char* base = (char*)pp->dbuf[s];
      if (k >= (uint64_t)S) RUDP_HIP(hipStreamWaitEvent(pp->h2d, pp->slot_free[s], 0));
      int rc = h2d(base, p0, m, pp->h2d);
      if (rc) return rc;
      RUDP_HIP(hipEventRecord(pp->in_ready[s], pp->h2d));
      RUDP_HIP(hipStreamWaitEvent(pp->comp, pp->in_ready[s], 0));
      if ((rc = kern(base, p0, m, pp->comp))) return rc;
      RUDP_HIP(hipEventRecord(pp->out_ready[s], pp->comp));
      RUDP_HIP(hipStreamWaitEvent(pp->d2h, pp->out_ready[s], 0));
      if ((rc = d2h(base, p0, m, pp->d2h))) return rc;
      RUDP_HIP(hipEventRecord(pp->slot_free[s], pp->d2h));
      p0 += m;
    }
    return 0;
  };
  const int rc = enqueue();
  const hipError_t e1 = hipStreamSynchronize(pp->h2d);
  const hipError_t e2 = hipStreamSynchronize(pp->comp);
  const hipError_t e3 = hipStreamSynchronize(pp->d2h);
  if (rc) return rc;
  if (e1 != hipSuccess) return hip_fail(e1, "pipeline H2D stream");
  if (e2 != hipSuccess) return hip_fail(e2, "pipeline kernel stream");
  if (e3 != hipSuccess) return hip_fail(e3, "pipeline D2H stream");
  return 0;
}

// Chunks of a fixed cn packets.
template <class H2D, class KERN, class D2H>
int run_pipeline(Pipeline* pp, uint64_t n, uint64_t cn, H2D h2d, KERN kern, D2H d2h) {
  return run_pipeline_planned(
      pp, n, [&](uint64_t p0) -> int64_t { return (int64_t)(n - p0 < cn ? n - p0 : cn); }, h2d, kern, d2h);
}

}  // namespace

void encode_tile_geometry(uint32_t L, uint32_t* T, uint32_t* glog) {
  // T = packets per tile: a power of two in [16, 256] with a tile payload of
  // about 8 KiB or more (T = 16 from L = 512 up; 128 at L = 64).  G = 256/T
  // lanes share a packet, so a group's 16-byte loads form contiguous runs.
  uint32_t t = 8192u / L;
  if (t > 256u) t = 256u;
  uint32_t tile = 16u;
  while (tile * 2u <= t) tile *= 2u;
  uint32_t lg = 0;
  while ((256u >> lg) > tile) ++lg;
  int forced = tuning().encode_tile;  // experiments only (rudpx_tune)
  while (forced > 4 && (uint32_t)forced * L > 65536u) forced >>= 1;  // LDS tile <= 64 KiB
  if (forced >= 4 && forced <= 256 && (forced & (forced - 1)) == 0) {
    uint32_t g = 256u / (uint32_t)forced, l2 = 0;
    while ((1u << l2) < g) ++l2;
    lg = l2;
  }
  *glog = lg;
  *T = 256u >> lg;
}

uint32_t decode_group_log2(uint32_t L) {
  // G = largest power of two <= min(16, V/2), at least 1: two or more 16-byte
  // chunks per lane keep enough loads in flight (measured: 1M x 64 B frames
  // 0.023 ms at G = 2 vs 0.031 ms at G = 4; 1M x 1472 B best at G = 16).
  const uint32_t V = L / 16u;
  uint32_t lg = 0;
  while (lg < 4 && (4u << lg) <= V) ++lg;
  return lg;
}

int decode_varlen(const uint8_t* d_frames, const uint64_t* d_frame_off, uint32_t len_hint, uint64_t n,
                  const uint16_t* d_csum_in, uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags,
                  uint8_t* d_ok, uint16_t* d_csum_out, uint8_t* d_payload_out, int layout,
                  int device, void* hip_stream, bool checked, uint32_t* status_out, uint64_t frames_lim,
                  uint8_t* d_valid, bool fixed_stride) {
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (d_payload_out)
    return fail(RUDP_ENOTSUP, "variable-length decode is zero-copy: payload i is "
                "frames[frame_off[i] + layout, frame_off[i + 1])");
  if (n == 0) return 0;
  if (!d_seq || !d_ack || !d_flags || !d_ok)
    return fail(RUDP_EINVAL, "rudp_decode: NULL buffer for a non-empty batch");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  VarlenArgs a{};
  a.frames = const_cast<unsigned char*>(d_frames);
  a.frame_off = d_frame_off;
  a.csum_in = d_csum_in;
  a.seq = d_seq;
  a.ack = d_ack;
  a.flags = d_flags;
  a.ok = d_ok;
  a.csum_out = d_csum_out;
  a.valid = d_valid;
  a.n = n;
  if (fixed_stride) {
    // Fixed-length frames of len_hint bytes that miss the fixed-length decode
    // tile: no offsets in memory (VarlenArgs::stride), the frames pointer
    // moved back to a 16-B boundary, every frame inside [0, n F).
    const uint64_t fmis = reinterpret_cast<uintptr_t>(d_frames) & 15u;
    a.frames = const_cast<unsigned char*>(d_frames) - fmis;
    a.frame_off = nullptr;
    a.fo_base = fmis;
    a.stride = len_hint;
    checked = true;
    frames_lim = fmis + n * (uint64_t)len_hint;
    status_out = nullptr;
  }
  // Lanes per frame from the caller's typical frame length (0 = unknown:
  // tiny frames).  Two or more 16-byte chunks per lane, G in [2, 16].
  const uint32_t chunks = len_hint / 16u + 1u;
  uint32_t lg = 1;
  while (lg < 4 && (4u << lg) <= chunks) ++lg;
  if (tuning().varlen_glog >= 1 && tuning().varlen_glog <= 6) lg = (uint32_t)tuning().varlen_glog;
  a.glog = tuning().varlen_vec ? lg : kNoVec;
  // LDS tile of T = 256 / G frames: room for 1.1x the hinted run (a tile
  // past it takes the per-frame path inside the launch).  1M x 1031 B 0.2299
  // -> 0.2190 ms, x 1479 B 0.2906 -> 0.2846 (varlen_decode_tile.json).  Hints
  // of 128 B and up since the tiles are sized by bytes and load their offsets
  // early: 1M x 263 B 0.080 -> 0.056 ms, 71 B equal, 8 B 0.0164 vs 0.0175
  // slower (profiles/r01/sweeps/varlen_decode_small.json).
  if (tuning().varlen_decode_tile && (len_hint >= 128u || tuning().varlen_decode_tile == 2)) {
    const uint64_t hint = len_hint ? len_hint : 16u;
    // Tile of T = 256 / G frames sized by bytes, not by chunks per lane: the
    // most frames (fewest lanes each, G >= 2) whose run stays within 34 KiB.
    // Four such tiles per CU keep ~130 KiB in flight; the chunks-per-lane
    // rule gave 16-frame tiles (8 KiB at 519 B) and the kernel's 76 VGPRs cap
    // a CU at 6 of them: 1M x 519 B 0.158 -> 0.103 ms, x 1031 B 0.213 ->
    // 0.207, x 1479 B unchanged (profiles/r01/sweeps/varlen_decode_lanes.json).
    if (tuning().varlen_glog < 1 && tuning().varlen_vec) {
      uint32_t tlg = 1;
      while (tlg < 4 && (256u >> tlg) * hint > 34816u) ++tlg;
      lg = tlg;
      a.glog = lg;
    }
    const uint64_t pct = (uint64_t)tuning().varlen_decode_cap_pct;
    a.dec_nt = tuning().varlen_decode_nt == 128 ? 128u : 256u;
    a.dec_r4 = tuning().varlen_decode_r4 ? 1u : 0u;
    const uint64_t cap = (((a.dec_nt >> lg) * hint * pct / 100u + 256u) + 15u) & ~15ull;
    a.tile_cap = cap <= 49152u ? (uint32_t)cap : 0u;
  }
  a.early_fo = tuning().varlen_early_fo ? 1u : 0u;
  a.xcd = tuning().tile_xcd ? 1u : 0u;
  // decode tile sums from 128-B block sums (the encode tile's scheme)
  {
    const int vb = tuning().varlen_decode_blocks;
    a.tile_sums = vb == 2 ? 2u : vb == 1 ? 1u : 0u;
  }
  // Small frames (payload hint under varlen_small bytes): tiles of 256 * fpt
  // frames with the per-frame outputs lane-strided (decode_varlen_small_kernel).
  {
    const int small_hint = tuning().varlen_small;
    if (small_hint > 0 && len_hint < (uint32_t)small_hint + (uint32_t)layout && tuning().varlen_vec) {
      // 4 frames per thread (1M frames of 1 / 4 / 9 / 15 B payload: 10.6 / 12.1 /
      // 11.9 / 13.6 us at 4 vs 11.1 / 12.4 / 12.4 / 13.3 at 2; small.json)
      const int fpt = tuning().varlen_small_fpt;
      a.small_fpt = (fpt == 1 || fpt == 2 || fpt == 8) ? (uint32_t)fpt : 4u;
      const uint64_t T = (uint64_t)256u * a.small_fpt;
      const uint64_t hint = len_hint ? len_hint : (uint64_t)layout + 1u;
      a.small_cap = (uint32_t)((T * hint * 5u / 4u + 256u + 15u) & ~15ull);
    }
  }
  a.status_out = status_out;
  a.frames_lim = frames_lim;
  a.lim_checked = checked ? 1u : 0u;
#if RUDP_TOOLS
  a.diag = (uint32_t)tuning().varlen_diag;
#endif
#if RUDP_TOOLS
  // Checked calls with MTU-scale hints: byte spans (decode_varlen_span_kernel)
  // instead of frame tiles; the span index lives in this stream's scratch
  // (measured slower than the frame tiles, DESIGN §7: diagnostics build only).
  const uint64_t S = (uint64_t)tuning().varlen_decode_span_bytes & ~15ull;
  const uint64_t span_cap = (S + 2u * (uint64_t)len_hint + 64u + 15u) & ~15ull;
  const uint64_t nt = S ? frames_lim / S + 1u : 0u;
  const bool span = checked && d_frame_off && tuning().varlen_decode_span && a.glog != kNoVec && !a.small_fpt &&
                    len_hint >= 256u && S >= 4096u && n < 0xFFFFFFFFull && nt < 0x7FFFFFFFull &&
                    decode_span_fits(span_cap) && (reinterpret_cast<uintptr_t>(d_frames) & 15u) == 0;
  std::optional<ScratchCall> call;
  if (span) {
    call.emplace((hipStream_t)hip_stream);
    void* buf = nullptr;
    RUDP_HIP(stream_scratch(&buf, (nt + 2u) * sizeof(SpanRec), (hipStream_t)hip_stream, kScratchRecords));
    static std::atomic<uint32_t> epoch{0};
    a.span_rec = static_cast<const SpanRec*>(buf);
    a.span_count = nt;
    a.span_flag = reinterpret_cast<const uint32_t*>(static_cast<SpanRec*>(buf) + nt + 1u);
    a.span_epoch = epoch.fetch_add(1u) + 1u;
    a.span_S = (uint32_t)S;
    a.tile_cap = (uint32_t)span_cap;
  }
#endif
  rc = launch_decode_varlen(a, layout, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "varlen decode launch");
  return 0;
}

// Fixed-length batches the fixed-length tile does not take (payloads not a
// multiple of 16 B -- the reference's one-character datagrams,
// utils/reliableUDP.py:11, :60 -- payloads over 4 KiB, unaligned views): the
// varlen tile kernels with implicit offsets (VarlenArgs::stride, frame p at
// p F, payload p at p L): no scan and no offsets in memory, one launch.
// Payloads under 16 B take the small-frame tile (frames built in an LDS image
// of the tile's output run), 16 B to 6 KiB the MTU tile, longer ones the
// per-packet vector kernel.
int encode_stride(const rudp_batch* in, uint8_t* d_frames, uint16_t* d_csum, int layout, hipStream_t s) {
  const uint32_t L = in->payload_len, H = (uint32_t)layout;
  const uint64_t fmis = reinterpret_cast<uintptr_t>(d_frames) & 15u;
  const uint64_t pmis = reinterpret_cast<uintptr_t>(in->payload) & 15u;
  VarlenArgs a{};
  a.payload = in->payload ? in->payload - pmis : nullptr;
  a.seq_in = in->seq;
  a.ack_in = in->ack;
  a.flags_in = in->flags;
  a.frames = d_frames - fmis;
  a.frame_off = nullptr;
  a.csum = d_csum;
  a.n = in->n;
  a.fo_base = fmis;
  a.stride = (uint64_t)L + H;
  a.po_delta = pmis - fmis;
  const uint32_t chunks = L / 16u + 1u;
  uint32_t lg = 0;
  while (lg < 4 && (4u << lg) <= chunks) ++lg;
  a.glog = tuning().varlen_vec ? lg : kNoVec;
  if (tuning().varlen_vec && tuning().varlen_tile) varlen_tile_geometry(L, &a.tile_T, &a.tile_glog, &a.tile_cap);
  a.align64 = tuning().out_align64 == 1 ? 1u : 0u;
  {
    const int early = tuning().encode_early_table;
    a.early_table = (early == 1 || (early < 0 && L >= 128u)) ? 1u : 0u;
    const int vhc = tuning().varlen_hchunk;
    a.vhc = (uint32_t)(vhc < 0 ? 0 : vhc > 2 ? 2 : vhc);
  }
  a.early_fo = tuning().varlen_early_fo ? 1u : 0u;
  a.xcd = tuning().tile_xcd ? 1u : 0u;
  a.tile_sums = tuning().varlen_tile_sums == 2 ? 2u : 0u;
  const int small_hint = tuning().varlen_small;
  if (small_hint > 0 && L < (uint32_t)small_hint && tuning().varlen_vec) {
    a.small_fpt = L <= 4u ? 4u : 2u;  // (the varlen small-frame tile's measured choice)
    const uint64_t T = (uint64_t)256u * a.small_fpt;
    const uint64_t hint = L ? L : 1u;
    a.small_cap = (uint32_t)((T * hint * 5u / 4u + 256u + 15u) & ~15ull);
    return launch_encode_stride_small(a, layout, s);
  }
  return launch_encode_varlen(a, layout, s);
}

// Adds a chunk's base to the frame offsets its encode wrote from 0 -- in
// place, or into the caller's pinned host array (`out`, no D2H copy) -- and
// ORs the chunk's device status into the call's (the chunks' kernels run in
// stream order on one stream, so a plain read-modify-write by one thread).
__global__ void __launch_bounds__(256) add_base_kernel(uint64_t* off, uint64_t* out, uint64_t n1, uint64_t base,
                                                      const uint32_t* st, uint32_t* acc) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n1 && (base || out != off)) out[i] = off[i] + base;
  if (i == 0) {
    const uint32_t v = *st;
    if (v) *acc |= v;
  }
}

}  // namespace rudp

using namespace RUDP_NS;

extern "C" {

int rudp_abi_version(void) { return RUDP_ABI_VERSION; }

const char* rudp_last_error(void) { return g_last_error.c_str(); }

int rudp_device_count(int* count) {
  if (!count) return fail(RUDP_EINVAL, "rudp_device_count: NULL");
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  return 0;
}

int rudp_encode(const rudp_batch* in, uint8_t* d_frames, uint16_t* d_csum_or_null, int layout,
                int device, void* hip_stream) {
  int rc = validate_batch(in, d_frames, layout);
  if (rc || in->n == 0) return rc;
  DeviceScope dev_scope;
  if ((rc = dev_scope.set(device))) return rc;
  if (!encode_tile_ok(in->payload_len, in->payload, d_frames)) {
    rc = encode_stride(in, d_frames, d_csum_or_null, layout, (hipStream_t)hip_stream);
    if (rc) return hip_fail((hipError_t)rc, "fixed-stride encode launch");
    return 0;
  }
  // Batches over `encode_launch_packets` go out as several launches on the
  // stream, each over a contiguous slice (a multiple of every tile size).
  const int lp = tuning().encode_launch_packets;
  const uint64_t chunk = lp > 0 ? ((uint64_t)lp + 255u) & ~255ull : in->n;
  const uint64_t F = (uint64_t)in->payload_len + (uint64_t)layout;
  for (uint64_t p0 = 0; p0 < in->n; p0 += chunk) {
    rudp_batch sub = *in;
    sub.n = in->n - p0 < chunk ? in->n - p0 : chunk;
    sub.seq = in->seq + p0;
    sub.ack = in->ack + p0;
    sub.flags = in->flags + p0;
    sub.payload = in->payload ? in->payload + p0 * in->payload_len : nullptr;
    EncodeTileArgs a = make_encode_args(&sub, d_frames + p0 * F, d_csum_or_null ? d_csum_or_null + p0 : nullptr,
                                        layout);
    rc = launch_encode(a, layout, (hipStream_t)hip_stream);
    if (rc) return hip_fail((hipError_t)rc, "encode launch");
  }
  return 0;
}

int rudp_decode(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null, uint32_t frame_len,
                uint64_t n, const uint16_t* d_csum_in_or_null, uint16_t* d_seq, uint16_t* d_ack,
                uint8_t* d_flags, uint8_t* d_ok, uint16_t* d_csum_out_or_null,
                uint8_t* d_payload_out_or_null, int layout, int device, void* hip_stream) {
  return rudp_decode_utf8(d_frames, d_frame_off_or_null, frame_len, n, d_csum_in_or_null, d_seq, d_ack, d_flags,
                          d_ok, d_csum_out_or_null, d_payload_out_or_null, nullptr, layout, device, hip_stream);
}

int rudp_decode_utf8(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null, uint32_t frame_len,
                     uint64_t n, const uint16_t* d_csum_in_or_null, uint16_t* d_seq, uint16_t* d_ack,
                     uint8_t* d_flags, uint8_t* d_ok, uint16_t* d_csum_out_or_null,
                     uint8_t* d_payload_out_or_null, uint8_t* d_valid_or_null, int layout, int device,
                     void* hip_stream) {
  if (d_frame_off_or_null) {
    return decode_varlen(d_frames, d_frame_off_or_null, frame_len, n, d_csum_in_or_null, d_seq, d_ack, d_flags,
                         d_ok, d_csum_out_or_null, d_payload_out_or_null, layout, device, hip_stream, false,
                         nullptr, 0, d_valid_or_null);
  }
  int rc = validate_decode(d_frames, nullptr, frame_len, n, d_seq, d_ack, d_flags, d_ok, layout);
  if (rc || n == 0) return rc;
  DeviceScope dev_scope;
  if ((rc = dev_scope.set(device))) return rc;
  uint8_t* pay_out = frame_len > (uint32_t)layout ? d_payload_out_or_null : nullptr;
  if (!decode_vec_ok(frame_len, layout, d_frames, pay_out)) {
    // Frames the fixed-length tiles do not take (payloads not a multiple of
    // 16 B -- the reference's 6-9 B datagrams -- short frames, unaligned
    // views): the varlen decode tiles with implicit offsets, strict UTF-8 in
    // the same pass; a payload copy-out is one more launch over the frames.
    rc = decode_varlen(d_frames, nullptr, frame_len, n, d_csum_in_or_null, d_seq, d_ack, d_flags, d_ok,
                       d_csum_out_or_null, nullptr, layout, device, hip_stream, false, nullptr, 0, d_valid_or_null,
                       true);
    if (rc) return rc;
    if (pay_out) {
      rc = launch_copy_payloads(d_frames, frame_len, (uint32_t)layout, n, pay_out, (hipStream_t)hip_stream);
      if (rc) return hip_fail((hipError_t)rc, "payload copy-out launch");
    }
    return 0;
  }
  DecodeArgs a{};
  a.align64 = tuning().out_align64 == 1 ? 1u : 0u;
  a.stage_out = (tuning().decode_stage_out &&
                 ((reinterpret_cast<uintptr_t>(d_seq) | reinterpret_cast<uintptr_t>(d_ack) |
                   reinterpret_cast<uintptr_t>(d_flags) | reinterpret_cast<uintptr_t>(d_ok) |
                   reinterpret_cast<uintptr_t>(d_csum_out_or_null) | reinterpret_cast<uintptr_t>(d_valid_or_null)) &
                  3u) == 0) ? 1u : 0u;
  a.xcd = (tuning().tile_xcd && frame_len >= 128u) ? 1u : 0u;
#if RUDP_TOOLS
  a.trace = tuning().encode_trace.load();  // decode tile timeline (tools/decode_timeline.py)
#endif
  a.frames = d_frames;
  a.csum_in = d_csum_in_or_null;
  a.seq = d_seq;
  a.ack = d_ack;
  a.flags = d_flags;
  a.ok = d_ok;
  a.csum_out = d_csum_out_or_null;
  a.payload_out = pay_out;
  a.n = n;
  a.F = frame_len;
  DecodePath path;
  {
    const uint32_t lg = decode_group_log2(frame_len - (uint32_t)layout);
    path = a.payload_out ? DecodePath::kCopy : DecodePath::kVerify;
    // the verify kernel reads the header from the group's first two lanes
    a.glog = (path == DecodePath::kVerify && lg == 0) ? 1 : lg;
    // stage whole tiles in LDS when a tile fits in 64 KiB
    const bool tile_fits = (size_t)(256u >> lg) * frame_len + 48 <= 65536;
    if (path == DecodePath::kCopy && tile_fits && tuning().decode_copy_tile)
      path = DecodePath::kCopyTile;
    if (path == DecodePath::kVerify && tile_fits && tuning().decode_verify_tile) {
      path = DecodePath::kVerifyTile;
      a.glog = lg;
    }
    const int forced = tuning().decode_glog;  // experiments only (rudpx_tune)
    if (path == DecodePath::kVerify && forced >= 1 && forced <= 4 &&
        (1u << forced) <= (frame_len - (uint32_t)layout) / 16u)
      a.glog = (uint32_t)forced;
    if ((path == DecodePath::kVerifyTile || path == DecodePath::kCopyTile) && forced >= 0 &&
        forced <= (RUDP_TOOLS ? 5 : 4) && (size_t)(256u >> forced) * frame_len + 48 <= 65536)
      a.glog = (uint32_t)forced;
  }
  // The tile kernels check each payload's UTF-8 in the same pass; the other
  // forms (frames past a 64 KiB tile, copy-out by register windows) leave it
  // to the validation kernels, a second read of the frames.
  const bool fused = path == DecodePath::kCopyTile || path == DecodePath::kVerifyTile;
  a.valid = fused ? d_valid_or_null : nullptr;
  rc = launch_decode(a, layout, path, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "decode launch");
  if (d_valid_or_null && !fused) {
    Utf8Args u{};
    u.frames = d_frames;
    u.n = n;
    u.F = frame_len;
    u.H = (uint32_t)layout;
    u.valid = d_valid_or_null;
    u.xcd = tuning().tile_xcd ? 1u : 0u;
    rc = launch_validate_utf8(u, (hipStream_t)hip_stream);
    if (rc) return hip_fail((hipError_t)rc, "utf8 validation launch");
  }
  return 0;
}

int rudp_synth(uint64_t seed, uint64_t first_index, uint64_t n, uint32_t payload_len, int ascii,
               uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_payload, int device,
               void* hip_stream) {
  if (n == 0) return 0;
  if (!d_seq || !d_ack || !d_flags || (payload_len && !d_payload))
    return fail(RUDP_EINVAL, "rudp_synth: NULL buffer");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  SynthArgs a{};
  const uint64_t k0 = stream64(seed, 0), k1 = stream64(seed, 1), k2 = stream64(seed, 2),
                 k3 = stream64(seed, 3);
  a.isn = (uint32_t)(1ull + stream64(k0, 0) % 5000ull);
  a.key_ack = k1;
  a.key_flags = k2;
  a.key_payload = k3;
  a.first = first_index;
  a.n = n;
  a.L = payload_len;
  a.ascii = ascii ? 1u : 0u;
  a.seq = d_seq;
  a.ack = d_ack;
  a.flags = d_flags;
  a.payload = d_payload;
  rc = launch_synth(a, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "synth launch");
  return 0;
}

static int encode_varlen(const rudp_batch* in, uint8_t* d_frames, uint64_t* d_frame_off,
                         uint16_t* d_csum_or_null, int layout, int device, void* hip_stream,
                         const ScanCheck& chk) {
  if (!in) return fail(RUDP_EINVAL, "rudp_encode_varlen: batch is NULL");
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (in->n == 0) return 0;
  if (!in->len || !d_frame_off)
    return fail(RUDP_EINVAL, "rudp_encode_varlen: len[] and frame_off[] are required");
  if (!in->seq || !in->ack || !in->flags || !d_frames || !in->payload)
    return fail(RUDP_EINVAL, "rudp_encode_varlen: NULL buffer for a non-empty batch");
  if (in->n > 0x7FFFFFFFull)
    return fail(RUDP_EINVAL, "rudp_encode_varlen: at most 2^31-1 packets per call");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)hip_stream;
  ScratchCall call(s);  // the scan's sums and the tile records, until the last launch
  VarlenArgs a{};
  a.payload = in->payload;
  a.len = in->len;
  a.payload_off = in->payload_off;
  a.seq_in = in->seq;
  a.ack_in = in->ack;
  a.flags_in = in->flags;
  a.frames = d_frames;
  a.frame_off = d_frame_off;
  a.csum = d_csum_or_null;
  a.n = in->n;
  // Lanes per packet from payload_len, the caller's typical payload length
  // (a hint for varlen batches; 0 = unknown/tiny): two+ chunks per lane.
  const uint32_t chunks = in->payload_len / 16u + 1u;
  uint32_t lg = 0;
  while (lg < 4 && (4u << lg) <= chunks) ++lg;
  if (tuning().varlen_glog >= 0 && tuning().varlen_glog <= 6) lg = (uint32_t)tuning().varlen_glog;
  a.glog = tuning().varlen_vec ? lg : kNoVec;
  if (tuning().varlen_vec && tuning().varlen_tile)
    varlen_tile_geometry(in->payload_len, &a.tile_T, &a.tile_glog, &a.tile_cap);
  a.align64 = tuning().out_align64 == 1 ? 1u : 0u;
  // Header-table loads before phase 1 for hints of 128 B and up: with the
  // fast phase 2 (varlen_hchunk) they measured 1M x 1472 B 0.637 -> 0.603 ms,
  // x 1024 B 0.489 -> 0.468, x 256 B 0.170 -> 0.164
  // (profiles/r01/sweeps/encode_early_table_varlen.json); before it they were
  // 0.5-2% slower everywhere, and small hints keep them after the barrier.
  {
    const int early = tuning().encode_early_table;
    a.early_table = (early == 1 || (early < 0 && in->payload_len >= 128u)) ? 1u : 0u;
  }
  {
    const int vhc = tuning().varlen_hchunk;
    a.vhc = (uint32_t)(vhc < 0 ? 0 : vhc > 2 ? 2 : vhc);
  }
  a.early_fo = tuning().varlen_early_fo ? 1u : 0u;
  a.xcd = tuning().tile_xcd ? 1u : 0u;
  a.status = chk.status;
#if RUDP_TOOLS
  a.diag = (uint32_t)tuning().varlen_diag;
#endif
  // Small frames (hints under varlen_small bytes, packed, aligned): the scan's
  // last pass and the framing in one tile kernel (launch_encode_varlen_small).
  const int small_hint = tuning().varlen_small;
  if (small_hint > 0 && in->payload_len < (uint32_t)small_hint && !in->payload_off && tuning().varlen_vec &&
      aligned16(in->payload) && aligned16(d_frames)) {
    // packets per thread: 4 for hints up to 4 B, 2 above (1M packets of 1 / 4 /
    // 1-4 B: 28.0 / 24.2 / 24.4 us at 4 vs 28.1 / 25.6 / 26.1 at 2; 9 / 15 B:
    // 29.8 / 28.8 at 2 vs 36.4 / 32.8 at 4; profiles/r02/sweeps/small.json)
    const int fpt = tuning().varlen_small_fpt;
    a.small_fpt = (fpt == 1 || fpt == 2 || fpt == 4 || fpt == 8) ? (uint32_t)fpt
                : in->payload_len <= 4u ? 4u : 2u;
    const uint64_t T = (uint64_t)256u * a.small_fpt;
    const uint64_t hint = in->payload_len ? in->payload_len : 1u;
    a.small_cap = (uint32_t)((T * hint * 5u / 4u + 256u + 15u) & ~15ull);
    a.len_code_base = in->payload_len;  // (pass 1's length codes count from the hint)
#if RUDP_TOOLS
    a.trace = tuning().encode_trace.load();
#endif
    rc = launch_encode_varlen_small(a, chk, layout, s);
    if (rc) return hip_fail((hipError_t)rc, "small-frame varlen encode launch");
    return 0;
  }
  // Sum pass of the tile kernel: 2 = from 128-B block sums
  a.tile_sums = tuning().varlen_tile_sums == 2 ? 2u : 0u;
  a.map_bal = tuning().varlen_map_bal ? 1u : 0u;
#if RUDP_TOOLS
  a.trace = tuning().encode_trace.load();  // tile-kernel phase timeline (tools/varlen_timeline.py)
#endif
  // Tiles by payload bytes (checked calls, where the payload size is known on
  // the host; hints from 1 KiB, varlen_btile_ok): spans of S = budget - 2 *
  // hint - 64 bytes, so a byte tile overflows its LDS budget only through a
  // packet over twice the hint; at most bt_slots packets per tile in LDS (more
  // take the per-packet path).  The scan chooses per call: pass 1 counts the
  // packet tiles likely to overflow, pass 2 picks byte tiles when they are
  // 1/32 of the tiles or more, and pass 3 writes one record per workgroup in
  // the chosen form, so every tile's first loads are two adjacent records
  // (varlen_btile 1; 2: byte tiles always, 3: packet tiles through records;
  // 0: packet tiles from frame_off).
  SpanStarts spans{};
  const int btile = tuning().varlen_btile;
  if (btile > 0 && chk.status && !in->payload_off && a.tile_T && aligned16(in->payload) && aligned16(d_frames)) {
    const uint64_t h = in->payload_len ? in->payload_len : 1u;
    const uint64_t ptiles = (in->n + a.tile_T - 1u) / a.tile_T;
    uint64_t S = a.tile_cap > 2u * h + 64u + h ? a.tile_cap - 2u * h - 64u : 0u;
    if (tuning().varlen_span_bytes > 0) S = (uint64_t)tuning().varlen_span_bytes;
    // 1.5x a span's mean packet count + 2 (fewer, down to the mean + 2, where
    // the slots' LDS would cost a tile per CU: each slot is 44 B, and at 1M x
    // 1472 B 32 slots ran 4 tiles per CU instead of 5)
    uint32_t slots = S ? (uint32_t)(3u * S / (2u * h) + 2u) : 4u;
    if (slots < 4u) slots = 4u;
    if (slots > 256u) slots = 256u;
    uint32_t min_slots = S ? (uint32_t)(S / h + 2u) : 4u;
#if RUDP_TOOLS
    if (a.diag & 2u) slots = min_slots = a.tile_T;
#endif
    if (S && (btile == 2 || varlen_btile_ok(a.tile_T, &slots, min_slots, a.tile_cap, a.tile_cap, (uint32_t)layout,
                                           a.vhc, ptiles, chk.payload_bytes / S + 1u))) {
      spans.bytes = S;
      spans.count = chk.payload_bytes / S + 1u;
      spans.ptiles = ptiles;
      spans.grid = ptiles > spans.count ? ptiles : spans.count;
      spans.min_over = btile == 2 ? 0u : btile == 3 ? 0xFFFFFFFFu : (uint32_t)(ptiles / 32u + 1u);
      spans.tile_T = a.tile_T;
      spans.tile_cap = a.tile_cap;
      void* buf = nullptr;
      // records [grid + 1], then pass 2's choice
      RUDP_HIP(stream_scratch(&buf, (spans.grid + 2u) * sizeof(SpanRec), s, kScratchRecords));
      spans.rec = static_cast<SpanRec*>(buf);
      spans.ctl = reinterpret_cast<uint32_t*>(spans.rec + spans.grid + 1u);
      a.span_rec = spans.rec;
      a.span_count = spans.grid;
      a.bt_slots = (uint32_t)slots;
    }
  }
  rc = scan_frame_offsets(in->len, in->n, (uint32_t)layout, d_frame_off, chk, s, spans);
  if (!rc) rc = launch_encode_varlen(a, layout, s);
  if (rc) return hip_fail((hipError_t)rc, "varlen encode");
  return 0;
}

int rudp_encode_varlen(const rudp_batch* in, uint8_t* d_frames, uint64_t* d_frame_off,
                       uint16_t* d_csum_or_null, int layout, int device, void* hip_stream) {
  return encode_varlen(in, d_frames, d_frame_off, d_csum_or_null, layout, device, hip_stream, ScanCheck{});
}

int rudp_encode_varlen_checked(const rudp_batch* in, uint64_t payload_bytes, uint8_t* d_frames,
                               uint64_t frames_cap, uint64_t* d_frame_off, uint16_t* d_csum_or_null,
                               uint32_t* d_status, int layout, int device, void* hip_stream) {
  if (!d_status) return fail(RUDP_EINVAL, "rudp_encode_varlen_checked: d_status is NULL");
  if (in && in->n == 0) {
    // nothing to launch a check from: the status is written here, on the stream
    DeviceScope dev_scope;
    int rc = dev_scope.set(device);
    if (rc) return rc;
    RUDP_HIP(hipMemsetAsync(d_status, 0, sizeof(uint32_t), (hipStream_t)hip_stream));
    if (d_frame_off) RUDP_HIP(hipMemsetAsync(d_frame_off, 0, sizeof(uint64_t), (hipStream_t)hip_stream));
    return 0;
  }
  ScanCheck chk{};
  chk.payload_off = in ? in->payload_off : nullptr;
  chk.payload_bytes = payload_bytes;
  chk.frames_cap = frames_cap;
  chk.status = d_status;
  return encode_varlen(in, d_frames, d_frame_off, d_csum_or_null, layout, device, hip_stream, chk);
}

int rudp_decode_varlen_checked(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                               uint32_t len_hint, uint64_t n, const uint16_t* d_csum_in_or_null,
                               uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_ok,
                               uint16_t* d_csum_out_or_null, uint32_t* d_status, int layout, int device,
                               void* hip_stream) {
  return rudp_decode_varlen_utf8(d_frames, frames_bytes, d_frame_off, len_hint, n, d_csum_in_or_null, d_seq, d_ack,
                                 d_flags, d_ok, d_csum_out_or_null, nullptr, d_status, layout, device, hip_stream);
}

int rudp_decode_varlen_utf8(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                            uint32_t len_hint, uint64_t n, const uint16_t* d_csum_in_or_null,
                            uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_ok,
                            uint16_t* d_csum_out_or_null, uint8_t* d_valid_or_null, uint32_t* d_status,
                            int layout, int device, void* hip_stream) {
  if (!d_frame_off) return fail(RUDP_EINVAL, "rudp_decode_varlen_checked: frame_off is NULL");
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (d_status) {
    // every frame checks its own pair of offsets inside the decode kernels
    // (a valid batch is exactly one whose frames all pass); they or
    // RUDP_ST_OFFSETS into the zeroed status word.  Without a status word the
    // call is the one kernel: d_ok == RUDP_OK_BAD_OFFSETS marks the rejections.
    DeviceScope dev_scope;
    int rc = dev_scope.set(device);
    if (rc) return rc;
    RUDP_HIP(hipMemsetAsync(d_status, 0, sizeof(uint32_t), (hipStream_t)hip_stream));
  }
  if (n == 0) return 0;
  return decode_varlen(d_frames, d_frame_off, len_hint, n, d_csum_in_or_null, d_seq, d_ack, d_flags, d_ok,
                       d_csum_out_or_null, nullptr, layout, device, hip_stream, true, d_status, frames_bytes,
                       d_valid_or_null);
}

int rudp_frame_off_check(const uint64_t* d_frame_off, uint64_t n, uint64_t frames_bytes, uint32_t* d_status,
                         int device, void* hip_stream) {
  if (!d_frame_off || !d_status) return fail(RUDP_EINVAL, "rudp_frame_off_check: NULL pointer");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  ScratchCall call((hipStream_t)hip_stream);  // the check's partials
  rc = check_frame_offsets(d_frame_off, n, frames_bytes, d_status, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "frame offset check");
  return 0;
}

int rudp_varlen_bounds(const uint32_t* d_len, const int64_t* d_payload_off_or_null, uint64_t n,
                       int64_t* h_out, int device, void* hip_stream) {
  if (!h_out) return fail(RUDP_EINVAL, "rudp_varlen_bounds: h_out is NULL");
  for (int i = 0; i < 5; ++i) h_out[i] = 0;
  if (n == 0) return 0;
  if (!d_len) return fail(RUDP_EINVAL, "rudp_varlen_bounds: len is NULL");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  Bounds b{};
  rc = compute_bounds(d_len, d_payload_off_or_null, n, false, &b, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "varlen bounds");
  h_out[0] = (int64_t)b.min_len;
  h_out[1] = (int64_t)b.max_len;
  h_out[2] = (int64_t)b.sum_len;
  h_out[3] = d_payload_off_or_null ? b.min_off : 0;
  h_out[4] = d_payload_off_or_null ? b.max_end : (int64_t)b.sum_len;
  return 0;
}

int rudp_frame_off_bounds(const int64_t* d_frame_off, uint64_t n, int64_t* h_out, int device,
                          void* hip_stream) {
  if (!h_out) return fail(RUDP_EINVAL, "rudp_frame_off_bounds: h_out is NULL");
  if (!d_frame_off) return fail(RUDP_EINVAL, "rudp_frame_off_bounds: frame_off is NULL");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  Bounds b{};
  rc = compute_bounds(nullptr, d_frame_off, n, true, &b, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "frame offset bounds");
  h_out[0] = b.min_off;
  h_out[1] = b.max_end;
  h_out[2] = (int64_t)b.n_decreasing;
  return 0;
}

int rudp_validate_utf8(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null,
                       uint32_t frame_len, uint64_t n, int layout, uint8_t* d_valid, int device,
                       void* hip_stream) {
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (n == 0) return 0;
  if (!d_valid || (!d_frames && (d_frame_off_or_null || frame_len)))
    return fail(RUDP_EINVAL, "rudp_validate_utf8: NULL buffer for a non-empty batch");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  Utf8Args a{};
  a.frames = d_frames;
  a.frame_off = d_frame_off_or_null;
  a.n = n;
  a.F = frame_len;
  a.H = (uint32_t)layout;
  a.valid = d_valid;
  a.xcd = tuning().tile_xcd ? 1u : 0u;
  rc = launch_validate_utf8(a, (hipStream_t)hip_stream);
  if (rc) return hip_fail((hipError_t)rc, "utf8 validation launch");
  return 0;
}

static int dedup_window(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null, uint32_t frame_len,
                        uint64_t n, uint32_t window, uint8_t* d_dup, int device, void* hip_stream,
                        bool checked, uint64_t frames_bytes) {
  if (window > dedup_max_window())
    return fail(RUDP_EINVAL, "window %u exceeds %u", window, dedup_max_window());
  if (n == 0) return 0;
  if (!d_dup || (!d_frames && (d_frame_off_or_null || frame_len)))
    return fail(RUDP_EINVAL, "rudp_dedup_window: NULL buffer for a non-empty batch");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)hip_stream;
  ScratchCall call(s);  // the hash scratch, until the table pass is enqueued
  DedupArgs a{};
  a.frames = d_frames;
  a.frame_off = d_frame_off_or_null;
  a.n = n;
  a.F = frame_len;
  a.window = window;
  a.dup = d_dup;
  // lanes per frame for the hash pass from the (typical) frame length: 1 for the
  // reference's 6-9 B datagrams, 2 to 64 B, 4 to 256 B, 8 above
  a.glog = frame_len <= 16u ? 0u : frame_len <= 64u ? 1u : frame_len <= 256u ? 2u : 3u;
  a.lim_checked = checked ? 1u : 0u;
  a.frames_lim = frames_bytes;
  // packed frames of the reference's sizes: one launch, nothing in HBM but the flags
  if (d_frame_off_or_null && aligned16(d_frames)) a.small_cap = dedup_small_cap(frame_len, window);
  if (!a.small_cap) {
    void* scratch = nullptr;
    RUDP_HIP(stream_scratch(&scratch, n * sizeof(uint64_t), s, kScratchHash));
    a.hash = (uint64_t*)scratch;
  }
  rc = launch_dedup(a, s);
  if (rc) return hip_fail((hipError_t)rc, "dedup launch");
  return 0;
}

int rudp_dedup_window(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null,
                      uint32_t frame_len, uint64_t n, uint32_t window, uint8_t* d_dup, int device,
                      void* hip_stream) {
  return dedup_window(d_frames, d_frame_off_or_null, frame_len, n, window, d_dup, device, hip_stream, false, 0);
}

int rudp_dedup_window_checked(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                              uint32_t len_hint, uint64_t n, uint32_t window, uint8_t* d_dup, int device,
                              void* hip_stream) {
  if (!d_frame_off) return fail(RUDP_EINVAL, "rudp_dedup_window_checked: frame_off is NULL");
  return dedup_window(d_frames, d_frame_off, len_hint, n, window, d_dup, device, hip_stream, true, frames_bytes);
}

int rudp_encode_host(const rudp_batch* h_in, uint8_t* h_frames, uint16_t* h_csum_or_null,
                     int layout, int device) {
  int rc = validate_batch(h_in, h_frames, layout);
  if (rc || h_in->n == 0) return rc;
  DeviceScope dev_scope;
  if ((rc = dev_scope.set(device))) return rc;
  const uint64_t n = h_in->n;
  const uint64_t L = h_in->payload_len;
  const uint64_t F = L + (uint64_t)layout;
  const uint64_t cn = chunk_packets(n, L + F + 7);
  // Slot layout: payload | frames | seq | ack | flags | csum.
  const size_t o_pay = 0, o_fr = up256(cn * L), o_seq = o_fr + up256(cn * F),
               o_ack = o_seq + up256(cn * 2), o_fl = o_ack + up256(cn * 2),
               o_cs = o_fl + up256(cn), slot = o_cs + up256(cn * 2);
  Pipeline* pp = pipeline_for(device);
  std::lock_guard<std::mutex> lk(pp->mu);
  if ((rc = pipeline_reserve(pp, pipeline_slots(), slot))) return rc;
  auto h2d = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    if (L) RUDP_HIP(hipMemcpyAsync(base + o_pay, h_in->payload + p0 * L, m * L, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_seq, h_in->seq + p0, m * 2, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_ack, h_in->ack + p0, m * 2, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_fl, h_in->flags + p0, m, hipMemcpyHostToDevice, s));
    return 0;
  };
  auto kern = [&](char* base, uint64_t, uint64_t m, hipStream_t s) -> int {
    rudp_batch sub = *h_in;
    sub.n = m;
    sub.seq = (const uint16_t*)(base + o_seq);
    sub.ack = (const uint16_t*)(base + o_ack);
    sub.flags = (const uint8_t*)(base + o_fl);
    sub.payload = (const uint8_t*)(base + o_pay);
    return rudp_encode(&sub, (uint8_t*)(base + o_fr), h_csum_or_null ? (uint16_t*)(base + o_cs) : nullptr,
                       layout, device, s);
  };
  auto d2h = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    RUDP_HIP(hipMemcpyAsync(h_frames + p0 * F, base + o_fr, m * F, hipMemcpyDeviceToHost, s));
    if (h_csum_or_null)
      RUDP_HIP(hipMemcpyAsync(h_csum_or_null + p0, base + o_cs, m * 2, hipMemcpyDeviceToHost, s));
    return 0;
  };
  return run_pipeline(pp, n, cn, h2d, kern, d2h);
}

int rudp_decode_host(const uint8_t* h_frames, uint32_t frame_len, uint64_t n,
                     const uint16_t* h_csum_in_or_null, uint16_t* h_seq, uint16_t* h_ack,
                     uint8_t* h_flags, uint8_t* h_ok, uint16_t* h_csum_out_or_null,
                     uint8_t* h_payload_out_or_null, uint8_t* h_valid_or_null, int layout, int device) {
  int rc = validate_decode(h_frames, nullptr, frame_len, n, h_seq, h_ack, h_flags, h_ok, layout);
  if (rc || n == 0) return rc;
  DeviceScope dev_scope;
  if ((rc = dev_scope.set(device))) return rc;
  const uint64_t F = frame_len;
  const uint64_t L = F > (uint64_t)layout ? F - (uint64_t)layout : 0;
  uint8_t* h_pay = L ? h_payload_out_or_null : nullptr;
  uint8_t* h_val = h_valid_or_null;
  const uint64_t cn = chunk_packets(n, F + (h_pay ? L : 0) + 10 + (h_val ? 1 : 0));
  // Slot layout: frames | payload | seq | ack | flags | ok | csum_in | csum_out | valid.
  const size_t o_fr = 0, o_pay = up256(cn * F), o_seq = o_pay + up256(h_pay ? cn * L : 0),
               o_ack = o_seq + up256(cn * 2), o_fl = o_ack + up256(cn * 2),
               o_ok = o_fl + up256(cn), o_ci = o_ok + up256(cn), o_co = o_ci + up256(cn * 2),
               o_va = o_co + up256(cn * 2), slot = o_va + up256(h_val ? cn : 0);
  Pipeline* pp = pipeline_for(device);
  std::lock_guard<std::mutex> lk(pp->mu);
  if ((rc = pipeline_reserve(pp, pipeline_slots(), slot))) return rc;
  auto h2d = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    if (F) RUDP_HIP(hipMemcpyAsync(base + o_fr, h_frames + p0 * F, m * F, hipMemcpyHostToDevice, s));
    if (h_csum_in_or_null)
      RUDP_HIP(hipMemcpyAsync(base + o_ci, h_csum_in_or_null + p0, m * 2, hipMemcpyHostToDevice, s));
    return 0;
  };
  auto kern = [&](char* base, uint64_t, uint64_t m, hipStream_t s) -> int {
    return rudp_decode_utf8((const uint8_t*)(base + o_fr), nullptr, frame_len, m,
                            h_csum_in_or_null ? (const uint16_t*)(base + o_ci) : nullptr,
                            (uint16_t*)(base + o_seq), (uint16_t*)(base + o_ack), (uint8_t*)(base + o_fl),
                            (uint8_t*)(base + o_ok), h_csum_out_or_null ? (uint16_t*)(base + o_co) : nullptr,
                            h_pay ? (uint8_t*)(base + o_pay) : nullptr, h_val ? (uint8_t*)(base + o_va) : nullptr,
                            layout, device, s);
  };
  auto d2h = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    RUDP_HIP(hipMemcpyAsync(h_seq + p0, base + o_seq, m * 2, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_ack + p0, base + o_ack, m * 2, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_flags + p0, base + o_fl, m, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_ok + p0, base + o_ok, m, hipMemcpyDeviceToHost, s));
    if (h_csum_out_or_null)
      RUDP_HIP(hipMemcpyAsync(h_csum_out_or_null + p0, base + o_co, m * 2, hipMemcpyDeviceToHost, s));
    if (h_pay) RUDP_HIP(hipMemcpyAsync(h_pay + p0 * L, base + o_pay, m * L, hipMemcpyDeviceToHost, s));
    if (h_val) RUDP_HIP(hipMemcpyAsync(h_val + p0, base + o_va, m, hipMemcpyDeviceToHost, s));
    return 0;
  };
  return run_pipeline(pp, n, cn, h2d, kern, d2h);
}

// Packed payloads in host memory to packed frames in host memory (the send
// side's socket buffer, utils/reliableUDP.py:53-61 per datagram).  A pre-pass
// over the lengths (sum and maximum, per chunk) checks every length and the
// frame buffer's capacity before anything is enqueued, and cuts the batch
// into chunks whose payload bytes fit a slot; each chunk is one checked
// device encode (its offsets from 0) plus one add of its base, so the
// offsets that come back are the batch's own.
int rudp_encode_varlen_host(const rudp_batch* h_in, uint64_t payload_bytes, uint8_t* h_frames, uint64_t frames_cap,
                            uint64_t* h_frame_off, uint16_t* h_csum_or_null, int layout, int device) {
  if (!h_in) return fail(RUDP_EINVAL, "rudp_encode_varlen_host: batch is NULL");
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (!h_frame_off) return fail(RUDP_EINVAL, "rudp_encode_varlen_host: frame_off is NULL");
  const uint64_t n = h_in->n;
  if (n == 0) {
    h_frame_off[0] = 0;
    return 0;
  }
  if (h_in->payload_off)
    return fail(RUDP_ENOTSUP, "rudp_encode_varlen_host: packed payloads only (payload_off must be NULL)");
  if (!h_in->len || !h_in->seq || !h_in->ack || !h_in->flags || !h_frames)
    return fail(RUDP_EINVAL, "rudp_encode_varlen_host: NULL buffer for a non-empty batch");
  if (n > 0x7FFFFFFFull) return fail(RUDP_EINVAL, "rudp_encode_varlen_host: at most 2^31-1 packets per call");
  const uint64_t H = (uint64_t)layout;
  // Zero copy: packed payloads of small frames (mean under varlen_small bytes)
  // in pinned host memory, every array pinned, payload and frames 16-B aligned:
  // ONE checked encode over the whole batch whose kernels read the lengths,
  // header table and payloads over PCIe and store frames, offsets and checksums
  // back over it.  No host pass over the lengths: the device's own checks
  // (lengths, their sum against payload_bytes, the frames' capacity) come back
  // as its status word, with the messages the host checks give.
  if (tuning().host_zero_copy && tuning().varlen_small > 0 && payload_bytes / n < (uint64_t)tuning().varlen_small &&
      h_in->payload && aligned16(h_in->payload) && aligned16(h_frames) && device_writable_host(h_in->payload) &&
      device_writable_host(h_in->len) && device_writable_host(h_in->seq) && device_writable_host(h_in->ack) &&
      device_writable_host(h_in->flags) && device_writable_host(h_frames) && device_writable_host(h_frame_off) &&
      device_writable_host(h_csum_or_null)) {
    DeviceScope dev_scope;
    int rc = dev_scope.set(device);
    if (rc) return rc;
    Pipeline* pp = pipeline_for(device);
    std::lock_guard<std::mutex> lk(pp->mu);
    if ((rc = pipeline_init(pp))) return rc;
    rudp_batch b = *h_in;
    b.payload_len = (uint32_t)(payload_bytes / n);  // the batch's mean: picks the tiles and the length codes
    rc = rudp_encode_varlen_checked(&b, payload_bytes, h_frames, frames_cap, h_frame_off, h_csum_or_null,
                                    pp->d_status, layout, device, pp->comp);
    if (!rc) {
      RUDP_HIP(hipMemcpyAsync(pp->h_status, pp->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost, pp->comp));
    }
    const hipError_t e = hipStreamSynchronize(pp->comp);
    if (rc) return rc;
    if (e != hipSuccess) return hip_fail(e, "zero-copy varlen encode");
    const uint32_t st = *pp->h_status;
    if (st & RUDP_ST_LEN) return fail(RUDP_EINVAL, "lengths must lie in [0, 65535]");
    if (st & RUDP_ST_PAYLOAD)
      return fail(RUDP_EINVAL, "packed payloads: sum(lengths) must equal payload.numel() (%llu)",
                  (unsigned long long)payload_bytes);
    if (st & RUDP_ST_FRAMES_CAP)
      return fail(RUDP_EINVAL, "out is too small for the frames (sum(lengths) + N * header bytes > %llu)",
                  (unsigned long long)frames_cap);
    if (st) return fail(RUDP_EINVAL, "rudp_encode_varlen_host: the device rejected the batch (status 0x%x)", st);
    return 0;
  }
  const uint64_t bmax = stage_bytes();
  const uint64_t hint = h_in->payload_len ? h_in->payload_len : 1u;
  uint64_t cn = chunk_packets(n, 2u * hint + H + 13u);
  if (cn > (1u << 22)) cn = 1u << 22;
  // the plan: chunk k = packets [start[k], start[k + 1]) with pay[k] payload bytes
  std::vector<uint64_t> start{0}, pay;
  uint64_t total = 0;
  for (uint64_t p0 = 0; p0 < n;) {
    uint64_t m = n - p0 < cn ? n - p0 : cn;
    for (;;) {
      uint64_t sum = 0;
      uint32_t mx = 0;
      lengths_sum_max(h_in->len + p0, m, &sum, &mx);
      if (mx > 65535u)
        return fail(RUDP_EINVAL, "lengths must lie in [0, 65535] (packets [%llu, %llu))",
                    (unsigned long long)p0, (unsigned long long)(p0 + m));
      if (sum <= bmax || m == 1) {
        pay.push_back(sum);
        total += sum;
        p0 += m;
        start.push_back(p0);
        break;
      }
      m /= 2;
    }
  }
  if (total != payload_bytes)
    return fail(RUDP_EINVAL, "packed payloads: sum(lengths) must equal payload.numel() (%llu vs %llu)",
                (unsigned long long)total, (unsigned long long)payload_bytes);
  if (total && !h_in->payload) return fail(RUDP_EINVAL, "rudp_encode_varlen_host: payload is NULL");
  if (total + n * H > frames_cap)
    return fail(RUDP_EINVAL, "out is too small for the frames (sum(lengths) + N * header bytes = %llu > %llu)",
                (unsigned long long)(total + n * H), (unsigned long long)frames_cap);
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  // Pinned offset / checksum arrays: for chunks that take the small-frame tile
  // (its checksums leave as coalesced stores) the kernels store them directly,
  // two D2H copies per chunk fewer; the frames always come back by one copy.
  const bool pinned_out = tuning().host_direct_out && device_writable_host(h_frame_off) &&
                          device_writable_host(h_csum_or_null);
  auto direct_chunk = [&](uint64_t pb, uint64_t m) {
    return pinned_out && tuning().varlen_small > 0 && pb / m < (uint64_t)tuning().varlen_small;
  };
  const size_t o_pay = 0, o_fr = up256(bmax), o_len = o_fr + up256(bmax + cn * H + 64u),
               o_seq = o_len + up256(cn * 4), o_ack = o_seq + up256(cn * 2), o_fl = o_ack + up256(cn * 2),
               o_cs = o_fl + up256(cn), o_off = o_cs + up256(cn * 2), o_st = o_off + up256((cn + 1) * 8),
               slot = o_st + 256;
  Pipeline* pp = pipeline_for(device);
  std::lock_guard<std::mutex> lk(pp->mu);
  if ((rc = pipeline_reserve(pp, pipeline_slots(), slot))) return rc;
  size_t k = 0;
  uint64_t pbase = 0;  // payload bytes before the current chunk
  auto plan = [&](uint64_t p0) -> int64_t {
    if (k > 0) pbase += pay[k - 1];
    (void)p0;
    const uint64_t m = start[k + 1] - start[k];
    ++k;
    return (int64_t)m;
  };
  auto h2d = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    const uint64_t pb = pay[k - 1];
    if (pb) RUDP_HIP(hipMemcpyAsync(base + o_pay, h_in->payload + pbase, pb, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_len, h_in->len + p0, m * 4, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_seq, h_in->seq + p0, m * 2, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_ack, h_in->ack + p0, m * 2, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_fl, h_in->flags + p0, m, hipMemcpyHostToDevice, s));
    return 0;
  };
  auto kern = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    const uint64_t pb = pay[k - 1];
    rudp_batch sub{};
    sub.n = m;
    sub.payload_len = (uint32_t)(pb / m < 65535u ? pb / m : 65535u);  // the chunk's mean: picks the tiles
    sub.seq = (const uint16_t*)(base + o_seq);
    sub.ack = (const uint16_t*)(base + o_ack);
    sub.flags = (const uint8_t*)(base + o_fl);
    sub.payload = (const uint8_t*)(base + o_pay);
    sub.len = (const uint32_t*)(base + o_len);
    const bool direct = direct_chunk(pb, m);
    uint16_t* cs = h_csum_or_null ? (direct ? h_csum_or_null + p0 : (uint16_t*)(base + o_cs)) : nullptr;
    int r = rudp_encode_varlen_checked(&sub, pb, (uint8_t*)(base + o_fr), pb + m * H + 64u, (uint64_t*)(base + o_off),
                                       cs, (uint32_t*)(base + o_st), layout, device, s);
    if (r) return r;
    const uint64_t fbase = pbase + p0 * H;
    // offsets [p0, p0 + m): the chunk's last entry is the next chunk's first
    const uint64_t last = start[k] == n ? m + 1 : m;
    uint64_t* off = (uint64_t*)(base + o_off);
    hipLaunchKernelGGL(add_base_kernel, dim3(fbase || direct ? (uint32_t)((m + 256u) / 256u) : 1u), dim3(256), 0, s,
                       off, direct ? h_frame_off + p0 : off, direct ? last : m + 1, fbase,
                       (const uint32_t*)(base + o_st), pp->d_status);
    RUDP_HIP(hipGetLastError());
    return 0;
  };
  auto d2h = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    const uint64_t fb = pay[k - 1] + m * H;
    RUDP_HIP(hipMemcpyAsync(h_frames + pbase + p0 * H, base + o_fr, fb, hipMemcpyDeviceToHost, s));
    if (direct_chunk(pay[k - 1], m)) return 0;  // offsets and checksums stored by the kernels
    // offsets [p0, p0 + m): the chunk's last entry is the next chunk's first
    const uint64_t last = start[k] == n ? m + 1 : m;
    RUDP_HIP(hipMemcpyAsync(h_frame_off + p0, base + o_off, last * 8, hipMemcpyDeviceToHost, s));
    if (h_csum_or_null) RUDP_HIP(hipMemcpyAsync(h_csum_or_null + p0, base + o_cs, m * 2, hipMemcpyDeviceToHost, s));
    return 0;
  };
  // The device's own checks of every chunk (RUDP_ST_*, the checked encode's
  // status) are read back, not assumed from the host's pre-pass.
  *pp->h_status = 0;
  RUDP_HIP(hipMemsetAsync(pp->d_status, 0, sizeof(uint32_t), pp->comp));
  rc = run_pipeline_planned(pp, n, plan, h2d, kern, d2h);
  if (rc) return rc;
  RUDP_HIP(hipMemcpyAsync(pp->h_status, pp->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost, pp->comp));
  RUDP_HIP(hipStreamSynchronize(pp->comp));
  if (*pp->h_status)
    return fail(RUDP_EINVAL, "rudp_encode_varlen_host: the device rejected the batch (status 0x%x)", *pp->h_status);
  return 0;
}

// Packed frames in host memory (a recvmmsg batch): chunks of consecutive
// frames, each staged as the byte range its offsets span.  The plan scans a
// chunk's n + 1 offsets for their least and greatest value at or below
// frames_bytes (the only ones any kernel reads at: a frame with an offset
// past frames_bytes or out of order is rejected before any of its bytes is
// read), copies that range, 16-B aligned, to the slot and hands the decode a
// frames pointer moved back by the range's start, so the caller's own
// offsets index the slot unchanged and the device applies the checked rule
// to them against frames_bytes: the result is rudp_decode_varlen_utf8's on
// the same bytes.  A chunk whose range outgrows the slot is halved (a
// ragged batch, offsets out of order) down to one frame; one valid frame
// larger than the slot is refused.
int rudp_decode_varlen_host(const uint8_t* h_frames, uint64_t frames_bytes, const uint64_t* h_frame_off,
                            uint32_t len_hint, uint64_t n, const uint16_t* h_csum_in_or_null, uint16_t* h_seq,
                            uint16_t* h_ack, uint8_t* h_flags, uint8_t* h_ok, uint16_t* h_csum_out_or_null,
                            uint8_t* h_valid_or_null, uint32_t* h_status_or_null, int layout, int device) {
  if (h_status_or_null) *h_status_or_null = 0;
  if (layout != RUDP_LAYOUT_RUDP5 && layout != RUDP_LAYOUT_RUDP7)
    return fail(RUDP_EINVAL, "unsupported layout %d (use 5 or 7)", layout);
  if (n == 0) return 0;
  if (!h_frame_off || !h_seq || !h_ack || !h_flags || !h_ok || (frames_bytes && !h_frames))
    return fail(RUDP_EINVAL, "rudp_decode_varlen_host: NULL buffer for a non-empty batch");
  if (n > 0x7FFFFFFFull) return fail(RUDP_EINVAL, "rudp_decode_varlen_host: at most 2^31-1 frames per call");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  const uint64_t hint = len_hint ? len_hint : (frames_bytes / n ? frames_bytes / n : 1u);
  const uint64_t bmax = stage_bytes();  // frame bytes a slot holds
  const bool small = tuning().varlen_small > 0 && hint < (uint64_t)tuning().varlen_small + (uint64_t)layout;
  // Zero copy: a batch of small frames whose every array is pinned host memory
  // (a recvmmsg ring, torch's pinned allocator) decodes in ONE launch of the
  // small-frame tile that reads the frames, offsets and sideband checksums over
  // PCIe and stores the fields back over it -- no staging slot, no chunks, no
  // copies.  The kernel applies the checked rule to every frame's offsets
  // itself, so the result is rudp_decode_varlen_utf8's.
  if (tuning().host_zero_copy && small && aligned16(h_frames) && device_writable_host(h_frames) &&
      device_writable_host(h_frame_off) && device_writable_host(h_csum_in_or_null) && device_writable_host(h_seq) &&
      device_writable_host(h_ack) && device_writable_host(h_flags) && device_writable_host(h_ok) &&
      device_writable_host(h_csum_out_or_null) && device_writable_host(h_valid_or_null)) {
    Pipeline* pp = pipeline_for(device);
    std::lock_guard<std::mutex> lk(pp->mu);
    if ((rc = pipeline_init(pp))) return rc;
    // (the rejected-offsets status from the kernels' own flag word, 4 bytes
    // back, not a host scan of ok[]: 1 MiB of pinned memory per 1M frames)
    if (h_status_or_null) RUDP_HIP(hipMemsetAsync(pp->d_status, 0, sizeof(uint32_t), pp->comp));
    rc = decode_varlen(h_frames, h_frame_off, (uint32_t)(hint < 0xFFFFFFFFull ? hint : 0xFFFFFFFFu), n,
                       h_csum_in_or_null, h_seq, h_ack, h_flags, h_ok, h_csum_out_or_null, nullptr, layout, device,
                       pp->comp, true, h_status_or_null ? pp->d_status : nullptr, frames_bytes, h_valid_or_null);
    if (!rc && h_status_or_null)
      RUDP_HIP(hipMemcpyAsync(pp->h_status, pp->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost, pp->comp));
    const hipError_t e = hipStreamSynchronize(pp->comp);
    if (rc) return rc;
    if (e != hipSuccess) return hip_fail(e, "zero-copy varlen decode");
    if (h_status_or_null) *h_status_or_null = *pp->h_status & RUDP_ST_OFFSETS;
    return 0;
  }
  // Pinned output arrays: the small-frame decode tile (the reference's 6-9 B
  // datagrams; its per-frame outputs leave as lane-strided, coalesced stores)
  // writes the fields into them directly: six D2H copies per chunk fewer.
  // Pageable arrays, and MTU frames (whose fields a group leader stores one at
  // a time: 2-B PCIe writes), take the slot and the copies.
  const bool direct = tuning().host_direct_out && small && device_writable_host(h_seq) &&
                      device_writable_host(h_ack) &&
                      device_writable_host(h_flags) && device_writable_host(h_ok) &&
                      device_writable_host(h_csum_out_or_null) && device_writable_host(h_valid_or_null);
  // frames per chunk: 3/4 of a slot's bytes at the hint (room for ragged
  // lengths), at least host_min_chunks chunks for a batch over 4 MiB
  uint64_t cn = chunk_packets(n, hint * 4u / 3u + 1u);
  if (cn > (1u << 22)) cn = 1u << 22;
  // (64 guard bytes before and after the staged range: the UTF-8 check reads the
  // dword before a payload chunk, the tile kernels whole 16-B chunks)
  const size_t o_fr = 64, o_off = up256(o_fr + bmax + 64u), o_ci = o_off + up256((cn + 1) * 8), o_seq = o_ci + up256(cn * 2),
               o_ack = o_seq + up256(cn * 2), o_co = o_ack + up256(cn * 2), o_fl = o_co + up256(cn * 2),
               o_ok = o_fl + up256(cn), o_va = o_ok + up256(cn), slot = o_va + up256(h_valid_or_null ? cn : 0);
  Pipeline* pp = pipeline_for(device);
  std::lock_guard<std::mutex> lk(pp->mu);
  if ((rc = pipeline_reserve(pp, pipeline_slots(), slot))) return rc;
  uint64_t a0 = 0, a1 = 0;  // the current chunk's staged range [a0, a1), a0 16-B aligned
  auto plan = [&](uint64_t p0) -> int64_t {
    uint64_t m = n - p0 < cn ? n - p0 : cn;
    for (;;) {
      uint64_t lo = ~0ull, hi = 0;
      offsets_range(h_frame_off + p0, m + 1, frames_bytes, &lo, &hi);
      if (lo > hi) lo = hi = 0;  // no offset inside the buffer: every frame is rejected unread
      const uint64_t b0 = lo & ~15ull;
      uint64_t b1 = (hi + 15u) & ~15ull;
      if (b1 > frames_bytes) b1 = frames_bytes;
      if (b1 - b0 <= bmax) {
        a0 = b0;
        a1 = b1 > b0 ? b1 : b0;
        return (int64_t)m;
      }
      if (m == 1) {
        // A frame the checked rule rejects (its offsets out of order, or past
        // the buffer) is decoded from no bytes at all: nothing is staged, and
        // the device marks it RUDP_OK_BAD_OFFSETS as rudp_decode_varlen_utf8
        // would.  Only a valid frame larger than a slot is refused.
        const uint64_t f0 = h_frame_off[p0], f1 = h_frame_off[p0 + 1];
        if (f0 > f1 || f1 > frames_bytes) {
          a0 = a1 = 0;
          return 1;
        }
        return fail(RUDP_ENOTSUP, "rudp_decode_varlen_host: frame %llu spans %llu bytes, over the %zu-byte staging slot",
                    (unsigned long long)p0, (unsigned long long)(b1 - b0), (size_t)bmax);
      }
      m /= 2;
    }
  };
  auto h2d = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    if (a1 > a0) RUDP_HIP(hipMemcpyAsync(base + o_fr, h_frames + a0, a1 - a0, hipMemcpyHostToDevice, s));
    RUDP_HIP(hipMemcpyAsync(base + o_off, h_frame_off + p0, (m + 1) * 8, hipMemcpyHostToDevice, s));
    if (h_csum_in_or_null)
      RUDP_HIP(hipMemcpyAsync(base + o_ci, h_csum_in_or_null + p0, m * 2, hipMemcpyHostToDevice, s));
    return 0;
  };
  auto kern = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    // frame bytes at offset x (a0 <= x < a1) sit at base + (x - a0)
    const uint8_t* frames = reinterpret_cast<const uint8_t*>(base + o_fr) - a0;
    const uint32_t h32 = (uint32_t)(hint < 0xFFFFFFFFull ? hint : 0xFFFFFFFFu);
    const uint16_t* ci = h_csum_in_or_null ? (const uint16_t*)(base + o_ci) : nullptr;
    if (direct)
      return decode_varlen(frames, (const uint64_t*)(base + o_off), h32, m, ci, h_seq + p0, h_ack + p0, h_flags + p0,
                           h_ok + p0, h_csum_out_or_null ? h_csum_out_or_null + p0 : nullptr, nullptr, layout, device,
                           s, true, nullptr, frames_bytes, h_valid_or_null ? h_valid_or_null + p0 : nullptr);
    return decode_varlen(frames, (const uint64_t*)(base + o_off), h32, m, ci, (uint16_t*)(base + o_seq),
                         (uint16_t*)(base + o_ack), (uint8_t*)(base + o_fl), (uint8_t*)(base + o_ok),
                         h_csum_out_or_null ? (uint16_t*)(base + o_co) : nullptr, nullptr, layout, device, s, true,
                         nullptr, frames_bytes, h_valid_or_null ? (uint8_t*)(base + o_va) : nullptr);
  };
  auto d2h = [&](char* base, uint64_t p0, uint64_t m, hipStream_t s) -> int {
    if (direct) return 0;  // the kernel wrote them
    RUDP_HIP(hipMemcpyAsync(h_seq + p0, base + o_seq, m * 2, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_ack + p0, base + o_ack, m * 2, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_flags + p0, base + o_fl, m, hipMemcpyDeviceToHost, s));
    RUDP_HIP(hipMemcpyAsync(h_ok + p0, base + o_ok, m, hipMemcpyDeviceToHost, s));
    if (h_csum_out_or_null)
      RUDP_HIP(hipMemcpyAsync(h_csum_out_or_null + p0, base + o_co, m * 2, hipMemcpyDeviceToHost, s));
    if (h_valid_or_null) RUDP_HIP(hipMemcpyAsync(h_valid_or_null + p0, base + o_va, m, hipMemcpyDeviceToHost, s));
    return 0;
  };
  rc = run_pipeline_planned(pp, n, plan, h2d, kern, d2h);
  if (rc) return rc;
  if (h_status_or_null && memchr(h_ok, RUDP_OK_BAD_OFFSETS, n)) *h_status_or_null = RUDP_ST_OFFSETS;
  return 0;
}

// ---- the proxy's retransmission count over a stream of batches ----------------
struct rudp_dedup_stream {
  static constexpr int kStages = 4;
  std::mutex mu;  // push and counts from any threads, one at a time (the relay's thread and a stats reader)
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t window = 0, max_batch = 0, max_frame = 0;
  uint8_t* arena[2] = {nullptr, nullptr};  // history, then the batch behind it; used in turn
  int cur = 0;
  uint64_t* d_off = nullptr;               // [window + max_batch + 1]
  uint8_t* d_dup = nullptr;                // [window + max_batch]
  uint8_t* d_side = nullptr;               // [max_batch]
  uint64_t* d_counts = nullptr;            // [2]
  struct Stage {                           // pinned staging of one push, reused after its copies ran
    uint8_t* frames = nullptr;
    uint64_t* off = nullptr;
    uint8_t* side = nullptr;
    uint64_t* counts = nullptr;
    hipEvent_t done = nullptr;
    bool used = false;
  } stage[kStages];
  int si = 0;
  std::deque<uint32_t> hist;               // lengths of the kept datagrams (host: every offset is known here)
  uint64_t hist_bytes = 0;
};

namespace {
void dedup_stream_free(rudp_dedup_stream* st) {
  if (!st) return;
  if (st->stream) (void)hipStreamSynchronize(st->stream);
  for (uint8_t* a : st->arena) (void)hipFree(a);
  (void)hipFree(st->d_off);
  (void)hipFree(st->d_dup);
  (void)hipFree(st->d_side);
  (void)hipFree(st->d_counts);
  for (auto& g : st->stage) {
    (void)hipHostFree(g.frames);
    (void)hipHostFree(g.off);
    (void)hipHostFree(g.side);
    (void)hipHostFree(g.counts);
    if (g.done) (void)hipEventDestroy(g.done);
  }
  delete st;
}
}  // namespace

int rudp_dedup_stream_create(uint32_t window, uint32_t max_batch, uint32_t max_frame, int device, void* hip_stream,
                             rudp_dedup_stream** out) {
  if (!out) return fail(RUDP_EINVAL, "rudp_dedup_stream_create: out is NULL");
  *out = nullptr;
  if (window > dedup_max_window()) return fail(RUDP_EINVAL, "window %u exceeds %u", window, dedup_max_window());
  if (max_batch == 0 || max_batch > (1u << 24) || max_frame > 65535u + 7u)
    return fail(RUDP_EINVAL, "rudp_dedup_stream_create: max_batch in [1, 2^24], max_frame <= 65542");
  DeviceScope dev_scope;
  int rc = dev_scope.set(device);
  if (rc) return rc;
  rudp_dedup_stream* st = new rudp_dedup_stream();
  st->device = device;
  st->stream = (hipStream_t)hip_stream;
  st->window = window;
  st->max_batch = max_batch;
  st->max_frame = max_frame;
  const uint64_t entries = (uint64_t)window + max_batch;
  const size_t arena = (size_t)(entries * (max_frame ? max_frame : 1u) + 16u);
  const size_t batch_bytes = (size_t)max_batch * max_frame + 16u;
  hipError_t e = hipSuccess;
  for (auto& a : st->arena)
    if (e == hipSuccess) e = hipMalloc(&a, arena);
  if (e == hipSuccess) e = hipMalloc(&st->d_off, (entries + 1) * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&st->d_dup, entries);
  if (e == hipSuccess) e = hipMalloc(&st->d_side, max_batch);
  if (e == hipSuccess) e = hipMalloc(&st->d_counts, 2 * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMemsetAsync(st->d_counts, 0, 2 * sizeof(uint64_t), st->stream);
  for (auto& g : st->stage) {
    if (e == hipSuccess) e = hipHostMalloc(&g.frames, batch_bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(&g.off, (entries + 1) * sizeof(uint64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(&g.side, max_batch, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(&g.counts, 2 * sizeof(uint64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&g.done, hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    dedup_stream_free(st);
    return hip_fail(e, "rudp_dedup_stream_create");
  }
  *out = st;
  return 0;
}

int rudp_dedup_stream_push(rudp_dedup_stream* st, const uint8_t* h_frames, const uint64_t* h_frame_off, uint64_t n,
                           const uint8_t* h_side_or_null, uint8_t* d_dup_or_null) {
  if (!st || (!h_frame_off && n)) return fail(RUDP_EINVAL, "rudp_dedup_stream_push: NULL argument");
  if (n == 0) return 0;
  if (n > st->max_batch) return fail(RUDP_EINVAL, "batch of %llu exceeds max_batch %u", (unsigned long long)n,
                                     st->max_batch);
  std::lock_guard<std::mutex> lk(st->mu);
  for (uint64_t i = 0; i < n; ++i)
    if (h_frame_off[i + 1] < h_frame_off[i] || h_frame_off[i + 1] - h_frame_off[i] > st->max_frame)
      return fail(RUDP_EINVAL, "rudp_dedup_stream_push: offsets decreasing or a frame over max_frame");
  const uint64_t bb = h_frame_off[n] - h_frame_off[0];
  if (bb && !h_frames) return fail(RUDP_EINVAL, "rudp_dedup_stream_push: frames is NULL");
  DeviceScope dev_scope;
  int rc = dev_scope.set(st->device);
  if (rc) return rc;
  hipStream_t s = st->stream;
  auto& g = st->stage[st->si];
  st->si = (st->si + 1) % rudp_dedup_stream::kStages;
  if (g.used) RUDP_HIP(hipEventSynchronize(g.done));  // its copies (kStages pushes ago) have run
  g.used = true;
  // the history's offsets, then the batch's behind them, all known on the host
  const uint64_t h = st->hist.size(), hb = st->hist_bytes;
  uint64_t o = 0, k = 0;
  for (const uint32_t len : st->hist) {
    g.off[k++] = o;
    o += len;
  }
  for (uint64_t i = 0; i <= n; ++i) g.off[h + i] = hb + (h_frame_off[i] - h_frame_off[0]);
  if (bb) memcpy(g.frames, h_frames + h_frame_off[0], bb);
  if (h_side_or_null) {
    for (uint64_t i = 0; i < n; ++i) g.side[i] = h_side_or_null[i] ? 1 : 0;
  }
  uint8_t* arena = st->arena[st->cur];
  if (bb) RUDP_HIP(hipMemcpyAsync(arena + hb, g.frames, bb, hipMemcpyHostToDevice, s));
  RUDP_HIP(hipMemcpyAsync(st->d_off, g.off, (h + n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  if (h_side_or_null) RUDP_HIP(hipMemcpyAsync(st->d_side, g.side, n, hipMemcpyHostToDevice, s));
  RUDP_HIP(hipEventRecord(g.done, s));
  // one dedup launch over history + batch (the checked rule; packed, 16-B aligned arena)
  {
    ScratchCall call(s);
    DedupArgs a{};
    a.frames = arena;
    a.frame_off = st->d_off;
    a.n = h + n;
    a.window = st->window;
    a.dup = st->d_dup;
    const uint64_t total = hb + bb;
    const uint32_t mean = (uint32_t)(total / (h + n));
    a.F = mean;
    a.glog = mean <= 16u ? 0u : mean <= 64u ? 1u : mean <= 256u ? 2u : 3u;
    a.lim_checked = 1;
    a.frames_lim = total;
    a.small_cap = dedup_small_cap(mean, st->window);
    if (!a.small_cap) {
      void* scratch = nullptr;
      RUDP_HIP(stream_scratch(&scratch, (h + n) * sizeof(uint64_t), s, kScratchHash));
      a.hash = (uint64_t*)scratch;
    }
    rc = launch_dedup(a, s);
    if (rc) return hip_fail((hipError_t)rc, "dedup launch");
  }
  rc = launch_dedup_count(st->d_dup + h, h_side_or_null ? st->d_side : nullptr, n, st->d_counts, s);
  if (rc) return hip_fail((hipError_t)rc, "dedup count launch");
  if (d_dup_or_null) RUDP_HIP(hipMemcpyAsync(d_dup_or_null, st->d_dup + h, n, hipMemcpyDeviceToDevice, s));
  // keep the last `window` datagrams, at the front of the other arena
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t len = (uint32_t)(h_frame_off[i + 1] - h_frame_off[i]);
    st->hist.push_back(len);
    st->hist_bytes += len;
  }
  uint64_t first_off = 0;
  while (st->hist.size() > st->window) {
    first_off += st->hist.front();
    st->hist_bytes -= st->hist.front();
    st->hist.pop_front();
  }
  if (st->hist_bytes)
    RUDP_HIP(hipMemcpyAsync(st->arena[1 - st->cur], arena + first_off, st->hist_bytes, hipMemcpyDeviceToDevice, s));
  st->cur = 1 - st->cur;
  return 0;
}

int rudp_dedup_stream_counts(rudp_dedup_stream* st, uint64_t* h_counts) {
  if (!st || !h_counts) return fail(RUDP_EINVAL, "rudp_dedup_stream_counts: NULL argument");
  std::lock_guard<std::mutex> lk(st->mu);  // (its pinned read-back buffer is the object's, shared with push)
  DeviceScope dev_scope;
  int rc = dev_scope.set(st->device);
  if (rc) return rc;
  uint64_t* pin = st->stage[0].counts;
  RUDP_HIP(hipMemcpyAsync(pin, st->d_counts, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st->stream));
  RUDP_HIP(hipStreamSynchronize(st->stream));
  h_counts[0] = pin[0];
  h_counts[1] = pin[1];
  return 0;
}

int rudp_dedup_stream_destroy(rudp_dedup_stream* st) {
  if (!st) return 0;
  { std::lock_guard<std::mutex> lk(st->mu); }  // a push or counts still running on another thread ends first
  DeviceScope dev_scope;
  (void)dev_scope.set(st->device);
  dedup_stream_free(st);
  return 0;
}

}  // extern "C"
