// Launcher interface between the C ABI (capi.hip) and the kernels.
//
// Two builds come from these sources (rudp/_build.py):
//   librudp.so        the product: every launch choice is the measured default
//                     (the Tuning values below are compile-time constants), no
//                     diagnostics in any kernel, only the include/rudp.h ABI;
//   librudp_tools.so  RUDP_TOOLS=1, for tools/ and the tests of the non-default
//                     kernel forms: the same ABI plus rudpx_tune (every Tuning
//                     value a runtime knob), rudpx_encode_trace (tile timelines),
//                     rudpx_stamp and the streaming-copy ceilings (tuning.hip).
#pragma once
// The diagnostics build (RUDP_TOOLS) puts every internal name in a namespace
// of its own, so its kernels and functions (whose argument structs differ
// from the product's) can never bind to the product library's in one process.
#ifndef RUDP_NS
#if defined(RUDP_TOOLS) && RUDP_TOOLS
#define RUDP_NS rudp_tools
#else
#define RUDP_NS rudp
#endif
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/rudp.h"

#ifndef RUDP_TOOLS
#define RUDP_TOOLS 0
#endif

namespace RUDP_NS {

struct EncodeTileArgs {
  const unsigned char* payload;
  const uint16_t* seq;
  const uint16_t* ack;
  const uint8_t* flags;
  unsigned char* frames;
  uint16_t* csum;       // may be null
  uint64_t n;
  uint32_t L;           // payload bytes per packet
  uint32_t T;           // packets per tile (power of 2, 4..256)
  uint32_t glog;        // log2(256 / T): lanes per packet
  uint32_t hdr_bytes;   // LDS bytes reserved for the tile's header words
  uint64_t invF;        // ceil(2^32 / (L + H)) for exact x / F, x < T*F
  uint32_t xcd_swizzle; // 1: map blocks b, b+8, ... to consecutive tiles (one XCD each)
  uint32_t num_tiles;
  uint32_t out_align64; // phase 2 deals full chunks from the tile's first 64-B boundary
  uint32_t early_table;     // tile kernel: header-table loads issued before phase 1 (2: by LDS-DMA
                            // into tab_off with the payload, full tiles of T = 16)
  uint32_t tab_off;         // LDS byte offset of that table copy: seq [16] u16, ack [16] u16, flags [16] u8
  uint32_t hchunk;          // tile kernel (T % 16 == 0): leaders prebuild header chunks in LDS
  uint32_t hc_off;          // LDS byte offset of the header-chunk array [T + 1][2] x 16 B
  uint32_t hc_scratch;      // leaders build header chunks through a 48-B LDS scratch per packet
  uint32_t scr_off;         // LDS byte offset of that scratch [T][48 B]
#if RUDP_TOOLS
  uint64_t* trace;          // diagnostics (rudpx_encode_trace): per tile {start, end, XCC, CU}
#endif
};

struct DecodeArgs {
  const unsigned char* frames;
  const uint16_t* csum_in;  // rudp5 sideband, may be null
  uint16_t* seq;
  uint16_t* ack;
  uint8_t* flags;
  uint8_t* ok;
  uint16_t* csum_out;       // may be null
  unsigned char* payload_out;  // may be null
  uint8_t* valid;           // tile kernels: strict UTF-8 of each payload in the same pass, or null
  uint64_t n;
  uint32_t F;               // frame bytes
  uint32_t glog;            // log2(lanes per packet)
  uint32_t align64;         // tile kernel: wave loads/stores start on 64-B sector boundaries
  uint32_t stage_out;       // tile kernel: outputs staged in LDS, written as dwords (pointers 4-B aligned)
  uint32_t xcd;             // tile kernel: XCD-contiguous tile order (xcd_tile)
#if RUDP_TOOLS
  uint64_t* trace;          // diagnostics (rudpx_encode_trace): per tile {start, staged, summed, end, XCC, CU}
#endif
};

struct SynthArgs {
  uint64_t key_ack, key_flags, key_payload;
  uint32_t isn;
  uint64_t first;
  uint64_t n;
  uint32_t L;
  uint32_t ascii;
  uint16_t* seq;
  uint16_t* ack;
  uint8_t* flags;
  unsigned char* payload;
};

// One span of the byte-tiled varlen encode (SpanStarts).
struct SpanRec {
  uint64_t fo;  // frame_off[p]
  uint32_t p;   // first packet whose payload starts in the span (n past the last)
  uint32_t pad;
};
struct VarlenArgs {
  const unsigned char* payload;   // encode: payload buffer
  const uint32_t* len;            // encode: payload bytes per packet
  const uint64_t* payload_off;    // encode: may be null (packed in order)
  const uint16_t* seq_in;
  const uint16_t* ack_in;
  const uint8_t* flags_in;
  unsigned char* frames;          // encode: output; decode: input (as const)
  const uint64_t* frame_off;      // [n + 1]
  uint16_t* csum;                 // encode sideband, may be null
  // decode outputs
  const uint16_t* csum_in;
  uint16_t* seq;
  uint16_t* ack;
  uint8_t* flags;
  uint8_t* ok;
  uint16_t* csum_out;
  uint8_t* valid;                 // decode: strict UTF-8 of each payload in the same pass, or null
  uint64_t n;
  uint32_t glog;                  // log2 lanes per packet (vector kernels); kNoVec = byte kernels
  // encode tile kernel (packed payload): packets per tile (power of two, 4..256),
  // log2(256 / tile_T), and the LDS payload bytes a tile may use (larger tiles
  // take the per-packet path inside the kernel).  tile_T = 0: no tile kernel.
  uint32_t tile_T;
  uint32_t tile_glog;
  uint32_t tile_cap;
  uint32_t align64;               // tile kernel: wave stores start on 64-B sector boundaries
  uint32_t early_table;           // tile kernel: header-table loads before phase 1
  uint32_t vhc;                   // tile kernel: prebuilt header chunks + pure-chunk fast phase 2
  uint32_t hc_off;                // LDS byte offset of the header-chunk array (set by the launcher)
  uint32_t early_fo;              // tile kernels: the tile's frame offsets loaded before phase 1
  // Sync-free entry points: the call's device status word (RUDP_ST_*), written
  // by an earlier kernel of the same call; every kernel returns without a
  // memory access past its own offsets when it is non-zero.  Null: unchecked.
  const uint32_t* status;
  // Decode: frames reach at most frames_lim bytes into the buffer, and a frame
  // whose offsets are decreasing or past it is rejected (ok = RUDP_OK_BAD_OFFSETS,
  // RUDP_ST_OFFSETS or'ed into *status_out when there is one, nothing read).
  // lim_checked 0: an unchecked caller, the limit is frame_off[n].
  uint64_t frames_lim;
  uint32_t* status_out;           // may be null also for a checked call (the rejections are in ok[])
  uint32_t lim_checked;           // decode: frames_lim bounds the frames (checked calls)
#if RUDP_TOOLS
  uint64_t* trace;                // diagnostics (rudpx_encode_trace): small-frame encode timeline per tile
  uint32_t diag;                  // diagnostics (rudpx_tune 61): varlen tile ablation bits
#endif
  uint32_t small_fpt;             // decode small-frame tile: frames per thread (0: not used)
  uint32_t small_cap;             // its LDS run budget in bytes
  uint32_t xcd;                   // tile kernels: XCD-contiguous tile order (xcd_tile)
  // Tile records (span_rec set, checked calls): workgroup t frames packets
  // span_rec[t].p .. span_rec[t+1].p, whose frames start at span_rec[t].fo.
  // The scan chose per call between packet tiles (tile_T packets each) and
  // byte tiles (the packets whose payload starts in one span of S bytes) and
  // wrote the chosen form's records; span_count = the grid (records - 1).
  // bt_slots is the most packets a tile holds in LDS; tile_Tl = max(tile_T,
  // bt_slots) sizes the LDS arrays.
  const struct SpanRec* span_rec;
  uint64_t span_count;
  uint32_t bt_slots;
  uint32_t tile_Tl;
  uint32_t tile_sums;             // tile sum pass: 2 from 128-B block sums, 0 chunk by chunk (decode: 1 per tile)
  // Decode by byte spans (checked calls): span_rec[k] = the first frame that
  // starts at or past k * span_S (decode_span_index_kernel); *span_flag ==
  // span_epoch when the offsets are not in order inside the buffer, and the
  // decode then checks frame by frame.
  const uint32_t* span_flag;
  uint32_t span_epoch;
  uint32_t span_S;
  uint32_t map_bal;               // encode tile: chunk map built by output units, not by frames
  uint32_t dec_nt;                // decode tile: threads per workgroup (256, or 128: two-wave tiles)
  uint32_t dec_r4;                // decode tile: payload chunks read four at a time
  // Fixed-stride batches through these kernels (frame_off == null): frame p
  // starts at fo_base + p * stride, and a packed payload at that offset - p * H
  // + po_delta (mod 2^64); len[] is stride - H for every packet.  The launcher
  // moves `frames` / `payload` back to a 16-B boundary and puts the distance
  // into fo_base / po_delta, so any caller alignment takes the tile kernels.
  // No offsets are read or written.
  uint64_t fo_base;
  uint64_t stride;
  uint64_t po_delta;
  // Small-frame encode after a pass 1 (varlen_small_nib): each thread's fpt
  // lengths as 8/fpt-bit offsets from len_code_base in one byte per thread of
  // each tile (all ones: read len[]); null: len[] only.
  const uint8_t* len_code;
  uint32_t len_code_base;
};
constexpr uint32_t kNoVec = 0xFFFFFFFFu;

struct Utf8Args {
  const unsigned char* frames;
  const uint64_t* frame_off;  // [n + 1] or null (fixed stride F)
  uint64_t n;
  uint32_t F;                 // fixed stride; with frame_off a mean-length hint
  uint32_t H;
  uint8_t* valid;
  uint32_t glog;              // log2 lanes per frame (vector kernel)
  uint32_t tile_cap;          // varlen tile kernel: LDS bytes a tile's run may use
  const uint32_t* status;     // sync-free call: RUDP_ST_* from check_frame_offsets, or null
  uint32_t xcd;               // tile kernels: XCD-contiguous tile order (xcd_tile)
};

struct DedupArgs {
  const unsigned char* frames;
  const uint64_t* frame_off;  // [n + 1] or null (fixed stride F)
  uint64_t n;
  uint32_t F;
  uint32_t window;
  uint32_t glog;              // hash pass: log2 lanes per frame (from the mean frame length)
  uint32_t lim_checked;       // frames reach at most frames_lim bytes: a frame whose offsets are
  uint64_t frames_lim;        // decreasing or past it gets dup = RUDP_DUP_BAD_OFFSETS, nothing read
  uint64_t* hash;             // scratch [n] (two-pass form)
  uint8_t* dup;
  uint32_t small_cap;         // > 0: the one-launch small-frame form, LDS run budget in bytes
};

constexpr uint32_t kTileMaxPayload = 4096;
// Largest payload accepted: a UDP datagram's size field is 16 bits, and it
// keeps every per-packet word sum exact in 32 bits (32768 words x 0xFFFF).
constexpr uint32_t kMaxPayload = 65535;

enum class DecodePath { kCopy, kCopyTile, kVerify, kVerifyTile };

// Launch choices, each at its measured default.  In librudp.so they are
// compile-time constants.  In the tools build each is an atomic int set by
// rudpx_tune (tuning.hip), read at launch, so a concurrent rudpx_tune is not a
// data race; a launch that runs while knobs change may see some old and some
// new values (the knobs are for sweeps, not for production callers).
#if RUDP_TOOLS
#define RUDP_KNOB(name, value) std::atomic<int> name{value};
#else
#define RUDP_KNOB(name, value) static constexpr int name = value;
#endif
struct Tuning {
  RUDP_KNOB(encode_nt_load, 1)
  RUDP_KNOB(encode_nt_store, 1)
  RUDP_KNOB(encode_tile, 0)    // packets per tile; 0 = automatic
  RUDP_KNOB(encode_p1, 8)      // phase-1 loads in flight per lane (2, 4, 8)
  RUDP_KNOB(encode_blocks_per_cu, -1)  // cap resident tiles per CU via LDS reservation; 0 = natural, -1 = auto
  RUDP_KNOB(decode_glog, -1)   // verify kernel lanes-per-packet log2; -1 = automatic
  // XCD-contiguous tile order (xcd_tile) for the fixed-length encode tile:
  // 1 on, 0 off, -1 from 512-B payloads (16M x 1472 B 0.540 -> 0.481 ms per
  // 2^20 packets; tools/launch_split.py, profiles/r02/sweeps/launch_split.json).
  RUDP_KNOB(encode_xcd_swizzle, -1)
#if RUDP_TOOLS
  std::atomic<uint64_t*> encode_trace{nullptr};  // diagnostics: tile timeline buffer (tools only)
#endif
  // The same order for the decode, varlen and UTF-8 tile kernels: fixed decode
  // verify 1M x 1472 B 0.240 -> 0.218 ms, x 1024 B 0.170 -> 0.154; copy-out
  // 1472 B 0.523 -> 0.504; varlen decode 1479 B 0.266 -> 0.230, ragged [0, 2944]
  // 0.306 -> 0.284; varlen encode 1472 B 0.587 -> 0.557; 256 B and below
  // within noise, fixed copy-out at 64 B 5% slower, so the fixed decode keeps
  // it off below 128-B frames (profiles/r02/sweeps/tile_xcd_*.json).
  RUDP_KNOB(tile_xcd, 1)
  RUDP_KNOB(encode_block, 256)  // tile workgroup size (64, 128 when T <= block; 256, 512, 1024)
  RUDP_KNOB(decode_copy_tile, 1)  // copy-out decode through an LDS tile (0: register windows)
  RUDP_KNOB(decode_verify_tile, 1)  // verify-only decode through an LDS tile (0: aligned-chunk kernel)
  RUDP_KNOB(varlen_vec, 1)     // varlen encode/decode: vector kernels (0: byte kernels)
  RUDP_KNOB(varlen_glog, -1)   // varlen lanes-per-packet log2 (0..6); -1 = from the length hint
  RUDP_KNOB(varlen_tile, 1)    // varlen encode of packed payloads through LDS tiles (0: vector kernel)
  RUDP_KNOB(varlen_tile_maxT, 256)     // varlen encode tile: most packets per tile
  RUDP_KNOB(varlen_tile_bytes, 0)  // varlen encode tile: payload bytes per tile at the hint (0 = automatic)
  // Wave loads/stores of the tile kernels start on a 64-B sector boundary
  // (1) or on the first 16-B one (0).  -1 = automatic: on for fixed-length
  // encode at every tile size (1M x 1472 B: 0.516 vs 0.533 ms; smaller
  // tiles equal or up to 1.3% faster since LDS-DMA phase 1), off for decode
  // and varlen, where it measured 1-3% slower
  // (profiles/r01/sweeps/align64.json, align64_after_dma.json).
  RUDP_KNOB(out_align64, -1)
  // Encode tile phase 1 by LDS-DMA (global_load_lds_dwordx4) in place of
  // register staging (256-thread contiguous tiles, nt loads and stores):
  // 1M x 256 B 0.0967 -> 0.0946 ms, x 512 B 0.1884 -> 0.1854, x 64 B 0.0301
  // -> 0.0292; x 1024 B and x 1472 B unchanged (profiles/r01/sweeps/span_vs_tile.json).
  RUDP_KNOB(encode_dma, 1)
  // Encode tile phase 2 with header chunks prebuilt by the packet leaders
  // (T % 16 == 0): 1M x 64 B 0.0295 -> 0.0287 ms, x 256 B 0.0962 -> 0.0938,
  // x 1024 B 0.3712 -> 0.3683, x 1472 B equal (profiles/r01/sweeps/encode_hchunk.json).
  RUDP_KNOB(encode_hchunk, 1)
  // Encode tile header-table loads before phase 1 (1), after it (0), by
  // LDS-DMA with the payload stream (2: full 16-packet tiles, aligned arrays),
  // or -1 = automatic: before for tiles of at most 16 KiB of payload (1M x 64 B
  // 0.0287 -> 0.0267 ms, x 256 B 0.0934 -> 0.0892, x 1024 B 0.3606 ->
  // 0.3557), by LDS-DMA above (x 1472 B 0.5126 -> 0.5086; round 1: after,
  // 0.5208 vs 0.5291 early).
  RUDP_KNOB(encode_early_table, -1)
  // Leaders build header chunks through a 48-B LDS scratch per packet
  // (constant shifts, one window per chunk) instead of variable-shift
  // funnels: 1, 0, or -1 = automatic (tiles of at most 16 KiB: 1M x 64 B
  // 0.0272 -> 0.0266 ms, x 256 B 0.0923 -> 0.0912; x 1472 B within noise;
  // profiles/r01/sweeps/encode_hc_scratch.json).
  RUDP_KNOB(encode_hc_scratch, -1)
  // Decode tile outputs staged in LDS and written as whole dwords (output
  // pointers 4-B aligned): 1M x 256 B verify 0.0489 -> 0.0470 ms, x 64 B
  // 0.0156 -> 0.0152, x 1472 B equal; copy-out equal to +1%
  // (profiles/r01/sweeps/decode_stage_out.json).
  RUDP_KNOB(decode_stage_out, 1)
  RUDP_KNOB(decode_blocks_per_cu, -1)  // decode tile: cap resident tiles per CU (0 = natural, -1 = auto)
  // Varlen encode tile: prebuilt header chunks and a one-window phase 2 for
  // tiles whose frames are all >= 32 B: 1M x 1472 B 0.738 -> 0.631 ms, x 1024
  // B 0.562 -> 0.477, x 256 B 0.196 -> 0.169 (Python entry, one box;
  // profiles/r01/sweeps/varlen_encode_hchunk.json).
  // 2 = the same with a coded u16 chunk map (owner frame + chunk class), so a
  // phase-2 chunk needs no frame-offset reads: 1M x 1472 B 0.581 -> 0.569 ms,
  // x 512 B 0.265 -> 0.256, x 256 B 0.165 -> 0.160, x 1024 B kept on the u8
  // map by the occupancy rule (profiles/r01/sweeps/varlen_coded_map.json).
  RUDP_KNOB(varlen_hchunk, 2)
  // Varlen decode tile: LDS budget in % of the hinted run.  110 lets six
  // 1472-B tiles share a CU (125 held five): 1M x 1479 B 0.288 -> 0.277 ms,
  // lengths uniform in [0, 2944] 0.315 -> 0.306 (overflowing tiles take the
  // per-frame path in the launch; profiles/r01/sweeps/varlen_decode_cap.json).
  RUDP_KNOB(varlen_decode_cap_pct, 110)
  // Varlen encode tile: LDS budget in % of the hinted run (110: 1M x 1472 B
  // 0.619 -> 0.586 ms, x 1024 B 0.468 -> 0.463, x 256 B 0.167 -> 0.164 vs
  // 125; profiles/r01/sweeps/varlen_encode_cap.json).
  RUDP_KNOB(varlen_encode_cap_pct, 110)
  RUDP_KNOB(varlen_decode_tile, 1)  // varlen decode through LDS tiles for hints >= 128 B (2: any hint; 0: never)
  RUDP_KNOB(dedup_table, 1)    // dedup window pass by LDS hash table (0: every frame scans its window)
  RUDP_KNOB(dedup_small, 1)  // packed small frames: dedup in one launch (dedup_small_kernel; 0: two passes)
  // Varlen decode tile frame sums from 128-B block sums taken in phase 1 (the
  // encode tile's scheme): lengths uniform in [0, 2944] 0.288 -> 0.278 ms, but
  // equal 1472-B lengths 0.246 -> 0.268 (the block sums' DPP work sits in the
  // streaming phase; profiles/r04/sweeps/varlen_decode_blocks.json).  1: per
  // tile, for tiles whose longest frame is over 1.25x their mean (every wave
  // reads the tile's lengths: uniform without a barrier): ragged 0.279 ->
  // 0.264 ms, but equal lengths 0.235 -> 0.252 (round 5,
  // profiles/r05/sweeps/varlen_decode_adaptive_blocks.json); 2: every tile;
  // 0: none (the product's form; 1 and 2 exist in the diagnostics build only).
  RUDP_KNOB(varlen_decode_blocks, 0)
  RUDP_KNOB(utf8_tile, 1)
  // Packed-frame UTF-8 validation through LDS tiles (hints >= 128 B) and its
  // LDS budget in % of the hinted run: 1M x 1479 B ASCII frames 0.287 ->
  // 0.279 ms, lengths uniform in [0, 2944] 0.373 -> 0.370 at 130% (110%:
  // more tiles overflow to the HBM path on ragged lengths; 150%: fewer tiles
  // per CU; round-1 tools/utf8_varlen_sweep.py (git history), profiles/r01/sweeps/utf8_varlen_tile.json).
  RUDP_KNOB(utf8_vtile, 1)
  RUDP_KNOB(utf8_vtile_cap_pct, 130)      // fixed-stride UTF-8 validation through LDS tiles (0: per-frame vector kernel)
  // Varlen tile kernels load the tile's frame offsets into registers before
  // phase 1 (1) instead of after its payload loads (0): decode 1M x 1479 B
  // 0.280 -> 0.265 ms, x 1031 B 0.222 -> 0.215; encode (Python entry) 1472 B
  // 0.583 -> 0.579, 1024 B 0.433 -> 0.428 (profiles/r01/sweeps/varlen_early_fo.json).
  RUDP_KNOB(varlen_early_fo, 1)
  // Varlen encode tile: minimum waves per SIMD imposed on its register
  // allocation (amdgpu_waves_per_eu: 6, 7, 8; 0 = none, 88 VGPRs = 5 waves;
  // -1 = automatic from the tile's LDS occupancy, see launch_varlen_tile).
  RUDP_KNOB(varlen_waves, -1)
  // Packed-frame UTF-8 tile: the most frames per tile whose LDS budget stays
  // within these bytes (0: lanes from chunks per lane).  A 34 KiB raw run
  // (T = 64 at 519 B) gave 0.164 -> 0.136 ms there but 0.228 -> 0.247 at
  // 1031 B (3 tiles per CU at the 130% budget; varlen_decode_lanes.json).
  RUDP_KNOB(utf8_vtile_bytes, 34816)
  RUDP_KNOB(varlen_scan, 1)    // frame offsets: 1 = reduce-then-scan (scan.hip), 0 = hipcub
  // Small-frame varlen encode (scan's last pass + framing in one tile kernel)
  // for packed batches whose mean payload hint is under this many bytes (0: off),
  // and its packets per thread (1, 2, 4, 8: tiles of 256 * fpt packets).
  RUDP_KNOB(varlen_small, 16)
  RUDP_KNOB(varlen_small_fpt, 0)  // 0: 4 for hints up to 4 B, 2 above (profiles/r02/sweeps/small.json)
  RUDP_KNOB(varlen_small_fused, 1)  // the framing kernel finds its own base (no pass-2 launch)
  RUDP_KNOB(varlen_small_single, 1)  // a checked call that is one small-frame tile: one launch, no pass 1
  // Small-frame encode: pass 1 leaves the lengths as 2-bit (4 packets a thread)
  // or 4-bit (2) codes for the framing kernel (1), which then reads 0.25-0.5 B
  // per packet instead of len[]'s 4 (0: len[]).
  RUDP_KNOB(varlen_small_nib, 1)
  // Checked varlen decode by byte spans: a workgroup decodes the frames that
  // start in one span of varlen_decode_span_bytes, its lanes over the bytes
  // (not over frames), after an index pass over the offsets (0: frame tiles).
  RUDP_KNOB(varlen_decode_span, 0)
  RUDP_KNOB(varlen_decode_span_bytes, 24576)
  // Varlen encode tile: the chunk -> frame map built by output units spread
  // evenly over the lanes (1) instead of G lanes per frame (0).
  RUDP_KNOB(varlen_map_bal, 0)
  // Varlen decode tile workgroup size: 256 (T = 256 / G frames) or 128.
  RUDP_KNOB(varlen_decode_nt, 256)
  // Varlen decode tile: a lane's payload chunks read four at a time (1) or
  // one at a time (0).
  RUDP_KNOB(varlen_decode_r4, 0)
  RUDP_KNOB(dedup_small_fpt, 4)  // one-launch dedup: frames per thread (4: 1024-frame tiles, 2: 512)
  // Fixed-length encode: batches of more packets than this go out as several
  // launches of at most this many (0: one launch).
  RUDP_KNOB(encode_launch_packets, 0)

  // Varlen encode tiles by payload bytes (spans from the scan) instead of by
  // packet count: no tile overflows short of one packet past the budget's
  // slack.  1: the scan chooses per call (byte tiles when over 1/32 of the
  // packet tiles would overflow) and writes the chosen form's tile records;
  // 2: byte tiles always; 3: packet tiles through records; 0: packet tiles
  // from frame_off (no records).  Round 2: packet 0.540 / byte 0.621 ms at 1M
  // x 1472 B, lengths uniform in [0, 2944] 0.728 / 0.644
  // (profiles/r02/sweeps/ragged_blocksums.json); round 3 (records instead of a
  // choice read by every tile): profiles/r03/sweeps/varlen_records.json.
  RUDP_KNOB(varlen_btile, 1)
  // Varlen tile sum pass from 128-B block sums (VarlenArgs::tile_sums 2): 1M x
  // 1472 B 0.544 -> 0.527 ms, lengths uniform in [0, 2944] 0.808 -> 0.729
  // (profiles/r02/sweeps/ragged_blocksums.json).
  RUDP_KNOB(varlen_tile_sums, 2)
  // Varlen byte tiles: span bytes S (0 = budget - 2 * hint - 64); sweeps only.
  RUDP_KNOB(varlen_span_bytes, 0)
#if RUDP_TOOLS
  // Varlen tile ablations (timing only, 1 = wrong output): 1 skip the edge
  // units; 2 byte tiles with tile_T slots.
  RUDP_KNOB(varlen_diag, 0)
#endif
  RUDP_KNOB(host_slots, 3)     // *_host pipeline: device staging slots (2..8)
  RUDP_KNOB(host_stage_mb, 128)  // *_host pipeline: MiB per slot (1M x 1472 B pinned: 33 ms at 128 vs 94 ms at 32)
  RUDP_KNOB(host_min_chunks, 4)  // *_host pipeline: batches over 4 MiB go as at least this many chunks (copy overlap)
  // *_host varlen decode: kernels store the per-frame outputs straight into the
  // caller's pinned arrays (1), or into the slot and D2H copies (0).
  RUDP_KNOB(host_direct_out, 1)
  // *_host varlen calls of small frames whose arrays are all pinned (and the
  // frame / payload buffers 16-B aligned): one launch that reads and writes
  // host memory over PCIe, no staging (1), or the slot pipeline (0).
  RUDP_KNOB(host_zero_copy, 1)

};
#undef RUDP_KNOB
#if RUDP_TOOLS
Tuning& tuning();
#else
inline const Tuning& tuning() {
  static constexpr Tuning t{};
  return t;
}
#endif

// Tile geometry for a fast-path payload length (L % 16 == 0, 16 <= L <= 4096).
void encode_tile_geometry(uint32_t L, uint32_t* T, uint32_t* glog);
uint32_t decode_group_log2(uint32_t L);

int launch_encode(const EncodeTileArgs& args, int layout, hipStream_t stream);
int launch_decode(const DecodeArgs& args, int layout, DecodePath path, hipStream_t stream);
int launch_synth(const SynthArgs& args, hipStream_t stream);
void varlen_tile_geometry(uint32_t len_hint, uint32_t* T, uint32_t* glog, uint32_t* cap);
bool varlen_btile_ok(uint32_t tile_T, uint32_t* bt_slots, uint32_t min_slots, uint32_t cap, uint32_t cap_packet,
                     uint32_t H, uint32_t vhc, uint64_t packet_tiles, uint64_t spans);
int launch_encode_varlen(const VarlenArgs& args, int layout, hipStream_t stream);
int launch_decode_varlen(const VarlenArgs& args, int layout, hipStream_t stream);
// The span decode's LDS (run budget `cap` plus its arrays) fits a workgroup.
bool decode_span_fits(uint64_t cap);
int launch_validate_utf8(const Utf8Args& args, hipStream_t stream);
int launch_dedup(const DedupArgs& args, hipStream_t stream);
uint32_t dedup_max_window();
// The one-launch dedup's LDS run budget for packed frames of this mean length
// and window, or 0 when the two-pass form is used.
uint32_t dedup_small_cap(uint32_t mean_len, uint32_t window);
// counts[side[i]] += (dup[i] == 1) for i < n (side null: all side 0), on `stream`.
int launch_dedup_count(const uint8_t* dup, const uint8_t* side, uint64_t n, uint64_t* counts, hipStream_t stream);
// Stream-ordered temporaries from a library-owned pool of the current device
// that keeps its memory across synchronizes (device_pool.hip).
hipError_t stream_alloc(void** ptr, size_t bytes, hipStream_t stream);
hipError_t stream_free(void* ptr, hipStream_t stream);
// A per-(device, stream, slot) temporary kept across calls (device_pool.hip),
// valid while the ScratchCall that covers the call is alive: every entry
// point that asks for scratch makes one on its stream before its first
// request and keeps it until its last kernel is enqueued.
enum ScratchSlot { kScratchSums = 0, kScratchRecords = 1, kScratchHash = 2, kScratchBounds = 3 };
class ScratchCall {
 public:
  explicit ScratchCall(hipStream_t stream);
  ~ScratchCall();
  ScratchCall(const ScratchCall&) = delete;
  ScratchCall& operator=(const ScratchCall&) = delete;

 private:
  friend hipError_t stream_scratch(void** ptr, size_t bytes, hipStream_t stream, int slot);
  static constexpr int kMaxFree = 4;
  hipStream_t stream_ = nullptr;
  int device_ = 0;
  bool outer_ = false;    // the outermost call on this thread (a nested one is a no-op)
  bool capture_ = false;  // the stream is being captured: temporaries live inside the graph
  void* set_ = nullptr;   // the (device, stream) scratch set this call holds
  void* free_[kMaxFree] = {};
  int nfree_ = 0;
};
hipError_t stream_scratch(void** ptr, size_t bytes, hipStream_t stream, int slot);
// Diagnostics (tools build): scratch sets held for a device, bytes in use in its pool.
size_t scratch_sets(int device);
hipError_t pool_used_bytes(int device, uint64_t* used);

struct Bounds {
  uint64_t min_len, max_len, sum_len;
  int64_t min_off, max_end;
  uint64_t n_decreasing;
};
// Bounds of len[] / payload_off[] (or, offsets_only, of frame_off[0..n]) on
// `stream`, copied to *host; synchronous (bounds.hip).
int compute_bounds(const uint32_t* len, const int64_t* off, uint64_t n, bool offsets_only,
                   Bounds* host, hipStream_t stream);
// Device-side validation folded into the offset scan (sync-free varlen
// encode).  status == null: no checks.
struct ScanCheck {
  const uint64_t* payload_off;  // gathered payloads, or null (packed)
  uint64_t payload_bytes;       // size of the payload buffer
  uint64_t frames_cap;          // capacity of the frame buffer
  uint32_t* status;             // written once: RUDP_ST_* bits, 0 = valid
};
// The scan's first two passes alone (scan.hip): block sums of len + H over
// blocks of kBlock * items packets (items 1, 2, 4 or 8; with the ScanCheck's
// bits), then the exclusive block bases in place, frame_off[n] and the status.
void scan_block_sums(const uint32_t* d_len, uint64_t n, uint32_t H, uint32_t items, uint64_t* sums,
                     const ScanCheck& chk, hipStream_t stream, uint32_t over_T = 0, uint32_t over_cap = 0,
                     uint8_t* codes = nullptr, uint32_t code_base = 0);
void scan_block_bases(uint64_t* sums, uint64_t nb, uint64_t* d_frame_off, uint64_t n, uint32_t H,
                      const ScanCheck& chk, hipStream_t stream, uint32_t* ctl = nullptr, uint32_t min_over = 0);
// Small-frame varlen encode of packed payloads (varlen.hip): the scan's first
// two passes, then one kernel per tile of kBlock * fpt packets that writes the
// tile's offsets and assembles its frames in LDS.
int launch_encode_varlen_small(const VarlenArgs& args, const ScanCheck& chk, int layout, hipStream_t stream);
// The same tile kernel for a fixed-stride batch (args.frame_off == null): every
// tile's base is known, so it is one launch and no scan (varlen.hip).
int launch_encode_stride_small(const VarlenArgs& args, int layout, hipStream_t stream);
// Payload copy-out of fixed-stride frames that miss the fixed-length decode
// tile (payloads not a multiple of 16 B, unaligned views): payload i =
// frames[i F + H, (i + 1) F) to out[i L, (i + 1) L), L = F - H (varlen.hip).
int launch_copy_payloads(const unsigned char* frames, uint32_t F, uint32_t H, uint64_t n, unsigned char* out,
                         hipStream_t stream);
// Span starts for the byte-tiled varlen encode: rec[k] (k = 0 .. count) holds
// p, the first packet whose packed payload starts at or after k * bytes, and
// fo = frame_off[p], so a tile has its packet range and frame run from two
// adjacent records in one round trip.
// With over set, the scan also counts into *over the tiles of tile_T packets
// whose payload run (16-B aligned) exceeds tile_cap.
// The varlen tile kernel's records (scan_apply_kernel): rec[0..grid] for
// grid = max(packet tiles, spans) workgroups.  Pass 1 counts the packet tiles
// of tile_T packets whose payload run (estimated as their length sum + 30)
// exceeds tile_cap; pass 2 writes *ctl = 1 (byte tiles) when the count is at
// least min_over, else 0; pass 3 writes the chosen form's records, the
// unused workgroups' records spread evenly as empty ones (rec_index).
struct SpanStarts {
  SpanRec* rec;  // [grid + 1], or null
  uint64_t bytes;      // span size S
  uint64_t count;      // spans: ceil over the payload bytes (+ 1)
  uint64_t ptiles;     // packet tiles
  uint64_t grid;       // max(ptiles, count)
  uint32_t* ctl;       // pass 2's choice
  uint32_t min_over;   // 0: byte tiles always; UINT32_MAX: packet tiles always
  uint32_t tile_T, tile_cap;
};
int scan_frame_offsets_3pass(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                             const ScanCheck& chk, hipStream_t stream, const SpanStarts& spans = SpanStarts{});
int scan_frame_offsets(const uint32_t* d_len, uint64_t n, uint32_t H, uint64_t* d_frame_off,
                       const ScanCheck& chk, hipStream_t stream, const SpanStarts& spans = SpanStarts{});
// frame_off[0..n] non-decreasing and inside [0, frames_bytes]: writes
// *d_status = 0 or RUDP_ST_OFFSETS, asynchronously (bounds.hip).
int check_frame_offsets(const uint64_t* d_frame_off, uint64_t n, uint64_t frames_bytes, uint32_t* d_status,
                        hipStream_t stream);

}  // namespace rudp
