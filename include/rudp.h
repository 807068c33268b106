/*
 * rudp.h — C ABI of librudp: batched Reliable-UDP wire codec on MI355X (gfx950).
 *
 * The reference (reotam5/Reliable-UDP) has no FFI: its boundary is the Python
 * class `Packet` in utils/packet.py:12-86 plus the module global
 * `custom_header` (utils/packet.py:3-10), imported by utils/reliableUDP.py:4
 * and proxy.py:10.  This header is the C boundary a maintainer binds (ctypes
 * stub in INTEGRATION.md) to move the per-packet work of that class onto the
 * GPU in batches.  Each entry point names the reference code it replaces.
 *
 * Wire format (utils/packet.py:3-10):
 *   byte 0-1  seq_num, big-endian u16
 *   byte 2-3  ack_num, big-endian u16
 *   byte 4    flags: bit7 SYN, bit6 ACK, bit5 FIN, bits4-0 `offset`
 *   RUDP_LAYOUT_RUDP7 only:
 *   byte 5-6  checksum, big-endian u16
 *   then the payload bytes.
 * Checksum (build-defined; the reference has none): RFC 1071 one's-complement
 * of the one's-complement sum of the frame taken as big-endian 16-bit words
 * with the checksum field (rudp7) zero and an odd tail zero-padded.  In the
 * rudp5 layout the frame carries no checksum field; the value is returned as
 * a sideband u16 per packet.
 *
 * Conventions
 *  - Buffers are caller-owned; the library never allocates or frees them.
 *  - Device (d_*) pointers are HIP device memory on `device`; calls are
 *    asynchronous on `hip_stream` (a hipStream_t, NULL = legacy default).
 *  - The *_host variants take host pointers and are synchronous.
 *  - Return 0 on success or a negative code (RUDP_E*); the message for the
 *    calling thread is available from rudp_last_error().
 *  - Reentrant and thread-safe: the only global state is mutex-guarded
 *    per-device caches (the *_host staging pipeline, the stream-ordered
 *    scratch pool, the call temporaries).  A call's device temporaries (scan
 *    sums, tile records, dedup hashes, offset-check partials) are kept per
 *    (device, stream), shared by all host threads: a call holds its stream's
 *    set while it enqueues (calls on one stream serialize on the host, as
 *    they do on the GPU) and the next call on that stream reuses it (stream
 *    order keeps them safe).  Nothing is held per host thread, so short-lived
 *    threads leave nothing behind; at most 64 streams per device keep a set.
 *    Once a device has 64, every call records an event behind its work as
 *    it ends, and a call on a 65th stream takes the least recently used set
 *    that has one, its own stream waiting for that event
 *    (hipStreamWaitEvent: stream order, no host wait, no device
 *    synchronize); with none, the call uses temporaries allocated and freed
 *    in stream order.  A temporary grown past 64 MiB is freed when its call
 *    ends.  Under stream capture the temporaries are allocated and freed
 *    inside the graph.  While another thread holds a GLOBAL-mode stream
 *    capture (hipStreamCaptureModeGlobal), the HIP runtime refuses
 *    stream-ordered allocations and cross-stream event waits made outside
 *    the capture: a call that needs either -- one on a stream without a set
 *    once the device has 64, or whose temporaries must grow -- fails with
 *    RUDP_EHIP_BASE - hipError and a message naming the capture, having
 *    enqueued nothing; the capture is unaffected, and the call succeeds if
 *    repeated after the capture ends.  Calls on streams that already hold
 *    a large-enough set, and captures in thread-local or relaxed mode, are
 *    not affected.
 *    Every launch choice is fixed at its
 *    measured default; librudp.so exports exactly the functions below.  (The
 *    diagnostics build of the same sources, librudp_tools.so, adds non-ABI
 *    rudpx_* sweep knobs and timelines for tools/ and is not a product library.)
 */
#ifndef RUDP_H_
#define RUDP_H_

#include <stdint.h>

/* Every entry point is exported; librudp is built with hidden default
 * visibility, so nothing else of it (kernels' host stubs, internal C++) can
 * interpose on another library's symbols or be interposed on. */
#if defined(__GNUC__)
#define RUDP_API __attribute__((visibility("default")))
#else
#define RUDP_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define RUDP_ABI_VERSION 7

/* Frame layouts: the value is the header length in bytes. */
#define RUDP_LAYOUT_RUDP5 5 /* reference-exact 5-byte header, checksum sideband */
#define RUDP_LAYOUT_RUDP7 7 /* {**custom_header, "checksum": 2}, checksum in-band */

/* Per-packet decode status written to d_ok. */
#define RUDP_OK_BAD_CSUM 0   /* checksum mismatch */
#define RUDP_OK_GOOD 1       /* checksum verified */
#define RUDP_OK_SHORT 2      /* frame shorter than the header */
#define RUDP_OK_UNVERIFIED 3 /* rudp5 decoded without a sideband checksum */
#define RUDP_OK_BAD_OFFSETS 4 /* variable-length decode: frame_off[i] > frame_off[i+1] or past the buffer */

/*
 * Status word of the sync-free variable-length calls (*_checked): written on
 * the device by the call itself, 0 when the batch is valid, else these bits.
 * Encode rejects the whole batch: with a non-zero status it writes no frames
 * and no checksums, and of d_frame_off only d_frame_off[n] (the total its scan
 * found); d_frame_off[0..n-1] are then unspecified.  Decode rejects frame by
 * frame: every frame whose pair of offsets is bad gets d_ok =
 * RUDP_OK_BAD_OFFSETS and nothing of it is read, every other frame is fully
 * decoded, and RUDP_ST_OFFSETS is set when any frame was rejected.
 */
#define RUDP_ST_LEN 1u        /* a len[i] > 65535 */
#define RUDP_ST_PAYLOAD 2u    /* packed: sum(len) != payload_bytes; gathered: payload outside the buffer */
#define RUDP_ST_FRAMES_CAP 4u /* sum(len) + n*layout > frames_cap */
#define RUDP_ST_OFFSETS 8u    /* frame_off decreasing, or outside [0, frames_bytes] */

/* Error codes (negative errno values, HIP errors offset by -1000). */
#define RUDP_EINVAL (-22)
#define RUDP_ENOMEM (-12)
#define RUDP_ENOTSUP (-95)
#define RUDP_EHIP_BASE (-1000) /* returned as RUDP_EHIP_BASE - hipError_t */

/*
 * A batch of packets to frame: the SoA header table plus payload bytes.
 * Fixed-length batches (rudp_encode): payload is n*payload_len contiguous
 * bytes and len/payload_off are NULL.  Variable-length batches
 * (rudp_encode_varlen): len[i] payload bytes of packet i (<= 65535) start at
 * payload[payload_off[i]], or, with payload_off NULL, the payloads are packed
 * back to back in packet order; payload_len is then a hint of the typical
 * payload length (0 = unknown/tiny) that picks lanes per packet, never the
 * result.
 *   seq   -> custom_header["seq_num"]  (utils/packet.py:4)
 *   ack   -> custom_header["ack_num"]  (utils/packet.py:5)
 *   flags -> header byte 4 verbatim: syn/ack/fin/offset (utils/packet.py:6-9)
 */
typedef struct rudp_batch {
  uint64_t n;
  uint32_t payload_len;
  uint32_t reserved;
  const uint16_t* seq;
  const uint16_t* ack;
  const uint8_t* flags;
  const uint8_t* payload;
  const uint32_t* len;          /* variable-length batches: payload bytes per packet */
  const uint64_t* payload_off;  /* variable-length batches: payload start, or NULL = packed */
} rudp_batch;

/*
 * Frame + checksum a device-resident batch.
 * Replaces, per packet, the encode sequence of utils/reliableUDP.py:53-61
 * (Packet(); set_header_field x2..4; set_payload; to_byte) i.e.
 * utils/packet.py:13-16, :43-57, :60-65, :76-81.
 * d_frames: n*(payload_len+layout) bytes.  d_csum_or_null: n u16 (rudp5
 * sideband; for rudp7 it receives a copy of the in-band value).
 * The fixed-length tile takes payload_len % 16 == 0, payload_len <= 4096
 * and 16-byte aligned d_frames and payload; any other shape (the reference's
 * 1-4 B datagrams, any length, unaligned views) runs the variable-length tile
 * kernels with implicit offsets (one launch, no offset array) with identical
 * results.  An unaligned buffer is read from the 16-byte boundary at or below
 * its first byte to the one at or above its last (the same aligned 16-byte
 * blocks, hence pages); nothing outside d_frames / d_csum is written.
 */
RUDP_API int rudp_encode(const rudp_batch* in, uint8_t* d_frames, uint16_t* d_csum_or_null,
                int layout, int device, void* hip_stream);

/*
 * Parse + verify a device-resident batch of fixed-length frames.
 * Replaces, per packet, utils/reliableUDP.py:118-123 / :67-73
 * (Packet(data); get_header_field x N; get_payload), i.e.
 * utils/packet.py:16, :29-40, :68-73.
 * Fixed-length frames: d_frame_off_or_null = NULL, frames at stride
 * frame_len.  Variable-length frames: d_frame_off_or_null = n+1 offsets
 * (frame i = d_frames[off[i], off[i+1]), as rudp_encode_varlen writes them),
 * frame_len is a hint of the typical frame length (0 = unknown/tiny; it
 * picks lanes per frame, never the result) and the payload is zero-copy only
 * (d_payload_out_or_null must be NULL).  d_csum_in_or_null: rudp5 sideband checksums to verify
 * (NULL: d_ok = RUDP_OK_UNVERIFIED).  d_csum_out_or_null: the recomputed
 * checksum per packet.  d_payload_out_or_null: n*(frame_len-layout) bytes,
 * payloads copied out aligned; NULL = zero-copy (view at frame offset layout).
 * Frames shorter than the header get d_ok = RUDP_OK_SHORT and the fields
 * that are present (truncated as utils/packet.py:31 slices them), 0 otherwise.
 * Fixed-length frames whose payload is not a multiple of 16 bytes, or whose
 * buffers are not 16-byte aligned, decode through the variable-length tiles
 * with implicit offsets (a payload copy-out is one more launch), with the
 * same results; buffers are read as rudp_encode reads them.
 */
RUDP_API int rudp_decode(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null,
                uint32_t frame_len, uint64_t n, const uint16_t* d_csum_in_or_null,
                uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_ok,
                uint16_t* d_csum_out_or_null, uint8_t* d_payload_out_or_null,
                int layout, int device, void* hip_stream);

/*
 * Frame + checksum a device-resident VARIABLE-LENGTH batch (in->len set).
 * The reference's own traffic: one UTF-8 character per datagram, 5-9 byte
 * frames (utils/reliableUDP.py:11, :53-61).  d_frame_off receives n+1
 * offsets, the exclusive scan of len[i] + layout (d_frame_off[n] = total
 * bytes); d_frames must hold sum(len) + n*layout bytes.  The concatenated
 * frames equal N calls of Packet(...).to_byte() back to back.
 */
RUDP_API int rudp_encode_varlen(const rudp_batch* in, uint8_t* d_frames, uint64_t* d_frame_off,
                       uint16_t* d_csum_or_null, int layout, int device, void* hip_stream);

/*
 * Sync-free forms of the two variable-length calls: the argument checks of
 * rudp_varlen_bounds / rudp_frame_off_bounds run on the device inside the call
 * (folded into the offset scan for encode; inside the decode kernels, where
 * every frame checks its own pair of offsets and a rejected frame gets
 * d_ok = RUDP_OK_BAD_OFFSETS) and land in *d_status (RUDP_ST_*), so the host
 * never waits.  The
 * caller reads d_status whenever it next synchronizes (the Python layer:
 * VarlenFrames.check() / DecodedBatch.check()).
 * rudp_encode_varlen_checked: payload_bytes = size of in->payload; frames_cap =
 *   capacity of d_frames.  Packed payloads (payload_off NULL) must satisfy
 *   sum(len) == payload_bytes; gathered ones payload_off[i] + len[i] <=
 *   payload_bytes.  d_frame_off[n] is always written; d_frame_off[0..n-1]
 *   when the batch is valid (status 0).
 * rudp_decode_varlen_checked: rudp_decode with offsets (zero-copy payload);
 *   frame_off[0..n] must be non-decreasing and <= frames_bytes.  d_status may
 *   be NULL (ABI 5): the call is then its one decode kernel, and the rejected
 *   frames are exactly those with d_ok == RUDP_OK_BAD_OFFSETS; with a status
 *   word the call zeroes it first (one more stream operation).
 * rudp_frame_off_check: only the offset check, for callers that run their own
 *   kernels on the frames afterwards.
 */
RUDP_API int rudp_encode_varlen_checked(const rudp_batch* in, uint64_t payload_bytes, uint8_t* d_frames,
                               uint64_t frames_cap, uint64_t* d_frame_off, uint16_t* d_csum_or_null,
                               uint32_t* d_status, int layout, int device, void* hip_stream);
RUDP_API int rudp_decode_varlen_checked(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                               uint32_t len_hint, uint64_t n, const uint16_t* d_csum_in_or_null,
                               uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_ok,
                               uint16_t* d_csum_out_or_null, uint32_t* d_status, int layout, int device,
                               void* hip_stream);
RUDP_API int rudp_frame_off_check(const uint64_t* d_frame_off, uint64_t n, uint64_t frames_bytes, uint32_t* d_status,
                         int device, void* hip_stream);

/*
 * Decode and strict-UTF-8 check in one pass (ABI 6): the reference's receive
 * parses every datagram AND decodes its payload (utils/reliableUDP.py:118-123:
 * Packet(data) -> get_header_field ... -> get_payload, whose strict
 * bytes.decode() is utils/packet.py:73).  As rudp_decode /
 * rudp_decode_varlen_checked, plus d_valid_or_null: d_valid[i] = 1 when
 * Packet(frame).get_payload() would return (an empty payload or a frame
 * shorter than the header: None), 0 when it would raise UnicodeDecodeError
 * -- rudp_validate_utf8's answer -- and 0 for a frame rejected for bad
 * offsets (nothing of it is read).  The LDS-tile decode kernels (fixed-length
 * frames whose 256/G-frame tile fits 64 KiB; packed frames of every hint)
 * judge each payload from the bytes they already hold, so every frame leaves
 * HBM once; other fixed-length shapes run the validation kernel after the
 * decode.  d_valid_or_null NULL: exactly rudp_decode / rudp_decode_varlen_checked.
 */
RUDP_API int rudp_decode_utf8(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null, uint32_t frame_len,
                     uint64_t n, const uint16_t* d_csum_in_or_null, uint16_t* d_seq, uint16_t* d_ack,
                     uint8_t* d_flags, uint8_t* d_ok, uint16_t* d_csum_out_or_null,
                     uint8_t* d_payload_out_or_null, uint8_t* d_valid_or_null, int layout, int device,
                     void* hip_stream);
RUDP_API int rudp_decode_varlen_utf8(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                            uint32_t len_hint, uint64_t n, const uint16_t* d_csum_in_or_null,
                            uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags, uint8_t* d_ok,
                            uint16_t* d_csum_out_or_null, uint8_t* d_valid_or_null, uint32_t* d_status,
                            int layout, int device, void* hip_stream);

/*
 * Bounds of a variable-length batch, computed on the device (argument checks
 * the varlen entry points need before they can size or trust a buffer; the
 * reference has no batch and so no counterpart).  Synchronous on hip_stream.
 * rudp_varlen_bounds: h_out[0..4] = min len, max len, sum of len, min
 * payload_off, max(payload_off + len); without offsets [3] = 0, [4] = sum.
 * len[] is read as u32 (a negative int32 length shows as > 65535).
 * rudp_frame_off_bounds: over d_frame_off[0..n], h_out[0..2] = min, max and
 * the number of i < n with d_frame_off[i+1] < d_frame_off[i] (0 = valid
 * offsets for rudp_decode; min and max are then the first and last).
 */
RUDP_API int rudp_varlen_bounds(const uint32_t* d_len, const int64_t* d_payload_off_or_null, uint64_t n,
                       int64_t* h_out, int device, void* hip_stream);
RUDP_API int rudp_frame_off_bounds(const int64_t* d_frame_off, uint64_t n, int64_t* h_out, int device,
                          void* hip_stream);

/*
 * Strict UTF-8 check of each frame's payload: d_valid[i] = 1 when
 * Packet(frame).get_payload() would return (utils/packet.py:68-73: empty
 * payload -> None; else bytes.decode(), strict UTF-8), 0 when it would raise
 * UnicodeDecodeError.  Frames as in rudp_decode (fixed stride or offsets;
 * with offsets frame_len is a typical-length hint, as there).
 */
RUDP_API int rudp_validate_utf8(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null,
                       uint32_t frame_len, uint64_t n, int layout, uint8_t* d_valid, int device,
                       void* hip_stream);

/*
 * Retransmission detection of the reference proxy (proxy.py:90: `packet in
 * self.packets`, a list of the last Proxy.MAX_MEMORY = 500 packets,
 * proxy.py:17, :92-94) over a batch of frames in arrival order:
 * d_dup[i] = 1 iff frame i equals (Packet.__eq__, utils/packet.py:83-86: same
 * get_hex(), so an empty datagram equals 00 00 00 00 00) one of frames
 * max(0, i - window) .. i-1.  window <= 4096 (the proxy uses 500).  To carry
 * history across batches, prepend the previous batch's last `window` frames.
 * Frames as in rudp_decode (fixed stride or n+1 offsets; with offsets
 * frame_len is a typical-length hint that picks lanes per frame).
 */
RUDP_API int rudp_dedup_window(const uint8_t* d_frames, const uint64_t* d_frame_off_or_null,
                      uint32_t frame_len, uint64_t n, uint32_t window, uint8_t* d_dup, int device,
                      void* hip_stream);

/*
 * rudp_dedup_window over packed frames with the argument check on the device
 * (ABI 5; the sync-free form the Python layer uses): every frame checks its
 * own pair of offsets against [0, frames_bytes]; a frame whose offsets are
 * decreasing or past the buffer gets d_dup = RUDP_DUP_BAD_OFFSETS, none of its
 * bytes is read, and it equals no other frame.  len_hint: the mean frame
 * length (picks lanes per frame, never the result).
 */
#define RUDP_DUP_BAD_OFFSETS 2
RUDP_API int rudp_dedup_window_checked(const uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_frame_off,
                              uint32_t len_hint, uint64_t n, uint32_t window, uint8_t* d_dup, int device,
                              void* hip_stream);

/*
 * The proxy's retransmission count over a datagram stream (ABI 6; proxy.py:79-94:
 * every datagram is checked against the last Proxy.MAX_MEMORY = 500 of both
 * directions, proxy.py:17, :90-94, and counted per side).  The history stays
 * on the device between batches and nothing here waits for the GPU:
 * rudp_dedup_stream_push copies a batch of host frames (packed, n + 1
 * offsets; any host memory, the caller may reuse it once the call returns)
 * behind the history, flags it with rudp_dedup_window_checked's rule, adds
 * the flags to per-side counters (h_side_or_null[i] = 0 or 1; NULL: all 0),
 * optionally copies the batch's flags to d_dup_or_null (n bytes, device), and
 * keeps the last `window` datagrams, all on the stream given at creation.
 * rudp_dedup_stream_counts synchronizes and returns the two counters.
 * window <= 4096; a batch holds at most max_batch datagrams of at most
 * max_frame bytes each.  Thread-safe: push and counts may come from different
 * threads (a relay thread pushing, another reading its counters); the object
 * serializes them.  destroy must be the object's last call.
 */
typedef struct rudp_dedup_stream rudp_dedup_stream;
RUDP_API int rudp_dedup_stream_create(uint32_t window, uint32_t max_batch, uint32_t max_frame, int device,
                                      void* hip_stream, rudp_dedup_stream** out);
RUDP_API int rudp_dedup_stream_push(rudp_dedup_stream* st, const uint8_t* h_frames, const uint64_t* h_frame_off,
                                    uint64_t n, const uint8_t* h_side_or_null, uint8_t* d_dup_or_null);
RUDP_API int rudp_dedup_stream_counts(rudp_dedup_stream* st, uint64_t* h_counts);
RUDP_API int rudp_dedup_stream_destroy(rudp_dedup_stream* st);

/*
 * Batched UDP socket I/O (host only, no device work): the reference moves one
 * datagram per system call (sendto, utils/reliableUDP.py:61; recvfrom(1024),
 * :67, :118; proxy.py:129).  These move up to 1024 per call (sendmmsg /
 * recvmmsg) between a socket and caller-owned host buffers, in the packed
 * frames + offsets layout of rudp_encode_varlen / variable-length rudp_decode.
 *
 * rudp_udp_recv_batch: waits up to timeout_ms (-1 forever, 0 not at all) for
 * a first datagram, then drains up to min(max_msgs, cap_bytes / slot_bytes)
 * without blocking.  A datagram longer than slot_bytes is truncated (as the
 * reference's recvfrom(1024) truncates).  Frames are packed from h_frames[0];
 * h_frame_off receives count+1 offsets.  Returns the count (0 on timeout) or
 * a negative errno.
 * rudp_udp_send_batch: sends frames [h_frame_off[i], h_frame_off[i+1]) for
 * i < n to ip:port.  Returns the count sent or a negative errno.
 */
RUDP_API int rudp_udp_recv_batch(int fd, uint8_t* h_frames, uint64_t cap_bytes, uint32_t slot_bytes,
                        uint32_t max_msgs, uint64_t* h_frame_off, int timeout_ms);
RUDP_API int rudp_udp_send_batch(int fd, const uint8_t* h_frames, const uint64_t* h_frame_off, uint64_t n,
                        const char* ip, uint16_t port);

/*
 * The same for a relay in the reference proxy's role, which forwards every
 * datagram by its source address (proxy.py:129-145) over one socket.  An
 * IPv4 endpoint travels as one integer: address (host byte order) << 16 | port.
 * rudp_udp_recv_batch_from: as rudp_udp_recv_batch, and h_src_or_null[i]
 *   receives datagram i's source (0 for a non-IPv4 source).
 * rudp_udp_send_batch_to: sends frame i to h_dst[i] (per_datagram != 0) or
 *   every frame to h_dst[0].  Returns the count sent or a negative errno.
 */
RUDP_API int rudp_udp_recv_batch_from(int fd, uint8_t* h_frames, uint64_t cap_bytes, uint32_t slot_bytes,
                             uint32_t max_msgs, uint64_t* h_frame_off, uint64_t* h_src_or_null,
                             int timeout_ms);
RUDP_API int rudp_udp_send_batch_to(int fd, const uint8_t* h_frames, const uint64_t* h_frame_off, uint64_t n,
                           const uint64_t* h_dst, int per_datagram);

/*
 * Host-memory conveniences: same semantics, host pointers in and out.
 * Staged through a ring of device slots in chunks, with H2D, kernel and D2H
 * on three streams chained by events so the three overlap.  Synchronous.  These model the reference's
 * real boundary, a UDP socket buffer in host memory (utils/reliableUDP.py:61,
 * :67, :118).  Pinned (page-locked) host buffers copy at the link's rate;
 * pageable ones through the runtime's bounce buffers, at about half of it.
 *
 * rudp_decode_host (ABI 7: h_valid_or_null added): rudp_decode_utf8 of
 *   fixed-length frames in host memory -- the reference's receive, Packet(data)
 *   + get_header_field + get_payload() per datagram (utils/reliableUDP.py:118-121,
 *   utils/packet.py:16, :29-40, :68-73) -- with h_valid_or_null[i] its strict
 *   UTF-8 answer, judged in the decode pass (NULL: not computed).
 * rudp_decode_varlen_host (ABI 7): rudp_decode_varlen_utf8 of packed frames
 *   in host memory (a recvmmsg batch: frame i = h_frames[h_frame_off[i],
 *   h_frame_off[i + 1]), frames_bytes = size of h_frames), with every frame's
 *   offsets checked against frames_bytes as there (a rejected frame gets
 *   h_ok = RUDP_OK_BAD_OFFSETS and h_valid = 0, and *h_status_or_null =
 *   RUDP_ST_OFFSETS); the payload is zero-copy (frame i's bytes from
 *   layout on).  len_hint: the typical frame length (0: frames_bytes / n).
 *   Each chunk stages the byte range its offsets span: one valid frame over
 *   host_stage bytes (128 MiB) is refused with RUDP_ENOTSUP.
 * rudp_encode_varlen_host (ABI 7): rudp_encode_varlen of packed payloads in
 *   host memory (h_in->payload_off must be NULL; h_in->payload_len is a hint
 *   of the typical length) to packed frames in host memory -- the send side,
 *   Packet() + set_header_field + set_payload + to_byte() per datagram
 *   (utils/reliableUDP.py:53-61, utils/packet.py:43-65, :76-81).
 *   h_frame_off receives n + 1 offsets (the exclusive scan of len[i] +
 *   layout).  Every length (<= 65535), sum(len) == payload_bytes (the size
 *   of h_in->payload) and frames_cap (>= sum(len) + n * layout) are checked
 *   before any frame byte is written: a bad batch returns RUDP_EINVAL and
 *   h_frames and h_csum_or_null are untouched.  The host checks the lengths
 *   before it enqueues any work, except for a batch of small frames (mean
 *   payload under 16 B) whose every array is pinned: that one runs as one
 *   checked device encode over PCIe, whose first pass makes the same checks
 *   (h_frame_off is then left unspecified on a bad batch).
 */
RUDP_API int rudp_encode_host(const rudp_batch* h_in, uint8_t* h_frames, uint16_t* h_csum_or_null,
                     int layout, int device);
RUDP_API int rudp_decode_host(const uint8_t* h_frames, uint32_t frame_len, uint64_t n,
                     const uint16_t* h_csum_in_or_null, uint16_t* h_seq, uint16_t* h_ack,
                     uint8_t* h_flags, uint8_t* h_ok, uint16_t* h_csum_out_or_null,
                     uint8_t* h_payload_out_or_null, uint8_t* h_valid_or_null, int layout, int device);
RUDP_API int rudp_decode_varlen_host(const uint8_t* h_frames, uint64_t frames_bytes, const uint64_t* h_frame_off,
                                     uint32_t len_hint, uint64_t n, const uint16_t* h_csum_in_or_null,
                                     uint16_t* h_seq, uint16_t* h_ack, uint8_t* h_flags, uint8_t* h_ok,
                                     uint16_t* h_csum_out_or_null, uint8_t* h_valid_or_null,
                                     uint32_t* h_status_or_null, int layout, int device);
RUDP_API int rudp_encode_varlen_host(const rudp_batch* h_in, uint64_t payload_bytes, uint8_t* h_frames,
                                     uint64_t frames_cap, uint64_t* h_frame_off, uint16_t* h_csum_or_null,
                                     int layout, int device);

/*
 * Deterministic synthetic batch, generated on the device:
 * packet i (global index first_index + local index) gets
 *   seq = (isn + i) mod 2^16, isn in [1, 5000]   (utils/reliableUDP.py:41, :54)
 *   ack = splitmix u16, flags uniform over {00,80,20,A0,40,60}
 *   payload bytes from splitmix64, masked to 0x00-0x7F when ascii != 0.
 * The same definition is restated on the CPU in oracle/synth.py.
 */
RUDP_API int rudp_synth(uint64_t seed, uint64_t first_index, uint64_t n, uint32_t payload_len,
               int ascii, uint16_t* d_seq, uint16_t* d_ack, uint8_t* d_flags,
               uint8_t* d_payload, int device, void* hip_stream);

RUDP_API int rudp_device_count(int* count);
RUDP_API const char* rudp_last_error(void);
RUDP_API int rudp_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RUDP_H_ */
