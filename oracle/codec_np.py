"""ORACLE (test infrastructure): numpy restatement of the batch codec.

Framing follows the reference wire format (utils/packet.py:3-10: seq_num u16
BE, ack_num u16 BE, one byte of syn/ack/fin/offset bits, then the payload,
:60-65 / :80-81), with the rudp7 layout inserting the build-defined checksum
field at bytes 5-6 ({**custom_header, "checksum": 2}).

The checksum is computed here straight from its definition — RFC 1071 over
the frame as big-endian 16-bit words, checksum field zero, odd tail padded
with a zero byte — not from the little-endian shortcut the HIP kernels use,
so this is an independent check of that shortcut.
"""
from __future__ import annotations

import numpy as np

CHUNK = 1 << 16  # packets per vectorised step (bounds temporary memory)


def inet_checksum(data: bytes) -> int:
    """RFC 1071 Internet checksum of a byte string (generic restatement)."""
    if len(data) % 2:
        data = bytes(data) + b"\x00"
    words = np.frombuffer(bytes(data), dtype=">u2").astype(np.uint64)
    s = int(words.sum())
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def _fold(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    for _ in range(4):
        s = (s & np.uint64(0xFFFF)) + (s >> np.uint64(16))
    return s


def frame_checksums(frames: np.ndarray, layout: int) -> np.ndarray:
    """Checksum of each frame row with its checksum field (rudp7) taken as zero."""
    n, F = frames.shape
    out = np.empty(n, dtype=np.uint16)
    for a in range(0, n, CHUNK):
        blk = frames[a:a + CHUNK]
        if layout == 7 and F >= 7:
            blk = blk.copy()
            blk[:, 5:7] = 0
        if F % 2:
            blk = np.concatenate([blk, np.zeros((blk.shape[0], 1), np.uint8)], axis=1)
        words = np.ascontiguousarray(blk).view(">u2")
        s = words.astype(np.uint64).sum(axis=1)
        out[a:a + CHUNK] = (~_fold(s)) & np.uint64(0xFFFF)
    return out


def encode(seq, ack, flags, payload, layout: int):
    """frames u8[n, L+layout] and checksum u16[n] for a fixed-length batch."""
    payload = np.asarray(payload, dtype=np.uint8)
    n, L = payload.shape
    H = layout
    seq = np.asarray(seq, dtype=np.uint16)
    ack = np.asarray(ack, dtype=np.uint16)
    frames = np.zeros((n, L + H), dtype=np.uint8)
    frames[:, 0] = seq >> 8
    frames[:, 1] = seq & 0xFF
    frames[:, 2] = ack >> 8
    frames[:, 3] = ack & 0xFF
    frames[:, 4] = np.asarray(flags, dtype=np.uint8)
    frames[:, H:] = payload
    csum = frame_checksums(frames, layout)
    if H == 7:
        frames[:, 5] = csum >> 8
        frames[:, 6] = csum & 0xFF
    return frames, csum


def decode(frames, layout: int, csum_in=None):
    """(seq, ack, flags, ok, csum, payload_view) with the ok codes of include/rudp.h."""
    frames = np.asarray(frames, dtype=np.uint8)
    n, F = frames.shape
    H = layout
    b = np.zeros((n, 7), dtype=np.uint16)
    b[:, :min(F, 7)] = frames[:, :min(F, 7)]
    if F >= H:
        seq = (b[:, 0] << 8) | b[:, 1]
        ack = (b[:, 2] << 8) | b[:, 3]
        flags = b[:, 4].astype(np.uint8)
        csum = frame_checksums(frames, layout)
        if H == 7:
            ok = (csum == ((b[:, 5] << 8) | b[:, 6])).astype(np.uint8)
        elif csum_in is not None:
            ok = (csum == np.asarray(csum_in, dtype=np.uint16)).astype(np.uint8)
        else:
            ok = np.full(n, 3, np.uint8)
        return seq.astype(np.uint16), ack.astype(np.uint16), flags, ok, csum, frames[:, H:]
    # short frames: fields truncated like a short bit-string slice (utils/packet.py:31)
    seq = (b[:, 0] << 8) | b[:, 1] if F >= 2 else b[:, 0]
    ack = (b[:, 2] << 8) | b[:, 3] if F >= 4 else b[:, 2]
    return (seq.astype(np.uint16), ack.astype(np.uint16), b[:, 4].astype(np.uint8),
            np.full(n, 2, np.uint8), np.zeros(n, np.uint16), frames[:, :0])


def encode_varlen(seq, ack, flags, payloads, layout: int):
    """Frames for a list of payload byte strings, back to back, plus n+1 offsets."""
    seq = np.asarray(seq, dtype=np.uint16)
    ack = np.asarray(ack, dtype=np.uint16)
    flags = np.asarray(flags, dtype=np.uint8)
    out, off, cs = bytearray(), [0], []
    for i, p in enumerate(payloads):
        fr, c = encode(seq[i:i + 1], ack[i:i + 1], flags[i:i + 1],
                       np.frombuffer(bytes(p), np.uint8).reshape(1, len(p)), layout)
        out += fr.tobytes()
        off.append(len(out))
        cs.append(int(c[0]))
    return (np.frombuffer(bytes(out), np.uint8), np.array(off, np.int64),
            np.array(cs, np.uint16))


def decode_varlen(frames, frame_off, layout: int, csum_in=None):
    """(seq, ack, flags, ok, csum) for frames packed back to back."""
    frames = np.asarray(frames, dtype=np.uint8)
    n = len(frame_off) - 1
    res = [np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8),
           np.zeros(n, np.uint8), np.zeros(n, np.uint16)]
    for i in range(n):
        fr = frames[frame_off[i]:frame_off[i + 1]].reshape(1, -1)
        ci = None if csum_in is None else np.asarray(csum_in)[i:i + 1]
        out = decode(fr, layout, ci)
        for k in range(5):
            res[k][i] = out[k][0]
    return tuple(res)


def utf8_valid(frames, frame_off, layout: int):
    """1 where Python's strict bytes.decode() accepts the payload (utils/packet.py:73)."""
    n = len(frame_off) - 1
    out = np.zeros(n, np.uint8)
    for i in range(n):
        body = bytes(frames[frame_off[i] + layout:frame_off[i + 1]]) \
            if frame_off[i + 1] - frame_off[i] > layout else b""
        try:
            body.decode()
            out[i] = 1
        except UnicodeDecodeError:
            out[i] = 0
    return out
