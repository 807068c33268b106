"""Batched UDP socket I/O at the codec's host boundary.

The reference does one system call per datagram: sendto (utils/
reliableUDP.py:61) and recvfrom(1024) (:67, :118; proxy.py:129).  Here up to
1024 datagrams move per call (recvmmsg / sendmmsg in librudp.so) directly
into / out of pinned host buffers, in the packed-frames + offsets layout the
variable-length GPU codec consumes and produces:

    rx = BatchReceiver(sock, max_msgs=65536)
    n = rx.recv(timeout_ms=100)              # socket -> pinned ring
    dec = rx.decode("rudp5", device)         # pinned ring -> HBM -> unpack_batch_varlen

    send_batch(sock, frames, frame_off, ip, port)   # pack_batch_varlen output -> wire
"""
from __future__ import annotations

import ctypes
import socket as _socket

import numpy as np

from . import _native
from . import batch as _batch


def _np_ptr(a) -> int:
    return a.ctypes.data


def addr_key(ip: str, port: int) -> int:
    """An IPv4 endpoint as the one integer the batched socket calls use:
    address (host byte order) << 16 | port."""
    return int.from_bytes(_socket.inet_aton(ip), "big") << 16 | port


def key_addr(key: int):
    """(ip, port) of an ``addr_key``."""
    return _socket.inet_ntoa(int(key >> 16).to_bytes(4, "big")), int(key & 0xFFFF)


def recv_batch(sock: _socket.socket, frames: np.ndarray, frame_off: np.ndarray, *,
               slot_bytes: int = 1024, max_msgs: int | None = None, timeout_ms: int = -1,
               sources: np.ndarray | None = None) -> int:
    """Receive up to ``max_msgs`` datagrams into ``frames`` (u8, packed) and
    ``frame_off`` (int64, count + 1).  Datagrams longer than ``slot_bytes`` are
    truncated, as recvfrom(1024) truncates in the reference.  ``sources``
    (u64, optional) receives each datagram's source as an ``addr_key``.
    Returns the count (0 on timeout)."""
    if frames.dtype != np.uint8 or frames.ndim != 1 or not frames.flags["C_CONTIGUOUS"]:
        raise TypeError("frames must be a contiguous 1-D uint8 array")
    if frame_off.dtype != np.int64 or frame_off.ndim != 1 or not frame_off.flags["C_CONTIGUOUS"]:
        raise TypeError("frame_off must be a contiguous 1-D int64 array")
    cap_msgs = frame_off.shape[0] - 1
    max_msgs = cap_msgs if max_msgs is None else min(max_msgs, cap_msgs)
    if max_msgs < 0:
        raise ValueError("frame_off needs at least one entry")
    src_ptr = None
    if sources is not None:
        if sources.dtype != np.uint64 or sources.ndim != 1 or not sources.flags["C_CONTIGUOUS"]:
            raise TypeError("sources must be a contiguous 1-D uint64 array")
        max_msgs = min(max_msgs, sources.shape[0])
        src_ptr = _np_ptr(sources)
    rc = _native.lib().rudp_udp_recv_batch_from(sock.fileno(), _np_ptr(frames), frames.nbytes,
                                                slot_bytes, max_msgs, _np_ptr(frame_off), src_ptr,
                                                timeout_ms)
    if rc < 0:
        raise OSError(-rc, f"recvmmsg: {rc}")
    return rc


def send_batch(sock: _socket.socket, frames: np.ndarray, frame_off: np.ndarray, ip: str,
               port: int) -> int:
    """Send frames [frame_off[i], frame_off[i+1]) to ip:port; returns the count sent."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    frame_off = np.ascontiguousarray(frame_off, dtype=np.int64)
    n = frame_off.shape[0] - 1
    if n > 0 and (frame_off[0] < 0 or frame_off[-1] > frames.nbytes or (np.diff(frame_off) < 0).any()):
        raise ValueError("frame_off must be non-decreasing offsets inside frames")
    rc = _native.lib().rudp_udp_send_batch(sock.fileno(), _np_ptr(frames) if frames.size else None,
                                           _np_ptr(frame_off), max(n, 0), ip.encode(), port)
    if rc < 0:
        raise OSError(-rc, f"sendmmsg: {rc}")
    return rc


def send_batch_to(sock: _socket.socket, frames: np.ndarray, frame_off: np.ndarray, dst: np.ndarray) -> int:
    """Send frame i to ``dst[i]`` (u64 ``addr_key`` per datagram); returns the count sent."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    frame_off = np.ascontiguousarray(frame_off, dtype=np.int64)
    dst = np.ascontiguousarray(dst, dtype=np.uint64)
    n = frame_off.shape[0] - 1
    if dst.shape[0] < n:
        raise ValueError(f"dst has {dst.shape[0]} entries for {n} frames")
    if n > 0 and (frame_off[0] < 0 or frame_off[-1] > frames.nbytes or (np.diff(frame_off) < 0).any()):
        raise ValueError("frame_off must be non-decreasing offsets inside frames")
    if n <= 0:
        return 0
    rc = _native.lib().rudp_udp_send_batch_to(sock.fileno(), _np_ptr(frames) if frames.size else None,
                                              _np_ptr(frame_off), n, _np_ptr(dst), 1)
    if rc < 0:
        raise OSError(-rc, f"sendmmsg: {rc}")
    return rc


class BatchReceiver:
    """A ring of pinned receive slots for one socket, decoded on the GPU.

    ``recv()`` fills the next slot with recvmmsg while the H2D copy and the
    decode of the previous batches run on ``stream``: a slot is handed to the
    socket again only after the event recorded behind its H2D copy has fired,
    so a copy still in flight is never overwritten (no reliance on any other
    synchronization).  ``decode()`` never waits for the device: it enqueues the
    copy and the sync-free varlen decode on ``stream`` and makes the caller's
    current stream wait for them, so ordinary torch work on the results is
    ordered after the decode.

        rx = BatchReceiver(sock, slots=3)
        while (k := rx.recv(timeout_ms=100)):
            dec, frames, off = rx.decode("rudp5", device)   # async
    """

    def __init__(self, sock: _socket.socket, max_msgs: int = 65536, slot_bytes: int = 1024,
                 slots: int = 3, device=None, stream=None, with_sources: bool = False):
        import torch
        if slots < 1:
            raise ValueError("slots must be >= 1")
        self.sock = sock
        self.slot_bytes = slot_bytes
        self.max_msgs = max_msgs
        self.device = torch.device(device) if device is not None else torch.device("cuda", 0)
        self.stream = stream if stream is not None else torch.cuda.Stream(self.device)
        self._frames_t = [torch.empty((max_msgs * slot_bytes,), dtype=torch.uint8, pin_memory=True)
                          for _ in range(slots)]
        self._off_t = [torch.empty((max_msgs + 1,), dtype=torch.int64, pin_memory=True) for _ in range(slots)]
        # each datagram's source (addr_key), for callers that route by it (the relay)
        self._src = [np.empty((max_msgs,), dtype=np.uint64) for _ in range(slots)] if with_sources else None
        self._copied = [None] * slots   # event behind the last H2D copy out of each slot
        # a caller that still reads a slot on the host after recv() returns (the relay's
        # sender thread) holds it; recv() hands a slot to the socket only once released
        import threading
        self._free = [threading.Event() for _ in range(slots)]
        for ev in self._free:
            ev.set()
        self._slot = -1
        self.count = 0

    @property
    def frames(self) -> np.ndarray:
        """Host view of the slot the last recv() filled."""
        return self._frames_t[self._slot].numpy()

    @property
    def frame_off(self) -> np.ndarray:
        return self._off_t[self._slot].numpy()

    @property
    def sources(self) -> np.ndarray:
        """Sources (addr_key) of the datagrams the last recv() took (with_sources=True)."""
        if self._src is None:
            raise RuntimeError("BatchReceiver(with_sources=True) keeps the sources")
        return self._src[self._slot][:self.count]

    def hold(self) -> int:
        """Keep the last batch's slot from the socket until ``release(slot)``
        (a host reader of it on another thread).  Returns the slot."""
        self._free[self._slot].clear()
        return self._slot

    def release(self, slot: int) -> None:
        self._free[slot].set()

    def recv(self, timeout_ms: int = -1) -> int:
        """Receive the next batch into the next slot; returns its datagram count,
        0 when nothing arrived within ``timeout_ms`` (-1: wait forever) -- also
        when the next slot is still held (``hold()``) for longer than that, so a
        caller polling with a timeout (the relay's loop) always gets control back."""
        k = (self._slot + 1) % len(self._frames_t)
        if not self._free[k].wait(None if timeout_ms < 0 else timeout_ms / 1e3):
            return 0
        if self._copied[k] is not None:
            self._copied[k].synchronize()  # that slot's H2D copy has left the pinned buffer
            self._copied[k] = None
        self._slot = k
        self.count = recv_batch(self.sock, self._frames_t[k].numpy(), self._off_t[k].numpy(),
                                slot_bytes=self.slot_bytes, max_msgs=self.max_msgs, timeout_ms=timeout_ms,
                                sources=self._src[k] if self._src is not None else None)
        return self.count

    def frame(self, i: int) -> bytes:
        return bytes(self.frames[self.frame_off[i]:self.frame_off[i + 1]])


    def decode(self, layout="rudp5", device=None, csum=None, stream=None, check=False, utf8=False):
        """H2D of the received frames, then parse + verify them on the device.

        Returns ``(VarlenDecoded, d_frames, d_frame_off)``; the device buffers are
        fresh (the caller owns them; the payload spans index ``d_frames``).
        ``check=True`` also waits for the device's offset check and raises on
        bad offsets (recvmmsg writes valid ones, so the default is not to wait).
        ``utf8=True``: the result's ``valid`` says, per datagram, whether the
        reference's receive (utils/reliableUDP.py:121, get_payload) would decode
        its payload, judged in the same kernel as the parse.
        """
        import torch
        if device is not None and torch.device(device) != self.device:
            raise ValueError(f"this receiver decodes on {self.device}")
        s = stream if stream is not None else self.stream
        k, n = self._slot, self.count
        if k < 0:
            raise RuntimeError("decode() before any recv()")
        total = int(self._off_t[k][n])
        s.wait_stream(torch.cuda.current_stream(self.device))  # e.g. csum written by the caller
        with torch.cuda.stream(s):
            d_frames = torch.empty((total,), dtype=torch.uint8, device=self.device)
            d_off = torch.empty((n + 1,), dtype=torch.int64, device=self.device)
            d_frames.copy_(self._frames_t[k][:total], non_blocking=True)
            d_off.copy_(self._off_t[k][:n + 1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
            self._copied[k] = ev
            dec = _batch.unpack_batch_varlen(d_frames, d_off, layout, csum=csum, stream=s, check=False, utf8=utf8)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(s)
        # allocated on `s`, used on the caller's stream from here on
        for t in (d_frames, d_off, dec._buf):  # the decode's outputs are views of one buffer
            t.record_stream(cur)
        return (dec.check() if check else dec), d_frames, d_off
