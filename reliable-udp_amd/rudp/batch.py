"""Batched encode / decode of Reliable-UDP frames on MI355X.

The reference frames one packet per Python call (utils/reliableUDP.py:53-61
encode, :118-123 decode, through utils/packet.py).  Here a whole batch is
framed, checksummed, parsed and verified by HIP kernels in librudp.so:

    frames, csum = pack_batch(headers, payloads, layout="rudp5")
    dec = unpack_batch(frames, layout="rudp5", csum=csum)

Inputs are either torch tensors on a HIP device (asynchronous, on the current
stream; the device-resident path the benchmark measures) or numpy arrays in
host memory (synchronous; staged through the GPU by rudp_encode_host /
rudp_decode_host, the model of the reference's socket-buffer boundary).
Nothing here computes on the CPU: without librudp.so or a HIP device the
calls raise.

Layouts:
  "rudp5"  the reference's 5-byte header (utils/packet.py:3-10) byte for
           byte; the RFC 1071 checksum comes back as a sideband u16 array.
  "rudp7"  {**custom_header, "checksum": 2}: the checksum in-band at bytes
           5-6, framed exactly as utils/packet.py frames that definition.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import Any, NamedTuple, Optional, Tuple, Union

import numpy as np

from . import _native

LAYOUTS = {"rudp5": 5, "rudp7": 7, 5: 5, 7: 7}

# header byte 4 (utils/packet.py:6-9): SYN 0x80, ACK 0x40, FIN 0x20, offset 0x1F
SYN, ACK, FIN, OFFSET_MASK = 0x80, 0x40, 0x20, 0x1F


def layout_header_len(layout: Union[str, int]) -> int:
    try:
        return LAYOUTS[layout]
    except (KeyError, TypeError):
        raise ValueError(f"unknown layout {layout!r}: use 'rudp5' or 'rudp7'") from None


def make_flags(syn=0, ack=0, fin=0, offset=0):
    """Header byte 4 from the four custom_header bit fields (utils/packet.py:6-9)."""
    return (syn & 1) << 7 | (ack & 1) << 6 | (fin & 1) << 5 | (offset & OFFSET_MASK)


@dataclass
class HeaderTable:
    """SoA header table: seq_num u16[N], ack_num u16[N], flags u8[N]."""
    seq: Any
    ack: Any
    flags: Any

    def __len__(self) -> int:
        return len(self.seq)


class PayloadSpans:
    """Payload i of a packed batch is frames[start[i]:end[i]] (zero-copy).

    Behaves as the pair ``(start, end)`` of int64 [N] tensors; ``start``
    (= min(frame_off[i] + H, frame_off[i + 1]), two device ops) is computed on
    first use, so a decode whose caller reads only the header fields does
    not pay for it.
    """

    __slots__ = ("_frame_off", "_H", "_start")

    def __init__(self, frame_off, H: int):
        self._frame_off = frame_off
        self._H = H
        self._start = None

    @property
    def start(self):
        if self._start is None:
            if isinstance(self._frame_off, np.ndarray):  # a host-memory decode's offsets
                self._start = np.minimum(self._frame_off[:-1] + self._H, self._frame_off[1:])
            else:
                import torch
                self._start = torch.minimum(self._frame_off[:-1] + self._H, self._frame_off[1:])
        return self._start

    @property
    def end(self):
        return self._frame_off[1:]

    def __iter__(self):
        return iter((self.start, self.end))

    def __getitem__(self, i):
        return (self.start, self.end)[i]

    def __len__(self):
        return 2


_ST_MESSAGES = (
    (_native.ST_LEN, "lengths must lie in [0, 65535]"),
    (_native.ST_PAYLOAD, "packed payloads: sum(lengths) must equal payload.numel(); "
                         "gathered payloads: payload_off + lengths must stay inside payload"),
    (_native.ST_FRAMES_CAP, "out is too small for the frames (sum(lengths) + N * header bytes)"),
    (_native.ST_OFFSETS, "frame_off must be non-decreasing offsets inside frames"),
)


def _raise_status(status) -> None:
    """Read a sync-free call's device status word (synchronizes) and raise
    ValueError with the reason when the device found the batch invalid."""
    if status is None:
        return
    bits = int(status.item())
    if bits:
        raise ValueError("; ".join(m for b, m in _ST_MESSAGES if bits & b) or f"status {bits:#x}")


class DecodedBatch(NamedTuple):
    seq: Any
    ack: Any
    flags: Any
    ok: Any          # 1 good, 0 bad checksum, 2 short frame, 3 unverified (rudp5, no csum)
    csum: Any        # recomputed checksum per packet
    payload: Any     # [N, L] view into frames (zero-copy) or a copy
    status: Any = None  # sync-free varlen decode: device u32[1], RUDP_ST_* (0 = valid)
    valid: Any = None   # utf8=True: u8 [N], 1 where get_payload() would return, 0 where it raises

    def check(self) -> "DecodedBatch":
        """Raise ValueError if the device rejected the batch (reads ``status``:
        one synchronization).  A no-op for calls that checked eagerly."""
        _raise_status(self.status)
        return self


def _is_torch(x) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


_PIN_DT = {np.uint8: "uint8", np.uint16: "uint16", np.int64: "int64"}


def _pinned_out(n: int, dtype) -> np.ndarray:
    """A per-packet output array of a *_host call: page-locked, from torch's
    caching host allocator (a repeated call of the same size reuses the block),
    so the pipeline's D2H lands at the link's rate instead of faulting fresh
    pageable pages in.  Only the small per-packet arrays come from here; frames
    and payloads are the caller's or plain numpy."""
    import torch
    return torch.empty((n,), dtype=getattr(torch, _PIN_DT[dtype]), pin_memory=True).numpy()


def _as_table(headers) -> HeaderTable:
    if isinstance(headers, HeaderTable):
        return headers
    if isinstance(headers, dict):
        return HeaderTable(headers["seq_num"], headers["ack_num"], headers["flags"])
    seq, ack, flags = headers
    return HeaderTable(seq, ack, flags)


# ---------------------------------------------------------------- device path
def _dev_check(t, name, dtype, ndim, device):
    import torch
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor on the same device")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _stream_ptr(stream, device) -> int:
    import torch
    if stream is not None:
        return int(stream.cuda_stream)
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)  # no Stream object per call
    if raw is not None:
        return int(raw(device.index if device.index is not None else torch.cuda.current_device()))
    return int(torch.cuda.current_stream(device).cuda_stream)


def _pack_device(tab: HeaderTable, payloads, H: int, out, csum_out, want_csum, stream):
    import torch
    dev = payloads.device
    if dev.type != "cuda":
        raise ValueError("device path needs tensors on a HIP device")
    _dev_check(payloads, "payloads", torch.uint8, 2, dev)
    n, L = payloads.shape
    for name, t, dt in (("seq", tab.seq, torch.uint16), ("ack", tab.ack, torch.uint16),
                        ("flags", tab.flags, torch.uint8)):
        _dev_check(t, name, dt, 1, dev)
        if t.shape[0] != n:
            raise ValueError(f"{name} has {t.shape[0]} entries for {n} payloads")
    F = L + H
    if out is None:
        out = torch.empty((n, F), dtype=torch.uint8, device=dev)
    else:
        _dev_check(out, "out", torch.uint8, 2, dev)
        if tuple(out.shape) != (n, F):
            raise ValueError(f"out must have shape {(n, F)}, got {tuple(out.shape)}")
    if csum_out is None and want_csum:
        csum_out = torch.empty((n,), dtype=torch.uint16, device=dev)
    elif csum_out is not None:
        _dev_check(csum_out, "csum_out", torch.uint16, 1, dev)
    b = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(),
                          ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(),
                          payload=payloads.data_ptr() if n * L else None, len=None,
                          payload_off=None)
    _native.check(_native.lib().rudp_encode(
        ctypes.byref(b), out.data_ptr() if n else None,
        csum_out.data_ptr() if (csum_out is not None and n) else None,
        H, dev.index if dev.index is not None else torch.cuda.current_device(),
        _stream_ptr(stream, dev)))
    return out, csum_out


def _unpack_device(frames, H: int, csum, copy_payload: bool, stream, utf8: bool = False):
    import torch
    dev = frames.device
    if dev.type != "cuda":
        raise ValueError("device path needs tensors on a HIP device")
    _dev_check(frames, "frames", torch.uint8, 2, dev)
    n, F = frames.shape
    L = max(F - H, 0)
    seq = torch.empty((n,), dtype=torch.uint16, device=dev)
    ack = torch.empty((n,), dtype=torch.uint16, device=dev)
    flags = torch.empty((n,), dtype=torch.uint8, device=dev)
    ok = torch.empty((n,), dtype=torch.uint8, device=dev)
    cs = torch.empty((n,), dtype=torch.uint16, device=dev)
    if csum is not None:
        _dev_check(csum, "csum", torch.uint16, 1, dev)
        if csum.shape[0] != n:
            raise ValueError(f"csum has {csum.shape[0]} entries for {n} frames")
    pay = torch.empty((n, L), dtype=torch.uint8, device=dev) if copy_payload else None
    valid = torch.empty((n,), dtype=torch.uint8, device=dev) if utf8 else None
    if n:
        _native.check(_native.lib().rudp_decode_utf8(
            frames.data_ptr() if F else None, None, F, n, csum.data_ptr() if csum is not None else None,
            seq.data_ptr(), ack.data_ptr(), flags.data_ptr(), ok.data_ptr(), cs.data_ptr(),
            pay.data_ptr() if (pay is not None and L) else None,
            valid.data_ptr() if valid is not None else None, H,
            dev.index if dev.index is not None else torch.cuda.current_device(),
            _stream_ptr(stream, dev)))
    if pay is None:
        pay = frames[:, H:] if F >= H else frames[:, :0]
    return DecodedBatch(seq, ack, flags, ok, cs, pay, None, valid)


# ------------------------------------------------------------------ host path
def _host_arr(a, name, dtype, ndim):
    a = np.ascontiguousarray(a)
    if a.dtype != dtype:
        raise TypeError(f"{name} must be {np.dtype(dtype)}, got {a.dtype}")
    if a.ndim != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {a.shape}")
    return a


def _ptr(a) -> Optional[int]:
    return a.ctypes.data if a.size else None


def _host_out(a, name, dtype, shape):
    if not isinstance(a, np.ndarray) or a.dtype != dtype or a.shape != shape \
            or not a.flags["C_CONTIGUOUS"] or not a.flags["WRITEABLE"]:
        raise ValueError(f"{name} must be a writeable C-contiguous {np.dtype(dtype)} array of shape {shape}")
    return a


def _pack_host(tab: HeaderTable, payloads, H, want_csum, device, out=None, csum_out=None):
    payloads = _host_arr(payloads, "payloads", np.uint8, 2)
    n, L = payloads.shape
    seq = _host_arr(tab.seq, "seq", np.uint16, 1)
    ack = _host_arr(tab.ack, "ack", np.uint16, 1)
    flags = _host_arr(tab.flags, "flags", np.uint8, 1)
    for name, a in (("seq", seq), ("ack", ack), ("flags", flags)):
        if a.shape[0] != n:
            raise ValueError(f"{name} has {a.shape[0]} entries for {n} payloads")
    frames = (_host_out(out, "out", np.uint8, (n, L + H)) if out is not None
              else np.empty((n, L + H), dtype=np.uint8))
    if csum_out is not None:
        csum = _host_out(csum_out, "csum_out", np.uint16, (n,))
    else:
        csum = _pinned_out(n, np.uint16) if want_csum else None
    b = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=_ptr(seq), ack=_ptr(ack),
                          flags=_ptr(flags), payload=_ptr(payloads), len=None, payload_off=None)
    _native.check(_native.lib().rudp_encode_host(
        ctypes.byref(b), _ptr(frames), _ptr(csum) if csum is not None else None, H, device))
    return frames, csum


def _unpack_host(frames, H, csum, copy_payload, device, utf8=False):
    frames = _host_arr(frames, "frames", np.uint8, 2)
    n, F = frames.shape
    L = max(F - H, 0)
    seq = _pinned_out(n, np.uint16)
    ack = _pinned_out(n, np.uint16)
    flags = _pinned_out(n, np.uint8)
    ok = _pinned_out(n, np.uint8)
    cs = _pinned_out(n, np.uint16)
    if csum is not None:
        csum = _host_arr(csum, "csum", np.uint16, 1)
        if csum.shape[0] != n:
            raise ValueError(f"csum has {csum.shape[0]} entries for {n} frames")
    pay = np.empty((n, L), np.uint8) if copy_payload else None
    valid = _pinned_out(n, np.uint8) if utf8 else None
    if n:
        _native.check(_native.lib().rudp_decode_host(
            _ptr(frames), F, n, _ptr(csum) if csum is not None else None, _ptr(seq), _ptr(ack),
            _ptr(flags), _ptr(ok), _ptr(cs), _ptr(pay) if pay is not None else None,
            _ptr(valid) if valid is not None else None, H, device))
    if pay is None:
        pay = frames[:, H:] if F >= H else frames[:, :0]
    return DecodedBatch(seq, ack, flags, ok, cs, pay, None, valid)


# ------------------------------------------------------------------ public API
def pack_batch(headers, payloads, layout: Union[str, int] = "rudp7", *, out=None,
               csum_out=None, want_csum: Optional[bool] = None, stream=None, device: int = 0
               ) -> Tuple[Any, Any]:
    """Frame + checksum a batch.  Returns ``(frames, csum)``.

    ``headers``: HeaderTable, ``(seq, ack, flags)`` or a dict keyed like
    custom_header (``seq_num``, ``ack_num``) plus ``flags``.  ``payloads``:
    uint8 ``[N, L]``.  ``csum`` is the per-packet checksum (always for rudp5,
    on request for rudp7; else None).  Torch tensors on a HIP device run
    asynchronously on ``stream`` (default: current stream); numpy arrays run
    synchronously through ``device``.
    """
    H = layout_header_len(layout)
    tab = _as_table(headers)
    if want_csum is None:
        want_csum = H == 5
    if _is_torch(payloads):
        return _pack_device(tab, payloads, H, out, csum_out, want_csum, stream)
    return _pack_host(tab, payloads, H, want_csum, device, out, csum_out)


def unpack_batch(frames, layout: Union[str, int] = "rudp7", *, csum=None,
                 copy_payload: bool = False, stream=None, device: int = 0, utf8: bool = False) -> DecodedBatch:
    """Parse + verify a batch of fixed-length frames ``[N, F]``.

    ``csum`` (rudp5 only): sideband checksums to verify against.  The payload
    is returned as a zero-copy view ``frames[:, H:]`` unless ``copy_payload``.
    ``utf8``: also ``valid``, u8 [N], 1 where Packet(frame).get_payload()
    would return and 0 where its strict UTF-8 decode would raise
    (utils/packet.py:68-73), judged in the same pass over the frames
    (rudp_decode_utf8; numpy frames: rudp_decode_host, staged through the GPU).
    """
    H = layout_header_len(layout)
    if H == 7 and csum is not None:
        raise ValueError("rudp7 carries its checksum in-band; csum= is for rudp5")
    if _is_torch(frames):
        return _unpack_device(frames, H, csum, copy_payload, stream, utf8)
    return _unpack_host(frames, H, csum, copy_payload, device, utf8)


def synth_batch(n: int, payload_len: int, seed: int, *, first_index: int = 0, ascii: bool = True,
                device=None, stream=None) -> Tuple[HeaderTable, Any]:
    """Generate the deterministic synthetic batch on a HIP device (rudp_synth)."""
    import torch
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    seq = torch.empty((n,), dtype=torch.uint16, device=dev)
    ack = torch.empty((n,), dtype=torch.uint16, device=dev)
    flags = torch.empty((n,), dtype=torch.uint8, device=dev)
    pay = torch.empty((n, payload_len), dtype=torch.uint8, device=dev)
    if n:
        _native.check(_native.lib().rudp_synth(
            seed & (2**64 - 1), first_index, n, payload_len, 1 if ascii else 0, seq.data_ptr(),
            ack.data_ptr(), flags.data_ptr(), pay.data_ptr() if payload_len else None,
            dev.index if dev.index is not None else 0, _stream_ptr(stream, dev)))
    return HeaderTable(seq, ack, flags), pay


# ------------------------------------------------------- variable-length batches
class VarlenFrames:
    """Result of ``pack_batch_varlen``: ``frames`` (u8, frames back to back, or
    the caller's ``out``), ``frame_off`` (int64 [N + 1]: frame i =
    frames[frame_off[i]:frame_off[i + 1]]), ``csum`` (u16 [N] or None) and
    ``status`` (device int32 [1], RUDP_ST_* of the call, 0 = valid).

    All of them live in one device allocation and are cut out of it on first
    access, so a sync-free caller that only keeps the result pays for one
    allocation and the launch.  Iterates as (frames, frame_off, csum, status).
    """

    __slots__ = ("_buf", "_n", "_cs_bytes", "_f_at", "_frames", "_frame_off", "_csum", "_status")

    # one allocation: frame_off (i64 [n + 1]) | status (i32) | pad | csum (u16 [n]) |
    # pad to 16 B | frames (unless the caller's)
    def __init__(self, buf, n: int, cs_bytes: int, f_at: int, frames=None):
        self._buf, self._n, self._cs_bytes, self._f_at = buf, n, cs_bytes, f_at
        self._frames, self._frame_off, self._csum, self._status = frames, None, None, None

    @staticmethod
    def layout(n: int, want_csum: bool):
        """(bytes before the frames, csum bytes): the allocation's head."""
        cs_bytes = 2 * n if want_csum else 0
        head = 8 * (n + 1) + 8 + cs_bytes
        return head + (-head % 16), cs_bytes

    @property
    def frames(self):
        if self._frames is None:
            self._frames = self._buf[self._f_at:]
        return self._frames

    @property
    def frame_off(self):
        if self._frame_off is None:
            import torch
            self._frame_off = self._buf[:8 * (self._n + 1)].view(torch.int64)
        return self._frame_off

    @property
    def status(self):
        if self._status is None:
            import torch
            at = 8 * (self._n + 1)
            self._status = self._buf[at:at + 4].view(torch.int32)
        return self._status

    @property
    def csum(self):
        if self._csum is None and self._cs_bytes:
            import torch
            at = 8 * (self._n + 1) + 8
            self._csum = self._buf[at:at + self._cs_bytes].view(torch.uint16)
        return self._csum

    def __iter__(self):
        return iter((self.frames, self.frame_off, self.csum, self.status))

    def __getitem__(self, i):
        return tuple(self)[i]

    def __len__(self):
        return 4

    def check(self) -> "VarlenFrames":
        """Raise ValueError if the device rejected the batch (one synchronization)."""
        _raise_status(self.status)
        return self


class VarlenDecoded:
    """Result of ``unpack_batch_varlen``, with the fields of ``DecodedBatch``:
    seq, ack (u16 [N]), flags, ok (u8 [N]), csum (u16 [N]), payload
    (``PayloadSpans``), status and valid (u8 [N] with ``utf8=True``, else
    None).  The output arrays share one device allocation and are cut out of
    it on first access.  Iterates as (seq, ack, flags, ok, csum, payload,
    status)."""

    __slots__ = ("_buf", "_n", "payload", "_v", "_utf8", "_stream")

    def __init__(self, buf, n: int, payload, utf8: bool = False, stream=None):
        self._buf, self._n, self.payload, self._v, self._utf8 = buf, n, payload, {}, utf8
        self._stream = stream  # the stream the decode was enqueued on (None: the current one)

    # one allocation: seq | ack | csum (u16 [n] each) | flags | ok | valid (u8 [n] each)
    def _cut(self, name, at, nbytes, dtype):
        v = self._v.get(name)
        if v is None:
            v = self._buf[at:at + nbytes]
            if dtype is not None:
                v = v.view(dtype)
            self._v[name] = v
        return v

    @property
    def seq(self):
        import torch
        return self._cut("seq", 0, 2 * self._n, torch.uint16)

    @property
    def ack(self):
        import torch
        return self._cut("ack", 2 * self._n, 2 * self._n, torch.uint16)

    @property
    def csum(self):
        import torch
        return self._cut("csum", 4 * self._n, 2 * self._n, torch.uint16)

    @property
    def flags(self):
        return self._cut("flags", 6 * self._n, self._n, None)

    @property
    def ok(self):
        return self._cut("ok", 7 * self._n, self._n, None)

    @property
    def valid(self):
        return self._cut("valid", 8 * self._n, self._n, None) if self._utf8 else None

    @property
    def status(self):
        """Device int32 [1]: RUDP_ST_OFFSETS when a frame was rejected for bad
        offsets (ok == RUDP_OK_BAD_OFFSETS), else 0, as ``VarlenFrames.status``.
        The decode keeps no status word of its own (a call is its one kernel,
        rudp_decode_varlen_checked with d_status NULL), so this is built from
        ``ok`` on first access: one device reduction, no synchronization, on
        the stream the decode ran on (so it reads ``ok`` after the decode wrote
        it), with the caller's current stream then made to wait for it."""
        v = self._v.get("status")
        if v is None:
            import torch
            if self._stream is None:
                v = ((self.ok == _native.OK_BAD_OFFSETS).any().to(torch.int32) * _native.ST_OFFSETS).reshape(1)
            else:
                cur = torch.cuda.current_stream(self._buf.device)
                with torch.cuda.stream(self._stream):
                    v = ((self.ok == _native.OK_BAD_OFFSETS).any().to(torch.int32) * _native.ST_OFFSETS).reshape(1)
                cur.wait_stream(self._stream)
                v.record_stream(cur)
            self._v["status"] = v
        return v

    def __iter__(self):
        return iter((self.seq, self.ack, self.flags, self.ok, self.csum, self.payload, self.status))

    def __getitem__(self, i):
        return tuple(self)[i]

    def __len__(self):
        return 7

    def check(self) -> "VarlenDecoded":
        """Raise ValueError if a frame was rejected for bad offsets (reads ok[]: one
        device reduction and one synchronization)."""
        _raise_status(self.status)
        return self


_tls = threading.local()


def _batch_struct() -> "_native.RudpBatch":
    """This thread's reusable struct rudp_batch (the C call only reads it during the call)."""
    b = getattr(_tls, "batch", None)
    if b is None:
        b = _tls.batch = _native.RudpBatch()
    return b


def _int_tensor(t, name, device, n=None, dtypes=None):
    import torch
    dtypes = dtypes or (torch.int32,)
    if not isinstance(t, torch.Tensor) or t.device != device or t.dtype not in dtypes \
            or t.dim() != 1 or not t.is_contiguous():
        raise TypeError(f"{name} must be a contiguous 1-D {'/'.join(map(str, dtypes))} tensor on {device}")
    if n is not None and t.shape[0] != n:
        raise ValueError(f"{name} has {t.shape[0]} entries, expected {n}")


class HostVarlenFrames(NamedTuple):
    """Result of ``pack_batch_varlen`` on numpy arrays (host memory, staged
    through the GPU by rudp_encode_varlen_host): frames (u8, back to back),
    frame_off (int64 [N + 1]), csum (u16 [N] or None), status (always 0: the
    batch was checked before any frame byte was written, and a bad one raised)."""
    frames: Any
    frame_off: Any
    csum: Any
    status: int = 0

    def check(self) -> "HostVarlenFrames":
        return self


def _pack_varlen_host(tab: HeaderTable, payload, lengths, H, payload_off, want_csum, out, device):
    if payload_off is not None:
        raise ValueError("host-memory varlen encode takes packed payloads (payload_off=None)")
    payload = _host_arr(payload, "payload", np.uint8, 1)
    lengths = np.ascontiguousarray(lengths)
    if lengths.dtype not in (np.int32, np.uint32) or lengths.ndim != 1:
        raise TypeError("lengths must be a 1-D int32/uint32 array")
    n = lengths.shape[0]
    seq = _host_arr(tab.seq, "seq", np.uint16, 1)
    ack = _host_arr(tab.ack, "ack", np.uint16, 1)
    flags = _host_arr(tab.flags, "flags", np.uint8, 1)
    for name, a in (("seq", seq), ("ack", ack), ("flags", flags)):
        if a.shape[0] != n:
            raise ValueError(f"{name} has {a.shape[0]} entries for {n} packets")
    # (the lengths, their sum against the payload and the capacity are checked by the
    # C entry before any frame byte is written: a bad batch raises ValueError)
    if out is not None:
        if not isinstance(out, np.ndarray) or out.dtype != np.uint8 or out.ndim != 1 \
                or not out.flags["C_CONTIGUOUS"] or not out.flags["WRITEABLE"]:
            raise ValueError("out must be a writeable C-contiguous 1-D uint8 array")
        frames = out
    else:
        frames = np.empty((payload.size + n * H,), np.uint8)
    off = _pinned_out(n + 1, np.int64)
    csum = _pinned_out(n, np.uint16) if want_csum else None
    b = _native.RudpBatch(n=n, payload_len=min(payload.size // n, 65535) if n else 0, reserved=0,
                          seq=_ptr(seq), ack=_ptr(ack), flags=_ptr(flags), payload=_ptr(payload),
                          len=_ptr(lengths.view(np.uint32)), payload_off=None)
    _native.check(_native.lib().rudp_encode_varlen_host(
        ctypes.byref(b), payload.size, _ptr(frames) if frames.size else 16, frames.size, off.ctypes.data,
        _ptr(csum) if csum is not None else None, H, device))
    return HostVarlenFrames(frames, off, csum, 0)


def pack_batch_varlen(headers, payload, lengths, layout: Union[str, int] = "rudp7", *,
                      payload_off=None, want_csum: Optional[bool] = None, stream=None, out=None,
                      check: bool = True, reuse: Optional[VarlenFrames] = None, device: int = 0) -> VarlenFrames:
    """Frame + checksum a variable-length batch on a HIP device.

    ``payload``: u8 1-D tensor holding the payload bytes; ``lengths``: int32
    [N] bytes per packet (<= 65535); ``payload_off``: int64 [N] start of each
    payload in ``payload``, or None when the payloads are packed back to back
    in packet order.  Returns frames packed back to back plus their offsets:
    frame i is byte-identical to Packet(...).to_byte() of that packet
    (utils/reliableUDP.py:53-61 builds one per character).

    The argument checks run on the device, inside the call (rudp_encode_varlen_checked):
    ``check=True`` waits for them and raises ValueError on a bad batch, as the
    reference's per-packet calls would fail; ``check=False`` never waits — the
    host does not touch the device — and the result's ``check()`` raises later.
    A rejected batch leaves ``frames`` unwritten.  ``out``: u8 1-D frame buffer
    of at least sum(lengths) + N * header bytes (its first frame_off[-1] bytes
    are the frames).  Without ``out`` the frame buffer is sized on the host for
    packed payloads (payload.numel() + N * header bytes) and, for gathered
    payloads, from one device read of the lengths' sum.  ``reuse``: an earlier
    result of this call for the same N and csum choice, whose buffers take this
    call's outputs (no allocation; the earlier result's contents are replaced).

    numpy arrays (packed payloads in host memory, a send buffer): staged
    through GPU ``device`` by rudp_encode_varlen_host, synchronously; the
    lengths are checked before any frame byte is written (ValueError) and the
    result is a ``HostVarlenFrames`` of numpy arrays.
    """
    H = layout_header_len(layout)
    tab = _as_table(headers)
    if want_csum is None:
        want_csum = H == 5
    if not _is_torch(payload):
        return _pack_varlen_host(tab, payload, lengths, H, payload_off, want_csum, out, device)
    import torch
    dev = payload.device
    if dev.type != "cuda":
        raise ValueError("varlen batches run on a HIP device")
    _dev_check(payload, "payload", torch.uint8, 1, dev)
    _int_tensor(lengths, "lengths", dev, dtypes=(torch.int32, torch.uint32))
    n = lengths.shape[0]
    for name, t, dt in (("seq", tab.seq, torch.uint16), ("ack", tab.ack, torch.uint16),
                        ("flags", tab.flags, torch.uint8)):
        _dev_check(t, name, dt, 1, dev)
        if t.shape[0] != n:
            raise ValueError(f"{name} has {t.shape[0]} entries for {n} packets")
    if payload_off is not None:
        _int_tensor(payload_off, "payload_off", dev, n, dtypes=(torch.int64,))
    frames = None
    if out is not None:
        _dev_check(out, "out", torch.uint8, 1, dev)
        frames = out
    if payload_off is None:
        # exact for a valid packed batch (the device checks it); an oversized `out`
        # is only capacity and never inflates the hint that picks the kernel's tiles
        lsum = payload.numel()
    elif out is not None:
        # gathered into the caller's buffer: no device read, the hint is bounded by
        # both the payload buffer and the frame buffer
        lsum = min(payload.numel(), max(out.numel() - n * H, 0))
    else:
        # gathered payloads: the frame bytes are unknown until the lengths are summed
        # (rudp_varlen_bounds, one 40-byte device read); lengths are read as u32
        lmin = lmax = lsum = omin = oend = 0
        if n:
            bnd = (ctypes.c_int64 * 5)()
            _native.check(_native.lib().rudp_varlen_bounds(
                lengths.data_ptr(), payload_off.data_ptr(), n, bnd, dev.index or 0, _stream_ptr(stream, dev)))
            lmin, lmax, lsum, omin, oend = list(bnd)
        if lmin < 0 or lmax > 65535:
            raise ValueError("lengths must lie in [0, 65535]")
        if omin < 0 or oend > payload.numel():
            raise ValueError("payload_off + lengths must stay inside payload")
    f_at, cs_bytes = VarlenFrames.layout(n, want_csum)
    if reuse is not None:
        # the caller's earlier result of the same shape: its buffer takes this call's outputs
        need = f_at + (0 if frames is not None else lsum + n * H)
        if not isinstance(reuse, VarlenFrames) or reuse._n != n or reuse._cs_bytes != cs_bytes \
                or reuse._buf.device != dev or reuse._buf.numel() != need:
            raise ValueError("reuse= must be an earlier pack_batch_varlen result for the same N, "
                             "csum choice, device and frame bytes (and out= or not, as then)")
        buf = reuse._buf
    else:
        # (payload is u8 on dev: new_empty skips torch.empty's dtype/device parsing, ~0.5 us a call)
        buf = payload.new_empty(f_at + (0 if frames is not None else lsum + n * H))
    base = buf.data_ptr()
    f_ptr = frames.data_ptr() if frames is not None else base + f_at
    f_cap = frames.numel() if frames is not None else buf.numel() - f_at
    # payload_len carries the mean payload length: a hint that picks lanes per packet
    b = _batch_struct()
    b.n, b.payload_len = n, min(lsum // n, 65535) if n else 0
    b.seq, b.ack, b.flags = tab.seq.data_ptr(), tab.ack.data_ptr(), tab.flags.data_ptr()
    b.payload = payload.data_ptr() if payload.numel() else 16  # never read: all lengths 0
    b.len = lengths.data_ptr()
    b.payload_off = payload_off.data_ptr() if payload_off is not None else None
    _native.check(_native.lib().rudp_encode_varlen_checked(
        ctypes.byref(b), payload.numel(), f_ptr if f_cap else 16, f_cap,
        base, base + 8 * (n + 1) + 8 if cs_bytes else None, base + 8 * (n + 1), H,
        dev.index or 0, _stream_ptr(stream, dev)))
    res = VarlenFrames(buf, n, cs_bytes, f_at, frames)
    return res.check() if check else res


def _check_offsets(frames, frame_off, stream=None) -> int:
    """Validate offsets (one device->host read); returns the mean frame length."""
    n = frame_off.shape[0] - 1
    if n < 1:
        return 0
    out = (ctypes.c_int64 * 3)()  # min, max, decreasing pairs (rudp_frame_off_bounds)
    _native.check(_native.lib().rudp_frame_off_bounds(
        frame_off.data_ptr(), n, out, frame_off.device.index or 0, _stream_ptr(stream, frame_off.device)))
    first, last, nbad = list(out)
    if first < 0 or nbad or last > frames.numel():
        raise ValueError("frame_off must be non-decreasing offsets inside frames")
    return min((last - first) // n, 0xFFFFFFFF)


def _unpack_varlen_host(frames, frame_off, H, csum, check, utf8, device, len_hint=0, reuse=None):
    frames = _host_arr(frames, "frames", np.uint8, 1)
    frame_off = np.ascontiguousarray(frame_off)
    if frame_off.dtype not in (np.int64, np.uint64) or frame_off.ndim != 1:
        raise TypeError("frame_off must be a 1-D int64 array")
    n = frame_off.shape[0] - 1
    if n < 0:
        raise ValueError("frame_off needs N + 1 entries")
    if csum is not None:
        csum = _host_arr(csum, "csum", np.uint16, 1)
        if csum.shape[0] != n:
            raise ValueError(f"csum has {csum.shape[0]} entries for {n} frames")
    if reuse is not None:
        # an earlier host result of the same N and utf8 choice: its arrays take this call's outputs
        if not isinstance(reuse, DecodedBatch) or not isinstance(reuse.seq, np.ndarray) or reuse.seq.shape != (n,) \
                or (reuse.valid is not None) != utf8:
            raise ValueError("reuse= must be an earlier host unpack_batch_varlen result for the same N and utf8 choice")
        seq, ack, cs, flags, ok, valid = reuse.seq, reuse.ack, reuse.csum, reuse.flags, reuse.ok, reuse.valid
        status = reuse.status
        status[0] = 0
    else:
        seq, ack, cs = (_pinned_out(n, np.uint16) for _ in range(3))
        flags, ok = _pinned_out(n, np.uint8), _pinned_out(n, np.uint8)
        valid = _pinned_out(n, np.uint8) if utf8 else None
        status = np.zeros((1,), np.uint32)
    if n:
        # (negative int64 offsets read as huge u64 ones: past the buffer, so rejected)
        _native.check(_native.lib().rudp_decode_varlen_host(
            _ptr(frames), frames.size, frame_off.ctypes.data, min(len_hint or frames.size // n, 0xFFFFFFFF), n,
            _ptr(csum) if csum is not None else None, _ptr(seq), _ptr(ack), _ptr(flags), _ptr(ok), _ptr(cs),
            _ptr(valid) if valid is not None else None, status.ctypes.data, H, device))
    # payload spans computed on first use (two passes over N offsets: ~1 ms per 1M frames)
    pay = PayloadSpans(frame_off.view(np.int64) if frame_off.dtype == np.uint64 else frame_off, H)
    res = DecodedBatch(seq, ack, flags, ok, cs, pay, status, valid)
    return res.check() if check else res


def unpack_batch_varlen(frames, frame_off, layout: Union[str, int] = "rudp7", *, csum=None,
                        stream=None, check: bool = True, reuse: Optional["VarlenDecoded"] = None,
                        utf8: bool = False, device: int = 0) -> "VarlenDecoded":
    """Parse + verify frames packed back to back (offsets as pack_batch_varlen returns).

    The payload is zero-copy: ``payload`` is the pair ``(start, end)`` of int64
    [N] tensors indexing ``frames`` (empty for frames shorter than the header),
    as a ``PayloadSpans`` that computes ``start`` on first use.  The offsets
    are checked on the device inside the call (rudp_decode_varlen_checked):
    every frame with bad offsets gets ok == RUDP_OK_BAD_OFFSETS, and
    ``check=True`` waits and raises ValueError when there is one;
    ``check=False`` never waits, and the result's ``check()`` raises later.
    ``reuse``: an earlier result for the same N whose output buffer takes this
    call's outputs (no allocation).  ``utf8``: also ``valid`` (u8 [N]: 1 where
    Packet(frame).get_payload() would return, 0 where its strict UTF-8 decode
    would raise, utils/packet.py:68-73; 0 for a rejected frame), judged by the
    decode kernel from the bytes it already holds (rudp_decode_varlen_utf8).

    numpy arrays (a receive buffer in host memory): staged through GPU
    ``device`` by rudp_decode_varlen_host, synchronously, with the same
    per-frame offset rule; the result is a ``DecodedBatch`` of numpy arrays
    (payload: ``PayloadSpans`` of int64 arrays, status u32 [1]); ``reuse``: an
    earlier such result whose arrays take this call's outputs (a receive loop
    keeps its buffers; pinned ones copy back at the link's rate).
    """
    H = layout_header_len(layout)
    if H == 7 and csum is not None:
        raise ValueError("rudp7 carries its checksum in-band; csum= is for rudp5")
    if not _is_torch(frames):
        return _unpack_varlen_host(frames, frame_off, H, csum, check, utf8, device, reuse=reuse)
    import torch
    dev = frames.device
    _dev_check(frames, "frames", torch.uint8, 1, dev)
    _int_tensor(frame_off, "frame_off", dev, dtypes=(torch.int64,))
    n = frame_off.shape[0] - 1
    if n < 0:
        raise ValueError("frame_off needs N + 1 entries")
    if csum is not None:
        _dev_check(csum, "csum", torch.uint16, 1, dev)
        if csum.shape[0] != n:
            raise ValueError(f"csum has {csum.shape[0]} entries for {n} frames")
    # one allocation for every output: seq | ack | csum (u16) | flags | ok (u8), cut
    # into views only when the caller reads them (per-view slicing was most of the
    # entry's host time at small batches)
    per = 9 if utf8 else 8
    if reuse is not None:
        if not isinstance(reuse, VarlenDecoded) or reuse._n != n or reuse._buf.device != dev \
                or reuse._utf8 != utf8:
            raise ValueError("reuse= must be an earlier unpack_batch_varlen result for the same N, device "
                             "and utf8 choice")
        buf = reuse._buf
    else:
        buf = frames.new_empty(per * n)  # (u8 on dev, checked above)
    base = buf.data_ptr()
    # mean frame length from the buffer size: a hint that picks lanes / tiles per frame
    hint = min(frames.numel() // n, 0xFFFFFFFF) if n else 0
    # no status word: a rejected frame is ok == RUDP_OK_BAD_OFFSETS (check() reads that)
    _native.check(_native.lib().rudp_decode_varlen_utf8(
        frames.data_ptr() if frames.numel() else 16, frames.numel(), frame_off.data_ptr(), hint, n,
        csum.data_ptr() if csum is not None else None, base, base + 2 * n, base + 6 * n, base + 7 * n,
        base + 4 * n, base + 8 * n if utf8 else None, None, H, dev.index or 0, _stream_ptr(stream, dev)))
    res = VarlenDecoded(buf, n, PayloadSpans(frame_off, H), utf8, stream)
    return res.check() if check else res


def validate_utf8(frames, layout: Union[str, int] = "rudp7", *, frame_off=None, stream=None):
    """u8 [N]: 1 where Packet(frame).get_payload() would succeed (utils/packet.py:68-73),
    0 where it would raise UnicodeDecodeError.  ``frames``: [N, F] fixed-length,
    or 1-D with ``frame_off`` (N + 1 offsets)."""
    import torch
    H = layout_header_len(layout)
    dev = frames.device
    if frame_off is None:
        _dev_check(frames, "frames", torch.uint8, 2, dev)
        n, F = frames.shape
        off_ptr = None
    else:
        _dev_check(frames, "frames", torch.uint8, 1, dev)
        _int_tensor(frame_off, "frame_off", dev, dtypes=(torch.int64,))
        n = frame_off.shape[0] - 1
        F = _check_offsets(frames, frame_off, stream)  # mean frame length: a lanes-per-frame hint
        off_ptr = frame_off.data_ptr()
    valid = torch.empty((n,), dtype=torch.uint8, device=dev)
    if n:
        _native.check(_native.lib().rudp_validate_utf8(
            frames.data_ptr() if frames.numel() else None, off_ptr, F, n, H, valid.data_ptr(),
            dev.index or 0, _stream_ptr(stream, dev)))
    return valid


PROXY_MAX_MEMORY = 500  # proxy.py:17


def detect_retransmissions(frames, *, frame_off=None, window: int = PROXY_MAX_MEMORY, stream=None,
                           check: bool = True):
    """u8 [N]: 1 where frame i equals one of the `window` frames before it.

    Batched form of the reference proxy's `packet in self.packets` check
    (proxy.py:90, with the 500-packet history of proxy.py:17, :92-94) and
    Packet.__eq__ semantics (utils/packet.py:83-86).  ``frames``: [N, F]
    fixed-length, or 1-D with ``frame_off`` (N + 1 offsets), checked on the
    device (rudp_dedup_window_checked): a frame whose offsets are decreasing or
    past ``frames`` gets 2 and is never read; ``check=True`` waits and raises
    ValueError when there is one, ``check=False`` never waits.
    """
    import torch
    dev = frames.device
    if frame_off is None:
        _dev_check(frames, "frames", torch.uint8, 2, dev)
        n, F = frames.shape
        off_ptr = None
    else:
        _dev_check(frames, "frames", torch.uint8, 1, dev)
        _int_tensor(frame_off, "frame_off", dev, dtypes=(torch.int64,))
        n = frame_off.shape[0] - 1
        if n < 0:
            raise ValueError("frame_off needs N + 1 entries")
        dup = torch.empty((n,), dtype=torch.uint8, device=dev)
        if n:
            # mean frame length from the buffer size: picks lanes per frame
            _native.check(_native.lib().rudp_dedup_window_checked(
                frames.data_ptr() if frames.numel() else 16, frames.numel(), frame_off.data_ptr(),
                min(frames.numel() // n, 0xFFFFFFFF), n, window, dup.data_ptr(), dev.index or 0,
                _stream_ptr(stream, dev)))
            if check and bool((dup == _native.DUP_BAD_OFFSETS).any()):
                raise ValueError("frame_off must be non-decreasing offsets inside frames")
        return dup
    dup = torch.empty((n,), dtype=torch.uint8, device=dev)
    if n:
        _native.check(_native.lib().rudp_dedup_window(
            frames.data_ptr() if frames.numel() else None, off_ptr, F, n, window, dup.data_ptr(),
            dev.index or 0, _stream_ptr(stream, dev)))
    return dup
