"""ctypes binding of librudp.so (C ABI declared in include/rudp.h).

There is no CPU fallback behind this module: if the library is missing, or a
compute entry point is called without a HIP device, the call raises.  The
library is loaded after ``torch`` so that it binds to the HIP runtime torch
already has in the process (same soname, libamdhip64.so.7) and device
pointers / streams from torch are valid in it.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

# RUDP_LIB names another build of the same ABI (A/B timing of two builds in one
# GPU call, tools/ only); the default is the in-tree build.
LIB_PATH = Path(os.environ.get("RUDP_LIB") or Path(__file__).resolve().parent / "librudp.so")
# The diagnostics build of the same sources (RUDP_TOOLS=1): the same ABI plus the
# rudpx_* sweep knobs, tile timelines and copy ceilings, for tools/ and the tests
# of the non-default kernel forms.  Never loaded by the product path on its own.
TOOLS_LIB_PATH = Path(os.environ.get("RUDP_TOOLS_LIB") or Path(__file__).resolve().parent / "librudp_tools.so")

LAYOUT_RUDP5 = 5
LAYOUT_RUDP7 = 7
OK_BAD_CSUM, OK_GOOD, OK_SHORT, OK_UNVERIFIED, OK_BAD_OFFSETS = 0, 1, 2, 3, 4
EINVAL, ENOMEM, ENOTSUP, EHIP_BASE = -22, -12, -95, -1000
ABI_VERSION = 7
# status bits of the sync-free varlen calls (RUDP_ST_*)
ST_LEN, ST_PAYLOAD, ST_FRAMES_CAP, ST_OFFSETS = 1, 2, 4, 8
DUP_BAD_OFFSETS = 2  # rudp_dedup_window_checked: a frame whose offsets were rejected

# Every symbol include/rudp.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "rudp_encode", "rudp_decode", "rudp_encode_host", "rudp_decode_host",
    "rudp_synth", "rudp_device_count", "rudp_last_error", "rudp_abi_version",
    "rudp_encode_varlen", "rudp_validate_utf8", "rudp_dedup_window",
    "rudp_udp_recv_batch", "rudp_udp_send_batch", "rudp_varlen_bounds", "rudp_frame_off_bounds",
    "rudp_encode_varlen_checked", "rudp_decode_varlen_checked", "rudp_frame_off_check",
    "rudp_udp_recv_batch_from", "rudp_udp_send_batch_to", "rudp_dedup_window_checked",
    "rudp_decode_utf8", "rudp_decode_varlen_utf8",
    "rudp_dedup_stream_create", "rudp_dedup_stream_push", "rudp_dedup_stream_counts", "rudp_dedup_stream_destroy",
    "rudp_decode_varlen_host", "rudp_encode_varlen_host",
)


class RudpBatch(ctypes.Structure):
    """struct rudp_batch (include/rudp.h)."""
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("payload_len", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("seq", ctypes.c_void_p),
        ("ack", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
        ("payload", ctypes.c_void_p),
        ("len", ctypes.c_void_p),
        ("payload_off", ctypes.c_void_p),
    ]


class RudpError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"librudp error {code}: {message}")
        self.code = code


_lock = threading.Lock()
_lib = None        # the library the batch API calls (librudp.so unless tools_lib() switched it)
_product = None
_tools = None


def _declare(lib: ctypes.CDLL) -> None:
    P, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "rudp_encode": [ctypes.POINTER(RudpBatch), P, P, I, I, P],
        "rudp_decode": [P, P, U32, U64, P, P, P, P, P, P, P, I, I, P],
        "rudp_encode_host": [ctypes.POINTER(RudpBatch), P, P, I, I],
        "rudp_decode_host": [P, U32, U64, P, P, P, P, P, P, P, P, I, I],
        "rudp_decode_varlen_host": [P, U64, P, U32, U64, P, P, P, P, P, P, P, P, I, I],
        "rudp_encode_varlen_host": [ctypes.POINTER(RudpBatch), U64, P, U64, P, P, I, I],
        "rudp_synth": [U64, U64, U64, U32, I, P, P, P, P, I, P],
        "rudp_encode_varlen": [ctypes.POINTER(RudpBatch), P, P, P, I, I, P],
        "rudp_validate_utf8": [P, P, U32, U64, I, P, I, P],
        "rudp_dedup_window": [P, P, U32, U64, U32, P, I, P],
        "rudp_dedup_window_checked": [P, U64, P, U32, U64, U32, P, I, P],
        "rudp_udp_recv_batch": [I, P, U64, U32, U32, P, I],
        "rudp_udp_send_batch": [I, P, P, U64, ctypes.c_char_p, ctypes.c_uint16],
        "rudp_udp_recv_batch_from": [I, P, U64, U32, U32, P, P, I],
        "rudp_udp_send_batch_to": [I, P, P, U64, P, I],
        "rudp_varlen_bounds": [P, P, U64, P, I, P],
        "rudp_frame_off_bounds": [P, U64, P, I, P],
        "rudp_encode_varlen_checked": [ctypes.POINTER(RudpBatch), U64, P, U64, P, P, P, I, I, P],
        "rudp_decode_varlen_checked": [P, U64, P, U32, U64, P, P, P, P, P, P, P, I, I, P],
        "rudp_decode_utf8": [P, P, U32, U64, P, P, P, P, P, P, P, P, I, I, P],
        "rudp_decode_varlen_utf8": [P, U64, P, U32, U64, P, P, P, P, P, P, P, P, I, I, P],
        "rudp_frame_off_check": [P, U64, U64, P, I, P],
        "rudp_dedup_stream_create": [U32, U32, U32, I, P, ctypes.POINTER(ctypes.c_void_p)],
        "rudp_dedup_stream_push": [P, P, P, U64, P, P],
        "rudp_dedup_stream_counts": [P, P],
        "rudp_dedup_stream_destroy": [P],
        "rudp_device_count": [ctypes.POINTER(ctypes.c_int)],
        "rudp_abi_version": [],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.rudp_last_error.argtypes = []
    lib.rudp_last_error.restype = ctypes.c_char_p


def _load(path: Path) -> ctypes.CDLL:
    if not path.exists():
        raise RuntimeError(
            f"{path} is missing: build it with "
            "`python reliable-udp_amd/rudp/_build.py` (or __graft_entry__.build())")
    import torch  # noqa: F401  -- bind to torch's HIP runtime first
    handle = ctypes.CDLL(str(path))
    _declare(handle)
    if handle.rudp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path.name} ABI version mismatch; rebuild it")
    return handle


def lib() -> ctypes.CDLL:
    """The library the batch API calls: librudp.so, loaded once per process
    (raises if it was not built), unless tools_lib() made the diagnostics build
    the active one."""
    global _lib, _product
    if _lib is not None:
        return _lib
    with _lock:
        if _product is None:
            _product = _load(LIB_PATH)
        if _lib is None:
            _lib = _product
    return _lib


def tools_lib(activate: bool = True) -> ctypes.CDLL:
    """The diagnostics build librudp_tools.so (rudpx_tune, rudpx_encode_trace,
    rudpx_stamp, rudpx_copy*).  ``activate``: the batch API calls it too until
    use_product() (its knobs only act on calls made through it)."""
    global _lib, _tools
    with _lock:
        if _tools is None:
            h = _load(TOOLS_LIB_PATH)
            P, I, U32, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
            for name, args in {"rudpx_tune": [I, I], "rudpx_encode_trace": [P], "rudpx_stamp": [P, P],
                               "rudpx_copy": [P, P, U64, U32, P], "rudpx_copy_vpt": [P, P, U64, I, I, P],
                               "rudpx_copy_tile": [P, P, U64, U32, U32, P],
                               "rudpx_copy_tile_dma": [P, P, U64, U32, U32, U32, I, P],
                               "rudpx_copy_tile_pipe": [P, P, U64, U32, U32, U32, P],
                               "rudpx_scratch_stats": [I, P]}.items():
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = I
            _tools = h
        if activate:
            _lib = _tools
    return _tools


def use_product() -> None:
    """Make librudp.so the library the batch API calls again."""
    global _lib
    with _lock:
        _lib = _product


def check(rc: int) -> None:
    """Map a librudp return code to a Python exception."""
    if rc == 0:
        return
    msg = (lib().rudp_last_error() or b"").decode(errors="replace")
    if rc in (EINVAL, ENOTSUP):
        raise ValueError(f"librudp: {msg}")
    if rc == ENOMEM:
        raise MemoryError(f"librudp: {msg}")
    raise RudpError(rc, msg)


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().rudp_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
