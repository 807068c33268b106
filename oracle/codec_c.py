"""ORACLE (test infrastructure): ctypes wrapper of codec_ref.c (built by make)."""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libcodec_ref.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        _lib = ctypes.CDLL(str(LIB))
        P, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        _lib.oracle_encode.argtypes = [P, P, P, P, U64, U32, I, P, P]
        _lib.oracle_encode.restype = None
        _lib.oracle_decode.argtypes = [P, U64, U32, I, P, P, P, P, P, P]
        _lib.oracle_decode.restype = None
        _lib.oracle_inet_checksum.argtypes = [P, ctypes.c_size_t]
        _lib.oracle_inet_checksum.restype = ctypes.c_uint16
    return _lib


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def encode(seq, ack, flags, payload, layout):
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    n, L = payload.shape
    seq = np.ascontiguousarray(seq, dtype=np.uint16)
    ack = np.ascontiguousarray(ack, dtype=np.uint16)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    frames = np.empty((n, L + layout), np.uint8)
    csum = np.empty(n, np.uint16)
    lib().oracle_encode(_p(seq), _p(ack), _p(flags), _p(payload), n, L, layout, _p(frames), _p(csum))
    return frames, csum


def decode(frames, layout, csum_in=None):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    n, F = frames.shape
    seq, ack = np.empty(n, np.uint16), np.empty(n, np.uint16)
    flags, ok, cs = np.empty(n, np.uint8), np.empty(n, np.uint8), np.empty(n, np.uint16)
    ci = np.ascontiguousarray(csum_in, dtype=np.uint16) if csum_in is not None else None
    lib().oracle_decode(_p(frames), n, F, layout, _p(ci), _p(seq), _p(ack), _p(flags), _p(ok), _p(cs))
    return seq, ack, flags, ok, cs


def inet_checksum(data: bytes) -> int:
    buf = np.frombuffer(bytes(data), np.uint8)
    return int(lib().oracle_inet_checksum(_p(buf), len(data)))
