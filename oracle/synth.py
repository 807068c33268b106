"""ORACLE (test infrastructure): numpy restatement of rudp_synth.

Must match reliable-udp_amd/csrc/synth.hip bit for bit.  Definition
(SURVEY.md §8d), for global packet index i:
  key_k   = stream(seed, k), k = 0..3
  isn     = 1 + stream(key_0, 0) mod 5000      (utils/reliableUDP.py:41)
  seq     = (isn + i) mod 2^16                   (utils/reliableUDP.py:54)
  ack     = stream(key_1, i) mod 2^16
  flags   = FLAGS6[(stream(key_2, i) >> 32) * 6 >> 32]
  payload = LE bytes of stream(key_3, i*W + w), W = ceil(L/8), & 0x7F if ascii
with stream(k, c) = splitmix64_mix(k + (c + 1) * 0x9E3779B97F4A7C15) mod 2^64.
"""
from __future__ import annotations

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1
FLAGS6 = np.array([0x00, 0x80, 0x20, 0xA0, 0x40, 0x60], dtype=np.uint8)


def mix64_int(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * M1) & MASK64
    z = ((z ^ (z >> 27)) * M2) & MASK64
    return z ^ (z >> 31)


def stream_int(key: int, ctr: int) -> int:
    return mix64_int(key + (ctr + 1) * GAMMA)


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(M1)
        z ^= z >> np.uint64(27)
        z *= np.uint64(M2)
        z ^= z >> np.uint64(31)
    return z


def stream(key: int, ctr: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(key) + (ctr.astype(np.uint64) + np.uint64(1)) * np.uint64(GAMMA)
    return mix64(z)


def keys(seed: int):
    k = [stream_int(seed & MASK64, i) for i in range(4)]
    isn = 1 + stream_int(k[0], 0) % 5000
    return k, isn


def synth(seed: int, first: int, n: int, L: int, ascii: bool = True):
    """(seq u16[n], ack u16[n], flags u8[n], payload u8[n, L]) for packets first..first+n-1."""
    k, isn = keys(seed)
    idx = np.arange(first, first + n, dtype=np.uint64)
    seq = ((idx + np.uint64(isn)) & np.uint64(0xFFFF)).astype(np.uint16)
    ack = (stream(k[1], idx) & np.uint64(0xFFFF)).astype(np.uint16)
    hi = stream(k[2], idx) >> np.uint64(32)
    with np.errstate(over="ignore"):
        sel = (hi * np.uint64(6)) >> np.uint64(32)
    flags = FLAGS6[sel.astype(np.intp)]
    W = (L + 7) // 8
    if n == 0 or L == 0:
        return seq, ack, flags, np.zeros((n, L), np.uint8)
    words = np.arange(W, dtype=np.uint64)
    ctr = idx[:, None] * np.uint64(W) + words[None, :]
    x = stream(k[3], ctr)
    if ascii:
        x &= np.uint64(0x7F7F7F7F7F7F7F7F)
    payload = x.astype("<u8").view(np.uint8).reshape(n, W * 8)[:, :L]
    return seq, ack, flags, np.ascontiguousarray(payload)
