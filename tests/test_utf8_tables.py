"""The strict UTF-8 table check of csrc/utf8_device.hpp, emulated on the CPU
instruction by instruction (v_perm_b32, v_bitop3_b32, v_alignbyte_b32,
v_alignbit_b32 on 32-bit lanes), against CPython's strict decoder: every 1-
and 2-byte payload, every 3- to 5-byte payload over an alphabet of the class
boundaries at each alignment in the dword, and random corrupted text.

The reference judges each payload with bytes.decode() (utils/packet.py:73,
called per datagram at utils/reliableUDP.py:121); the GPU tests compare the
kernels with the reference's own get_payload() outcomes, this one pins the
table constants and bit tricks the kernels are built from, without a GPU.
"""
from __future__ import annotations

import itertools
import re
from pathlib import Path

import numpy as np

HDR = Path(__file__).resolve().parent.parent / "reliable-udp_amd" / "csrc" / "utf8_device.hpp"
M32 = np.uint64(0xFFFFFFFF)

# the constants of utf8_pre_from / utf8_dword_errors (asserted to be the header's below)
T1 = (0x8B170121, 0x40404040)        # perm(S0, S1): t1, entries 0-3 from S1
T2_HI = (0xCBCBDBCB, 0xCBCBCBCB)     # low-nibble table, nibbles 8-15
T2_LO = (0xCBCBCB4B, 0x434363E7)     # nibbles 0-7
T3 = (0x01010101, 0x78786CE4)
SEL_MASK = 0x0B090A08


def test_constants_are_the_headers():
    text = HDR.read_text()
    for s0, s1 in (T1, T2_HI, T2_LO, T3):
        assert re.search(rf"perm\(0x{s0:08X}u, 0x{s1:08X}u", text), hex(s0)
    assert "0x0B090A08u" in text and "0x8A)" in text and "0x80)" in text
    assert "alignbit(c.t1, p.t1, 11)" in text and "alignbit(c.t1, p.t1, 5)" in text
    assert "Utf8Pre{0x40404040u, 0x01010101u, 0x40404040u}" in text


def perm(s0, s1, sel):
    """v_perm_b32 on uint64 arrays holding u32 lanes."""
    s0 = np.broadcast_to(np.asarray(s0, np.uint64), np.shape(sel))
    s1 = np.broadcast_to(np.asarray(s1, np.uint64), np.shape(sel))
    comb = (s0 << np.uint64(32)) | s1
    out = np.zeros(np.shape(sel), np.uint64)
    for k in range(4):
        b = (sel >> np.uint64(8 * k)) & np.uint64(0xFF)
        pick = (comb >> (np.uint64(8) * np.minimum(b, 7))) & np.uint64(0xFF)
        sign_byte = {8: 1, 9: 3, 10: 5, 11: 7}
        r = np.where(b < 8, pick, np.uint64(0))
        for sv, byte in sign_byte.items():
            sgn = (comb >> np.uint64(8 * byte + 7)) & np.uint64(1)
            r = np.where(b == sv, sgn * np.uint64(0xFF), r)
        r = np.where(b >= 13, np.uint64(0xFF), r)
        out |= r << np.uint64(8 * k)
    return out


def bitop3(a, b, c, tt):
    a, b, c = (np.asarray(x, np.uint64) for x in (a, b, c))
    out = np.zeros(np.broadcast(a, b, c).shape, np.uint64)
    for idx in range(8):
        if tt >> idx & 1:
            ma = a if idx & 4 else ~a
            mb = b if idx & 2 else ~b
            mc = c if idx & 1 else ~c
            out |= ma & mb & mc
    return out & M32


def align(hi, lo, bits):
    return (((hi << np.uint64(32)) | lo) >> np.uint64(bits)) & M32


def pre(x):
    """utf8_pre(x): (t12, t3, t1)."""
    x4, x12, x8, xr4 = (x << np.uint64(4)) & M32, (x << np.uint64(12)) & M32, (x << np.uint64(8)) & M32, x >> np.uint64(4)
    sel_lo = x & np.uint64(0x07070707)
    m_lo = perm(x4, x12, np.full(x.shape, SEL_MASK, np.uint64))
    m_hi = perm(x, x8, np.full(x.shape, SEL_MASK, np.uint64))
    sel_c = bitop3(m_hi, xr4, 0x07070707, 0x80)
    sel_s = bitop3(m_hi, xr4, 0x07070707, 0x8A)
    t1 = perm(*T1, sel_c)
    t2 = bitop3(m_lo, perm(*T2_HI, sel_lo), perm(*T2_LO, sel_lo), 0xCA)
    return t1 & t2, perm(*T3, sel_s), t1


def dword_errors(c, p):
    t12 = align(c[0], p[0], 24)  # alignbyte 3
    must23 = bitop3(align(c[2], p[2], 11), align(c[2], p[2], 5), 0x40404040, 0xA8)
    return bitop3(t12, c[1], must23, 0x6A)


def device_valid(payloads: list[bytes]) -> np.ndarray:
    """Every payload checked as the window check does: dwords from the payload's
    start, zero bytes before it and after it (one zero dword past the end)."""
    n = max(len(p) for p in payloads)
    nd = (n + 3) // 4 + 1
    buf = np.zeros((len(payloads), nd * 4), np.uint8)
    for i, p in enumerate(payloads):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    dw = buf.view("<u4").astype(np.uint64)
    prev = tuple(np.full(len(payloads), v, np.uint64) for v in (0x40404040, 0x01010101, 0x40404040))
    assert all((a == b).all() for a, b in zip(prev, pre(np.zeros(len(payloads), np.uint64))))
    err = np.zeros(len(payloads), np.uint64)
    for k in range(nd):
        cur = pre(dw[:, k])
        err |= dword_errors(cur, prev)
        prev = cur
    return err == 0


def cpython_valid(p: bytes) -> bool:
    try:
        p.decode("utf-8")
        return True
    except UnicodeDecodeError:
        return False


def check(payloads):
    got = device_valid(payloads)
    want = np.array([cpython_valid(p) for p in payloads])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [payloads[i].hex() for i in bad[:8]]


def test_every_one_and_two_byte_payload():
    check([bytes([a]) for a in range(256)])
    check([bytes(t) for t in itertools.product(range(256), repeat=2)])


ALPHA = [0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC,
         0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xFF]


def test_short_sequences_at_every_alignment():
    for n in (3, 4):
        seqs = [bytes(t) for t in itertools.product(ALPHA, repeat=n)]
        for lead in range(4):  # the sequence at each byte offset of a dword
            check([b"a" * lead + s for s in seqs])


def test_five_byte_sequences_sampled():
    rng = np.random.default_rng(5)
    seqs = [bytes(rng.choice(ALPHA, 5).astype(np.uint8)) for _ in range(40000)]
    for lead in range(4):
        check([b"a" * lead + s for s in seqs])


def test_random_text_with_corruption():
    rng = np.random.default_rng(7)
    chars = [chr(c) for c in list(range(0x20, 0x7F)) + list(range(0x80, 0x800, 7)) +
             list(range(0x800, 0xD800, 97)) + list(range(0xE000, 0x10000, 89)) + list(range(0x10000, 0x110000, 997))]
    rows = []
    for k in range(6000):
        b = bytearray("".join(rng.choice(chars, 20)).encode()[:48])
        if k % 2:
            b[rng.integers(0, len(b))] = rng.integers(0, 256)
        rows.append(bytes(b))
    check(rows)


def window_rows_valid(payloads: list[bytes], GL: int) -> np.ndarray:
    """utf8_check_windows_rows's round structure emulated over equal-length
    payloads: lane g of a GL-lane group takes 16-B windows g, g + GL, ...; a
    window's bytes before are lane g - 1's last dword of the same round, or
    for lane 0 the carry (lane GL - 1's of the round before); a window past
    the end is a re-read of window V - 1 whose errors do not count; the lane
    holding window V - 1 checks a zero dword after it."""
    L = len(payloads[0])
    assert all(len(p) == L for p in payloads)
    n = len(payloads)
    V = (L + 15) // 16
    if V == 0:
        return np.ones(n, bool)
    buf = np.zeros((n, V * 16), np.uint8)
    for i, p in enumerate(payloads):
        buf[i, :L] = np.frombuffer(p, np.uint8)
    dw = buf.view("<u4").astype(np.uint64).reshape(n, V, 4)
    zero = tuple(np.full(n, x, np.uint64) for x in (0x40404040, 0x01010101, 0x40404040))
    carry = zero
    last = [zero] * GL
    err = np.zeros((GL, n), np.uint64)
    for r in range((V + GL - 1) // GL):
        p4s = []
        for g in range(GL):
            v = g + GL * r
            w = dw[:, min(v, V - 1)]
            ps = [pre(w[:, k]) for k in range(4)]
            p0 = p4s[g - 1] if g else carry
            e = dword_errors(ps[0], p0) | dword_errors(ps[1], ps[0]) | dword_errors(ps[2], ps[1]) | \
                dword_errors(ps[3], ps[2])
            if v < V:
                err[g] |= e
            last[g] = ps[3]
            p4s.append(ps[3])
        carry = p4s[GL - 1]
    gl = (V - 1) % GL
    err[gl] |= dword_errors(zero, last[gl])
    return (err == 0).all(axis=0)


def test_window_rounds_and_carries_every_group_size():
    """The lane-group window check's rounds, carries, clamped re-reads and end
    check (csrc/utf8_device.hpp utf8_check_windows_rows) give CPython's answer
    for payloads of every length up to 300 B in groups of 1, 2, 4, 8 and 16
    lanes: multi-byte text, corrupted at a random byte, cut mid-character,
    or ASCII."""
    rng = np.random.default_rng(11)
    text = ("é中😀aßЖ€𝄞" * 60).encode()
    for L in list(range(1, 70)) + list(range(70, 301, 7)):
        rows = []
        for k in range(48):
            b = bytearray(text[:L].decode("utf-8", "ignore").encode())
            b += b"q" * (L - len(b))
            if k % 4 == 1:
                b[rng.integers(0, L)] = int(rng.integers(0x80, 0x100))
            elif k % 4 == 2:
                b[-1] = 0xE2
            elif k % 4 == 3:
                b = bytearray(b"x" * L)
            rows.append(bytes(b))
        want = np.array([cpython_valid(r) for r in rows])
        for GL in (1, 2, 4, 8, 16):
            assert np.array_equal(window_rows_valid(rows, GL), want), (L, GL)
