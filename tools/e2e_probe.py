"""Where the host-memory (*_host) calls spend their time: the raw C-ABI call
with pinned outputs, the same with pageable outputs, and the Python entry
(which allocates its per-packet outputs from torch's caching pinned allocator,
or takes them from reuse=), for 1M one-character rudp5 datagrams (decode
and encode, packed) and 1M x 1472 B rudp7 frames (decode + UTF-8).

usage: python tools/e2e_probe.py [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def pinned(k, dt):
    return torch.empty(k, dtype=dt, pin_memory=True).numpy()


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    lib = _native.lib()
    out = {}
    m = 1 << 20
    rng = np.random.default_rng(1)
    seq, ack, flg = pinned(m, torch.uint16), pinned(m, torch.uint16), pinned(m, torch.uint8)
    seq[:] = np.arange(m, dtype=np.uint16)
    ack[:] = rng.integers(0, 1 << 16, m, dtype=np.uint16)
    flg[:] = 0x40
    pay = pinned(m, torch.uint8)
    pay[:] = rng.integers(0x20, 0x7F, m, dtype=np.uint8)
    lens = pinned(m, torch.int32)
    lens[:] = 1
    enc = batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True)
    fr, fo, cs = pinned(enc.frames.size, torch.uint8), pinned(m + 1, torch.int64), pinned(m, torch.uint16)
    fr[:], fo[:], cs[:] = enc.frames, enc.frame_off, enc.csum
    outs_p = [pinned(m, torch.uint16), pinned(m, torch.uint16), pinned(m, torch.uint8), pinned(m, torch.uint8),
              pinned(m, torch.uint16), pinned(m, torch.uint8)]
    outs_u = [np.empty(m, np.uint16), np.empty(m, np.uint16), np.empty(m, np.uint8), np.empty(m, np.uint8),
              np.empty(m, np.uint16), np.empty(m, np.uint8)]
    st = np.zeros(1, np.uint32)

    def dec_raw(o):
        return lambda: _native.check(lib.rudp_decode_varlen_host(
            fr.ctypes.data, fr.size, fo.ctypes.data, 6, m, cs.ctypes.data, *[a.ctypes.data for a in o],
            st.ctypes.data, 5, 0))
    out["decode_varlen_1M_1char"] = {
        "raw_pinned_out_ms": med(dec_raw(outs_p), args.reps),
        "raw_pageable_out_ms": med(dec_raw(outs_u), args.reps),
        "python_entry_ms": med(lambda: batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True), args.reps)}
    prev = batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True)
    out["decode_varlen_1M_1char"]["python_entry_reuse_ms"] = med(
        lambda: batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True, reuse=prev), args.reps)
    fo_out = pinned(m + 1, torch.int64)
    cs_out = pinned(m, torch.uint16)
    b = _native.RudpBatch(n=m, payload_len=1, reserved=0, seq=seq.ctypes.data, ack=ack.ctypes.data,
                          flags=flg.ctypes.data, payload=pay.ctypes.data, len=lens.ctypes.data, payload_off=None)
    out["encode_varlen_1M_1char"] = {
        "raw_pinned_out_ms": med(lambda: _native.check(lib.rudp_encode_varlen_host(
            ctypes.byref(b), m, fr.ctypes.data, fr.size, fo_out.ctypes.data, cs_out.ctypes.data, 5, 0)), args.reps),
        "python_entry_ms": med(lambda: batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True,
                                                               out=fr), args.reps)}
    del fr, fo, cs
    n, L = 1 << 20, 1472
    tab, p = batch.synth_batch(n, L, 0x5EED0004, device=torch.device("cuda", 0))
    frames_d, _ = batch.pack_batch(tab, p, 7)
    frames = pinned((n, L + 7), torch.uint8)
    frames[:] = frames_d.cpu().numpy()
    del frames_d, p, tab
    o16 = [pinned(n, torch.uint16) for _ in range(3)]
    o8 = [pinned(n, torch.uint8) for _ in range(3)]

    def fixed_raw(valid):
        return lambda: _native.check(lib.rudp_decode_host(
            frames.ctypes.data, L + 7, n, None, o16[0].ctypes.data, o16[1].ctypes.data, o8[0].ctypes.data,
            o8[1].ctypes.data, o16[2].ctypes.data, None, o8[2].ctypes.data if valid else None, 7, 0))
    out["decode_1Mx1472"] = {
        "raw_pinned_out_ms": med(fixed_raw(False), args.reps),
        "raw_pinned_out_utf8_ms": med(fixed_raw(True), args.reps),
        "python_entry_utf8_ms": med(lambda: batch.unpack_batch(frames, 7, utf8=True), args.reps),
        "h2d_GBs_at_raw_utf8": n * (L + 7) / 1e9}
    out["decode_1Mx1472"]["h2d_GBs_at_raw_utf8"] /= out["decode_1Mx1472"]["raw_pinned_out_utf8_ms"] / 1e3
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
