"""Dedup window pass: LDS hash table (rudpx_tune 32 = 1) vs window scan (0).

usage: python tools/dedup_sweep.py [--reps 15]
Kernel-only timing (HIP events around rudp_dedup_window through the C ABI, no
Python bounds checks) on 1M one-character datagrams (the bench leg's frames)
and 1M x 64 B fixed frames with 10% retransmissions; results checked equal.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    n = 1 << 20
    tab, pay = batch.synth_batch(n, 1, 0x5EED0004, device=dev)
    enc = batch.pack_batch_varlen(tab, pay.view(-1), torch.ones(n, dtype=torch.int32, device=dev), "rudp5")
    tab64, pay64 = batch.synth_batch(n, 64, 0x5EED0005, device=dev)
    fr64, _ = batch.pack_batch(tab64, pay64, "rudp7")
    src = torch.randint(0, n, (n // 10,), device=dev)
    dst = torch.clamp(src + torch.randint(1, 400, (n // 10,), device=dev), max=n - 1)
    fr64[dst] = fr64[src]
    cases = {"1char_varlen": (enc.frames, enc.frame_off), "64B_fixed_10pct_dups": (fr64, None)}
    out = {}
    for name, (frames, off) in cases.items():
        for window in (500, 4096):
            res = {}
            for table in (1, 0):
                lib.rudpx_tune(32, table)
                want = batch.detect_retransmissions(frames, frame_off=off, window=window)
                times = []
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(5):
                        batch.detect_retransmissions(frames, frame_off=off, window=window)
                    b.record()
                    b.synchronize()
                    times.append(a.elapsed_time(b) / 5)
                res[table] = (statistics.median(times), want)
            lib.rudpx_tune(32, 1)
            same = bool(torch.equal(res[1][1], res[0][1]))
            out[f"{name}_w{window}"] = {"table_ms": res[1][0], "scan_ms": res[0][0], "equal": same,
                                        "dups": int(res[1][1].sum())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
