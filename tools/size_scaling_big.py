"""Encode time per packet at 1M..16M x 1472 B (is the 16M C5 shape slower per packet?).

usage: python tools/size_scaling_big.py [--reps 10]
One buffer set per size (>= 1.5 GB, far past the 256 MiB Infinity Cache).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--L", type=int, default=1472)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = args.L
    out = {}
    for lg in (20, 21, 22, 23, 24):
        n = 1 << lg
        tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
        fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        times = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        ms = statistics.median(times)
        out[f"n{n}"] = {"ms": ms, "us_per_Mpkt": ms * 1e3 / (n / 2 ** 20), "frac": n * (2 * L + 12) / ms / 1e9 / 8.0}
        print(json.dumps({f"n{n}": out[f"n{n}"]}), flush=True)
        del tab, pay, fr
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
