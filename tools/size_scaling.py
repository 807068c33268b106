"""Time per launch against batch size (fixed cost vs per-packet cost).

usage: python tools/size_scaling.py [--L 64] [--reps 30]
For encode, verify-only decode and copy-out decode at 2^18..2^22 packets,
rotating buffer sets so every launch streams from HBM.  One JSON object.
"""
from __future__ import annotations

import argparse
import json
import math
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=64)
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = args.L
    out = {}
    for lg in (18, 19, 20, 21, 22):
        n = 1 << lg
        nsets = max(1, min(16, math.ceil((1 << 30) / (n * (2 * L + 20)))))
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
            batch.pack_batch(tab, pay, 7, out=fr)
            sets.append((tab, pay, fr))
        ops = {
            "encode": lambda s: batch.pack_batch(s[0], s[1], 7, out=s[2], want_csum=False),
            "verify": lambda s: batch.unpack_batch(s[2], 7),
            "copyout": lambda s: batch.unpack_batch(s[2], 7, copy_payload=True),
        }
        for name, fn in ops.items():
            for s in sets:
                fn(s)
            times = []
            for r in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for s in sets:
                    fn(s)
                b.record()
                b.synchronize()
                times.append(a.elapsed_time(b) / nsets)
            out[f"{name}_n{n}"] = {"ms": statistics.median(times), "us_per_Mpkt": statistics.median(times) * 1e3 / (n / 1e6)}
        del sets
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
