"""Checked varlen encode and decode-verify (the sync-free Python entries)
across length shapes: equal lengths at several hints and uniform ragged ones,
median of HIP-event pairs per call.  Run under two builds (RUDP_LIB) for an A/B.

usage: python tools/varlen_shapes.py [--reps 30] [--only L64,U0-512]
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

SHAPES = ("L64", "L256", "L512", "L1024", "L1472", "L4000", "U0-512", "U0-2944", "U0-8000")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--only", default="", help="comma-separated shape names")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    out = {}
    for name in (args.only.split(",") if args.only else SHAPES):
        n = args.n if not name.endswith("8000") and name != "L4000" else args.n // 4
        if name[0] == "U":
            hi = int(name.split("-")[1])
            lens = torch.randint(0, hi + 1, (n,), dtype=torch.int32, device=dev, generator=g)
        else:
            lens = torch.full((n,), int(name[1:]), dtype=torch.int32, device=dev)
        total = int(lens.sum().item())
        pay = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
        tab, _ = batch.synth_batch(n, 0, 0x5EED0009, device=dev)
        res = batch.pack_batch_varlen(tab, pay, lens, "rudp7", want_csum=False).check()
        frames = torch.empty_like(res.frames)
        for _ in range(3):
            batch.pack_batch_varlen(tab, pay, lens, "rudp7", want_csum=False, out=frames, check=False)
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch.pack_batch_varlen(tab, pay, lens, "rudp7", want_csum=False, out=frames, check=False)
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        ms = statistics.median(x.elapsed_time(y) for x, y in ts)
        alg = 2 * total + n * (7 + 4 + 5 + 8)
        same = bool(torch.equal(frames, res.frames))
        # decode-verify of the same frames (sync-free entry)
        want = batch.unpack_batch_varlen(res.frames, res.frame_off, "rudp7").ok
        for _ in range(3):
            batch.unpack_batch_varlen(res.frames, res.frame_off, "rudp7", check=False)
        td = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            d = batch.unpack_batch_varlen(res.frames, res.frame_off, "rudp7", check=False)
            b.record()
            td.append((a, b))
        torch.cuda.synchronize()
        ms_d = statistics.median(x.elapsed_time(y) for x, y in td)
        ok = bool(torch.equal(d.ok, want) and bool((want == 1).all().item()))
        out[name] = {"n": n, "ms": ms, "frac": alg / ms / 1e9 / 8.0, "exact_vs_first_call": same,
                     "decode_ms": ms_d, "decode_frac": (total + n * (7 + 16 + 8)) / ms_d / 1e9 / 8.0,
                     "decode_all_ok": ok}
        del lens, pay, tab, res, frames
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
