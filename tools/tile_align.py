"""Encode tile size x 64-B store alignment at 1M x 1472 B (interleaved A/B).

usage: python tools/tile_align.py [--L 1472] [--reps 11]"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd"), str(REPO / "tools")]

import torch  # noqa: E402

from rudp import batch  # noqa: E402
from sweep import interleaved, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--reps", type=int, default=11)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, args.L
    tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
    fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
    want, _ = batch.pack_batch(tab, pay, 7)
    variants = {}
    for tile in (4, 8, 16):
        for align in (0, 1):
            for per_cu in (-1, 0):
                def setup(tile=tile, align=align, per_cu=per_cu):
                    lib.rudpx_tune(2, tile)
                    lib.rudpx_tune(23, align)
                    lib.rudpx_tune(6, per_cu)
                variants[f"T{tile}_align{align}_percu{per_cu}"] = (
                    setup, lambda: batch.pack_batch(tab, pay, 7, out=fr, want_csum=False))
    res = interleaved(variants, args.reps)
    out = {}
    alg = n * (2 * L + 12)
    for k, (setup, fn) in variants.items():
        setup()
        got, _ = batch.pack_batch(tab, pay, 7)
        out[k] = {"ms": res[k], "frac": alg / res[k] / 1e9 / 8.0, "exact": bool(torch.equal(got, want))}
    lib.rudpx_tune(2, 0)
    lib.rudpx_tune(23, -1)
    lib.rudpx_tune(6, -1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
