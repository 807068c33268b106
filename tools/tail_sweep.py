"""Small-tile launch tail and tiles-per-CU caps of the fixed-length encode (C3 work).

A launch of 1M x 64 B packets is 8192 tiles of 128 packets, about 5.3 waves of
the ~1500 tiles resident at once (tools/tile_timeline.py): the last, partial
wave runs with the GPU part idle, 6-7 us of a 26 us launch.  Here the launch's
last `tail` packets go in tiles of tail_T packets (rudpx_tune 55 / 56), which
are dispatched last and spread that wave's work over every CU.  Interleaved
A/B with 8 rotating buffer sets (as the bench), median of repeats; every
variant's frames are compared with the default's.

usage: python tools/tail_sweep.py [--L 64] [--reps 15] [--percu 0,5,6]
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

from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=64)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--tails", default="0,16384,32768,65536,98304,131072,196608")
    ap.add_argument("--tail-T", default="16,32,64")
    ap.add_argument("--percu", default="-1")
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--persist", default="0", help="workgroups per CU of a persistent launch (rudpx_tune 57; 0 = off)")
    args = ap.parse_args()
    lib = _native.tools_lib()
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, args.L
    sets = []
    for _ in range(args.sets):
        tab, pay = batch.synth_batch(n, L, 0x5EED0003, device=dev)
        sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
    cur = [0]

    def enc():
        tab, pay, fr = sets[cur[0] % len(sets)]
        cur[0] += 1
        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)

    variants = {}
    for ps in (int(x) for x in args.persist.split(",")):
        for pc in (int(x) for x in args.percu.split(",")):
            for tail in (int(x) for x in args.tails.split(",")):
                for tT in ((32,) if tail == 0 else (int(x) for x in args.tail_T.split(","))):
                    variants[f"persist{ps}_percu{pc}_tail{tail}_T{tT}"] = (pc, tail, tT, ps)

    def apply(v):
        pc, tail, tT, ps = v
        lib.rudpx_tune(6, pc)
        lib.rudpx_tune(55, tail)
        lib.rudpx_tune(56, tT)
        lib.rudpx_tune(57, ps)

    # bit-exact against the default form
    apply((-1, 0, 32, 0))
    tab, pay, fr = sets[0]
    batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
    want = fr.clone()
    for name, v in variants.items():
        apply(v)
        fr.fill_(0)
        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        if not torch.equal(fr, want):
            raise SystemExit(f"{name}: frames differ from the default form")
    times = {k: [] for k in variants}
    for _ in range(args.reps):
        for name, v in variants.items():
            apply(v)
            for _ in range(3):
                enc()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                enc()
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / 20)
    apply((-1, 0, 32, 0))
    med = {k: statistics.median(v) for k, v in times.items()}
    alg = n * (2 * L + 12)
    out = {"L": L, "n": n, "buffer_sets": args.sets, "reps": args.reps,
           "ms": med, "roofline_frac": {k: alg / (v * 1e-3) / 8e12 for k, v in med.items()},
           "best": min(med, key=med.get)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
