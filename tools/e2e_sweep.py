"""End-to-end (host memory in, host memory out) codec throughput sweep.

Times rudp_encode_host / rudp_decode_host on 1M x 1472 B over pipeline slot
counts and chunk sizes (rudpx_tune keys 8, 9), with pinned and pageable host
buffers.  PCIe-bound; the numbers go to DESIGN.md, never to bench `value`.
usage: python tools/e2e_sweep.py [--reps 3]
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

lib = _native.tools_lib()
lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
GIB = float(1 << 30)


def timed(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--L", type=int, default=1472)
    args = ap.parse_args()
    n, L = args.n, args.L
    dev = torch.device("cuda", 0)
    tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
    pin = lambda shape, dt: torch.empty(shape, dtype=dt, pin_memory=True)  # noqa: E731
    P = {"pay": pin((n, L), torch.uint8), "seq": pin((n,), torch.uint16),
         "ack": pin((n,), torch.uint16), "flags": pin((n,), torch.uint8),
         "out": pin((n, L + 7), torch.uint8)}
    P["pay"].copy_(pay)
    P["seq"].copy_(tab.seq)
    P["ack"].copy_(tab.ack)
    P["flags"].copy_(tab.flags)
    torch.cuda.synchronize()
    pinned = {k: v.numpy() for k, v in P.items()}
    pageable = {k: np.array(v) for k, v in pinned.items()}
    want, _ = batch.pack_batch(tab, pay, 7)
    want = want.cpu().numpy()
    res = {}
    for name, B in (("pinned", pinned), ("pageable", pageable)):
        for slots in (2, 3, 4):
            for mb in (8, 32, 128):
                lib.rudpx_tune(8, slots)
                lib.rudpx_tune(9, mb)

                def enc():
                    batch.pack_batch((B["seq"], B["ack"], B["flags"]), B["pay"], 7, out=B["out"])
                dt = timed(enc, args.reps)
                exact = bool(np.array_equal(B["out"], want))
                res[f"encode_{name}_s{slots}_mb{mb}"] = {
                    "ms": dt * 1e3, "payload_GiBs": n * L / dt / GIB,
                    "pcie_GBs_each_way": n * (L + 6) / dt / 1e9, "exact": exact}

                def dec():
                    batch.unpack_batch(B["out"], 7)
                dt = timed(dec, args.reps)
                res[f"decode_{name}_s{slots}_mb{mb}"] = {
                    "ms": dt * 1e3, "payload_GiBs": n * L / dt / GIB,
                    "pcie_GBs_h2d": n * (L + 7) / dt / 1e9}
            if name == "pageable":
                break
    # raw copy engines alone, for reference: one direction, then both at once
    d = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h2d = timed(lambda: (d.copy_(P["out"], non_blocking=True), torch.cuda.synchronize()), args.reps)
    d2h = timed(lambda: (P["out"].copy_(d, non_blocking=True), torch.cuda.synchronize()), args.reps)
    d2 = torch.empty_like(d)
    hbuf = pin((n, L + 7), torch.uint8)

    def both():
        with torch.cuda.stream(s1):
            d.copy_(P["out"], non_blocking=True)
        with torch.cuda.stream(s2):
            hbuf.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()
    bd = timed(both, args.reps)
    nb = n * (L + 7)
    res["raw_h2d_GBs"] = nb / h2d / 1e9
    res["raw_d2h_GBs"] = nb / d2h / 1e9
    res["raw_bidir_GBs_each_way"] = nb / bd / 1e9
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
