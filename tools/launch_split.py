"""Fixed-length encode of one batch as one launch or as several launches of
`encode_launch_packets` packets (rudpx_tune 48), and with the XCD-contiguous
tile order (key 5), at 1M and 16M x 1472 B (C4 / C5 shapes).

The 16M (C5) single launch ran ~5% slower per packet than 1M launches, while
the same 16M buffers encoded as 16 launches of 1M ran faster than either
(tools/cache_residency.py): a launch-length effect, not the address space.
usage: python tools/launch_split.py [--reps 9]
Per-packet ms (per 2^20 packets), medians of interleaved rounds; outputs
checked bit-exact against the single launch.
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
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--chunks", default="0,131072,262144,524288,1048576,2097152")
    args = ap.parse_args()
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    L = 1472
    out = {}
    for n in (1 << 20, 1 << 24):
        tab, pay = batch.synth_batch(n, L, 0x5EED0005, device=dev)
        fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
        ref = torch.empty_like(fr)
        batch.pack_batch(tab, pay, 7, out=ref, want_csum=False)
        variants = {f"chunk{c}": ((48, c), (5, 0)) for c in map(int, args.chunks.split(","))}
        variants["xcd_swizzle"] = ((48, 0), (5, 1))
        variants["xcd_swizzle_chunk1M"] = ((48, 1 << 20), (5, 1))
        times = {k: [] for k in variants}
        exact = {}
        reps = args.reps if n == 1 << 20 else max(3, args.reps // 3)
        for r in range(args.reps):
            for k, kv in variants.items():
                old = [(key, lib.rudpx_tune(key, v)) for key, v in kv]
                try:
                    batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)  # warm
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(reps):
                        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
                    b.record()
                    b.synchronize()
                    times[k].append(a.elapsed_time(b) / reps / (n / 2 ** 20))
                    if r == 0:
                        exact[k] = bool(torch.equal(fr, ref))
                finally:
                    for key, v in reversed(old):
                        lib.rudpx_tune(key, v)
        for k, v in times.items():
            ms = statistics.median(v)
            out[f"n{n}_{k}"] = {"ms_per_2^20": ms, "frac": (1 << 20) * (2 * L + 12) / ms / 1e9 / 8.0,
                                "exact": exact[k]}
            print(json.dumps({f"n{n}_{k}": out[f"n{n}_{k}"]}), flush=True)
        del tab, pay, fr, ref
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
