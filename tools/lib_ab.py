"""Interleaved A/B of the fixed-length encode across library builds.

Loads several builds of librudp (the product, the diagnostics build, an older
tree's build) side by side through ctypes and times rudp_encode of each on the
same buffers, round by round (median of --reps rounds of 10 launches), with
every build's frames compared byte for byte with the first's.

usage: python tools/lib_ab.py --libs name=path,... [--L 1472,1024,64]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--L", default="1472,1024,64")
    ap.add_argument("--reps", type=int, default=11)
    args = ap.parse_args()
    _native.lib()  # torch's HIP runtime first
    libs = {}
    for item in args.libs.split(","):
        name, path = item.split("=")
        h = ctypes.CDLL(str(REPO / path))
        h.rudp_encode.argtypes = [ctypes.POINTER(_native.RudpBatch), ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_encode.restype = ctypes.c_int
        libs[name] = h
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    for L in (int(x) for x in args.L.split(",")):
        n = 1 << 20
        nsets = max(1, min(8, math.ceil((1 << 30) / (n * (2 * L + 12)))))
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
            b = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                                  flags=tab.flags.data_ptr(), payload=pay.data_ptr(), len=None, payload_off=None)
            sets.append((tab, pay, fr, b))
        ref = None
        exact = {}
        for name, h in libs.items():
            _, _, fr, b = sets[0]
            fr.zero_()
            assert h.rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, stream) == 0
            got = fr.clone()
            ref = got if ref is None else ref
            exact[name] = bool(torch.equal(got, ref))
        times = {k: [] for k in libs}
        for _ in range(args.reps):
            for name, h in libs.items():
                for i in range(2):
                    _, _, fr, b = sets[i % nsets]
                    h.rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, stream)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(10):
                    _, _, fr, b = sets[i % nsets]
                    h.rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, stream)
                e.record()
                e.synchronize()
                times[name].append(s.elapsed_time(e) / 10)
        out[L] = {"ms": {k: statistics.median(v) for k, v in times.items()}, "exact": exact}
        print(L, out[L], file=sys.stderr, flush=True)
        del sets
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
