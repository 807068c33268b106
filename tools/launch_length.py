"""Why does a 16M x 1472 B launch encode faster per packet than a 1M launch?

Per launch (median of HIP-event pairs), interleaved round by round:
  own_1M        the headline: 1M packets in buffers of their own (1.55 GB each way)
  big_1M@k      1M-packet launches on slices of one 16M allocation (offset k x 1M)
  big_nM        one launch of n x 1M packets on the start of that allocation
  copy_own/big  the streaming copy (rudpx_copy_vpt) over the same byte counts
Separates the launch length (a fixed cost per launch) from the allocation the
buffers come from (page fragments).  Prints one JSON object.

With --orders, the same shapes with the XCD tile order on and off
(rudpx_tune 5).  The chunked and rotated orders of
profiles/r02/headline/xcd_orders.json were measured within 2% and removed.

usage: python tools/launch_length.py [--reps 12] [--rounds 3] [--orders]
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
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--orders", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L, M = args.L, 1 << 20
    F = L + 7
    tab1, pay1 = batch.synth_batch(M, L, 0x5EED0004, device=dev)
    out1 = torch.empty((M, F), dtype=torch.uint8, device=dev)
    tab16, pay16 = batch.synth_batch(16 * M, L, 0x5EED0005, device=dev)
    out16 = torch.empty((16 * M, F), dtype=torch.uint8, device=dev)
    lib = _native.tools_lib()
    lib.rudpx_copy_vpt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream

    def enc_slice(k, n):
        sl = slice(k * M, (k + n) * M)
        t = batch.HeaderTable(tab16.seq[sl], tab16.ack[sl], tab16.flags[sl])
        return lambda: batch.pack_batch(t, pay16[sl], 7, out=out16[sl], want_csum=False)

    def copy(src, dst, nbytes):
        return lambda: lib.rudpx_copy_vpt(src.data_ptr(), dst.data_ptr(), nbytes // 16, 1, 1, stream)

    nb1 = M * L
    own = lambda: batch.pack_batch(tab1, pay1, 7, out=out1, want_csum=False)  # noqa: E731
    cases = {}
    if args.orders:
        lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
        orders = {"contig": 1, "hw_rr": 0}

        def tuned(fn, mode):
            def run():
                lib.rudpx_tune(5, mode)
                fn()
            return run
        for oname, mode in orders.items():
            cases[f"{oname}/own_1M"] = (tuned(own, mode), 1)
            cases[f"{oname}/big_1M@15"] = (tuned(enc_slice(15, 1), mode), 1)
            cases[f"{oname}/big_16M"] = (tuned(enc_slice(0, 16), mode), 16)
    else:
        cases["own_1M"] = (own, 1)
        for k in (0, 5, 15):
            cases[f"big_1M@{k}"] = (enc_slice(k, 1), 1)
        for n in (2, 4, 8, 16):
            cases[f"big_{n}M"] = (enc_slice(0, n), n)
        cases["copy_own_1M"] = (copy(pay1, out1, nb1), 1)
        cases["copy_big_1M@5"] = (copy(pay16[5 * M:], out16[5 * M:], nb1), 1)
        cases["copy_big_16M"] = (copy(pay16, out16.view(-1)[: 16 * nb1], 16 * nb1), 16)

    per = {k: [] for k in cases}
    for r in range(args.rounds):
        for name, (fn, n) in cases.items():
            for _ in range(2):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps if n < 8 else max(3, args.reps // 4))]
            for a, b in ev:
                a.record()
                fn()
                b.record()
            torch.cuda.synchronize()
            per[name] += [a.elapsed_time(b) / n for a, b in ev]
        print(f"round {r} done", file=sys.stderr, flush=True)
    if args.orders:
        lib.rudpx_tune(5, -1)
    res = {}
    for name, ts in per.items():
        ts.sort()
        res[name] = {"ms_per_1M": statistics.median(ts), "min": ts[0], "max": ts[-1], "launches": len(ts)}
        if "copy" in name:
            res[name]["GBs"] = 2 * nb1 / (res[name]["ms_per_1M"] / 1e3) / 1e9
        else:
            res[name]["frac"] = M * (2 * L + 12) / (res[name]["ms_per_1M"] / 1e3) / 1e9 / 8000.0
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
