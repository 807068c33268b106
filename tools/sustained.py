"""Per-launch time across a long back-to-back run: does the rate sag?

A tile trace (tools/tile_timeline.py) of one 1M x 1472 B encode launch after
an idle period spans 481-486 us (6.6 TB/s, the copy ceiling), while the bench's
50 back-to-back launches average ~0.515 ms.  Here, after a 0.5 s idle, N
back-to-back launches each get an event pair; printed as means of groups of 5
launches, for the encode and for the streaming copy of the same bytes
(rudpx_copy_vpt), each run twice in alternation.

usage: python tools/sustained.py [--n 200]
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

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--variants", action="store_true",
                    help="also: a stamp kernel before every launch, the tile trace on")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.tools_lib()
    lib.rudpx_copy_vpt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p]
    L, M = args.L, 1 << 20
    tab, pay = batch.synth_batch(M, L, 0x5EED0004, device=dev)
    fr = torch.empty((M, L + 7), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    lib.rudpx_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.rudpx_encode_trace.argtypes = [ctypes.c_void_p]
    stamps = torch.zeros((4,), dtype=torch.int64, device=dev)
    tbuf = torch.zeros((M // 16 * 4,), dtype=torch.int64, device=dev)

    def enc():
        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)

    def enc_stamped():
        lib.rudpx_stamp(stamps.data_ptr(), stream)
        enc()

    def enc_traced():
        lib.rudpx_encode_trace(tbuf.data_ptr())
        enc()
        lib.rudpx_encode_trace(None)

    fns = {
        "encode": enc,
        "copy": lambda: lib.rudpx_copy_vpt(pay.data_ptr(), fr.data_ptr(), M * L // 16, 1, 1, stream),
    }
    if args.variants:
        fns.update({"encode_stamped": enc_stamped, "encode_traced": enc_traced})
    out = {}
    for rep in range(2):
        for name, fn in fns.items():
            fn()
            torch.cuda.synchronize()
            time.sleep(0.5)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.n)]
            for a, b in ev:
                a.record()
                fn()
                b.record()
            torch.cuda.synchronize()
            ts = [a.elapsed_time(b) for a, b in ev]
            groups = [round(sum(ts[i:i + 5]) / 5, 4) for i in range(0, len(ts), 5)]
            out[f"{name}_{rep}"] = {"ms_by_5": groups, "mean_ms": sum(ts) / len(ts),
                                    "first10_ms": sum(ts[:10]) / 10, "last50_ms": sum(ts[-50:]) / 50}
            print(f"{name}_{rep} done", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
