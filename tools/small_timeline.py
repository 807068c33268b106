"""Timeline of the small-frame varlen encode (1M one-character datagrams).

Each tile of the framing kernel records (rudpx_encode_trace) its start, the
time its base is known, its end and its XCD.  A one-lane stamp kernel
brackets the call (pass 1 + framing).  For 2 and 4 packets per thread prints
the call's span between the stamps, the framing kernel's span, and per-tile
percentiles of: start, base known, end (us from the first start).

usage: python tools/small_timeline.py [--L 1] [--n 1048576]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402

TICK_US = 0.01


def pct(x):
    return {p: round(float(np.percentile(x, p)), 2) for p in (0, 50, 90, 100)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_encode_trace.argtypes = [ctypes.c_void_p]
    lib.rudpx_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    n, L, H = args.n, args.L, 7
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    total = n * L
    tab, pay = batch.synth_batch(n, max(L, 16), 0x5EED000B, device=dev)
    flat = pay.view(-1)[:total].contiguous()
    frames = torch.empty(total + n * H, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    stamps = torch.zeros(4, dtype=torch.int64, device=dev)
    b = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                          flags=tab.flags.data_ptr(), payload=flat.data_ptr(), len=lens.data_ptr(), payload_off=None)

    def enc():
        _native.check(lib.rudp_encode_varlen_checked(ctypes.byref(b), total, frames.data_ptr(), frames.numel(),
                                                     off.data_ptr(), None, st.data_ptr(), H, 0, stream))
    forms = {"fpt4": 4, "fpt2": 2}
    out = {}
    old = lib.rudpx_tune(47, 0)
    for name, fpt in forms.items():
        lib.rudpx_tune(47, fpt)
        tiles = (n + 256 * fpt - 1) // (256 * fpt)
        buf = torch.zeros(tiles * 4, dtype=torch.int64, device=dev)
        runs = []
        for rep in range(4):
            for _ in range(3):
                enc()
            lib.rudpx_stamp(stamps.data_ptr(), stream)
            lib.rudpx_encode_trace(buf.data_ptr())
            enc()
            lib.rudpx_encode_trace(None)
            lib.rudpx_stamp(stamps[2:].data_ptr(), stream)
            torch.cuda.synchronize()
            assert int(st.item()) == 0
            r = buf.view(-1, 4).cpu().numpy().astype(np.int64)
            s0 = stamps.cpu().numpy()
            base = r[:, 0].min()
            rel = lambda c: (r[:, c] - base) * TICK_US  # noqa: E731
            runs.append({
                "call_span_us": float((s0[2] - s0[0]) * TICK_US),
                "stamp_to_first_tile_us": float((base - s0[0]) * TICK_US),
                "kernel_span_us": float(rel(2).max()),
                "start": pct(rel(0)),
                "base_known": pct(rel(1)),
                "end": pct(rel(2)),
                "tile_us": pct(rel(2) - rel(0)),
            })
        out[name] = {"tiles": tiles, "runs": runs}
        print(f"{name} done", file=sys.stderr, flush=True)
    lib.rudpx_tune(47, old)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
