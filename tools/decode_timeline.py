"""Timeline of the fused decode + UTF-8 tiles (diagnostics build): every tile
records (rudpx_encode_trace) its start, the end of its staging barrier, the end
of its sums, its end, XCD and CU.  Reports how a CU's resident tiles spread
over the phases: the share of time a CU has k tiles staging (HBM) and j tiles
checking (VALU), and whether the phases of a CU's tiles move in step.

usage: python tools/decode_timeline.py [--L 1472] [--text] [--runs 3]
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("RUDP_LIB", str(REPO / "reliable-udp_amd" / "rudp" / "librudp_tools.so"))
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def text_frames(n, L, dev):
    text = ("é中😀aßЖ€𝄞" * (L // 8 + 8)).encode()[:L]
    while True:
        try:
            text.decode()
            break
        except UnicodeDecodeError:
            text = text[:-1]
    text += b"x" * (L - len(text))
    return torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev).expand(n, L).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--text", action="store_true")
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    lib = _native.lib()
    lib.rudpx_encode_trace.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    tab, pay = batch.synth_batch(args.n, args.L, 0x5EED0004, device=dev)
    if args.text:
        pay = text_frames(args.n, args.L, dev)
    fr, _ = batch.pack_batch(tab, pay, 7)
    for _ in range(5):
        batch.unpack_batch(fr, 7, utf8=True)
    torch.cuda.synchronize()
    blocks_max = args.n  # more than enough records
    buf = torch.zeros(6 * blocks_max, dtype=torch.int64, device=dev)
    out = {"L": args.L, "n": args.n, "text": args.text, "runs": []}
    for _ in range(args.runs):
        buf.zero_()
        lib.rudpx_encode_trace(buf.data_ptr())
        batch.unpack_batch(fr, 7, utf8=True)
        torch.cuda.synchronize()
        lib.rudpx_encode_trace(None)
        rec = buf.view(-1, 6).cpu().numpy()
        rec = rec[rec[:, 0] != 0]
        t0 = rec[:, 0].min()
        start, staged, summed, end = [(rec[:, i] - t0).astype(np.int64) for i in range(4)]
        cu = rec[:, 4] * 1000 + rec[:, 5]
        span = int(end.max())
        stage_d, sum_d, check_d = staged - start, summed - staged, end - summed
        # per CU, per 10-ns tick: tiles staging / tiles past staging (sums + checks)
        hist = collections.Counter()
        insync = []
        for c in np.unique(cu):
            m = cu == c
            ticks = np.zeros((span + 2, 2), np.int32)
            # +1 at an interval's start, -1 at its end, then a running sum
            np.add.at(ticks[:, 0], start[m], 1)
            np.add.at(ticks[:, 0], staged[m], -1)
            np.add.at(ticks[:, 1], staged[m], 1)
            np.add.at(ticks[:, 1], end[m], -1)
            ticks = np.cumsum(ticks, axis=0)
            codes = np.bincount(np.minimum(ticks[:, 0], 15) * 16 + np.minimum(ticks[:, 1], 15), minlength=256)
            for code in np.nonzero(codes)[0]:
                hist[(int(code) // 16, int(code) % 16)] += int(codes[code])
            # in step: how often a tile of this CU finishes staging within 1 us of another's
            st = np.sort(staged[m])
            if len(st) > 1:
                insync.append(float(np.mean(np.diff(st) < 100)))
        tot = sum(hist.values())
        busy_share = {f"staging{k}_checking{j}": round(v / tot, 4) for (k, j), v in sorted(hist.items()) if v / tot >= 0.005}
        out["runs"].append({
            "tiles": int(len(rec)), "span_us": span / 100.0,
            "stage_us_median": float(np.median(stage_d)) / 100.0, "sums_us_median": float(np.median(sum_d)) / 100.0,
            "check_us_median": float(np.median(check_d)) / 100.0,
            "cu_time_share": busy_share,
            "cu_time_no_tile_checking": round(sum(v for (k, j), v in hist.items() if j == 0) / tot, 4),
            "staged_within_1us_of_previous_on_cu": round(float(np.mean(insync)), 3) if insync else None,
        })
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
