"""Tile-phase timeline of the varlen encode tile kernel (encode_varlen_tile_kernel).

Every workgroup that frames a tile records (rudpx_encode_trace, tools build):
start, phase-1 loads landed, sums done, chunk map + header words done, end
(100 MHz wall clock), its XCD, its packet count, whether it was a byte tile and
took the fast phase 2, its frame bytes, and when its last wave finished its
sums, its map and its header chunks.  For each shape and form this
prints per-phase percentiles (us), the span, resident tiles, and the share of
tiles on the slow phase 2.

Shapes: 1M x 1472 B equal lengths and 1M lengths uniform in [0, 2944], each as
packet tiles (rudpx_tune 51 = 0) and byte tiles (51 = 2) -- the comparison
VERDICT r02 asked for: why byte tiles lose at equal lengths, where ragged
lengths lose against equal ones.

usage: python tools/varlen_timeline.py [--save DIR]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402

TICK_US = 0.01


def pct(x):
    return {p: round(float(np.percentile(x, p)), 3) for p in (10, 50, 90)} if len(x) else {}


def analyse(rec):
    rec = rec[rec[:, 0] != 0]
    t0, tl, ts, tm, te = (rec[:, i].astype(np.int64) for i in range(5))
    base = t0.min()
    s, e = (t0 - base) * TICK_US, (te - base) * TICK_US
    span = float(e.max())
    nb = int(span) + 2
    conc = np.zeros(nb + 1)
    np.add.at(conc, np.floor(s).astype(int), 1)
    np.add.at(conc, np.floor(e).astype(int), -1)
    conc = np.cumsum(conc)[:nb]
    info = rec[:, 6].astype(np.int64)
    fast = (info >> 17) & 1
    tv = info & 0xFFFF
    d = lambda a, b: (b - a) * TICK_US  # noqa: E731
    out = {"tiles": int(len(rec)), "span_us": span,
           "median_resident": float(np.median(conc[:max(1, int(span))])),
           "packets_per_tile": pct(tv), "slow_phase2_share": float(1 - fast.mean()),
           "load_us": pct(d(t0, tl)), "sums_us": pct(d(tl, ts)), "map_hdr_us": pct(d(ts, tm)),
           "phase2_us": pct(d(tm, te)), "tile_us": pct(d(t0, te)),
           # from the phase-1 barrier to the LAST wave's sums / map / header chunks done
           "last_wave_sums_us": pct(d(tl, rec[:, 8].astype(np.int64))),
           "last_wave_map_us": pct(d(tl, rec[:, 9].astype(np.int64))),
           "last_wave_hdr_us": pct(d(tl, rec[:, 10].astype(np.int64))),
           "barrier_after_hdr_us": pct(d(rec[:, 10].astype(np.int64), tm))}
    for name, m in (("fast", fast == 1), ("slow", fast == 0)):
        if m.any():
            out[f"phase2_us_{name}"] = pct(d(tm, te)[m])
            out[f"map_hdr_us_{name}"] = pct(d(ts, tm)[m])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", default="")
    ap.add_argument("--forms", default="packet_tiles:51=0;byte_tiles:51=2",
                    help="name:key=value,...;... (rudpx_tune knobs per form; unnamed knobs keep their defaults)")
    ap.add_argument("--shapes", default="equal_1472,ragged_0_2944")
    args = ap.parse_args()
    lib = _native.tools_lib()
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, 1472
    g = torch.Generator(device=dev).manual_seed(0x5EED0004)
    shapes = {}
    tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
    shapes["equal_1472"] = (tab, pay.view(-1), torch.full((n,), L, dtype=torch.int32, device=dev))
    lens = torch.randint(0, 2 * L + 1, (n,), dtype=torch.int32, device=dev, generator=g)
    tot = int(lens.sum().item())
    tab2, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
    shapes["ragged_0_2944"] = (tab2, torch.randint(0, 256, (tot,), dtype=torch.uint8, device=dev, generator=g), lens)
    forms = {}
    for item in args.forms.split(";"):
        fname, _, kvs = item.partition(":")
        forms[fname] = {int(k): int(v) for k, v in (kv.split("=") for kv in kvs.split(",") if kv)}
    keys = sorted({k for kv in forms.values() for k in kv})
    defaults = {k: lib.rudpx_tune(k, 0) for k in keys}
    for k, v in defaults.items():
        lib.rudpx_tune(k, v)
    out = {}
    for name, (t, flat, ln) in shapes.items():
        if name not in args.shapes.split(","):
            continue
        blocks = flat.numel() // 1000 + n // 8 + 16
        buf = torch.zeros((blocks * 12,), dtype=torch.int64, device=dev)
        for form, knobs in forms.items():
            for k in keys:
                lib.rudpx_tune(k, knobs.get(k, defaults[k]))
            res = batch.pack_batch_varlen(t, flat, ln, "rudp7")
            for _ in range(3):
                batch.pack_batch_varlen(t, flat, ln, "rudp7", reuse=res, check=False)
            ts = []
            for _ in range(10):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                batch.pack_batch_varlen(t, flat, ln, "rudp7", reuse=res, check=False)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            runs = []
            for k in range(2):
                buf.zero_()
                batch.pack_batch_varlen(t, flat, ln, "rudp7", reuse=res, check=False)
                lib.rudpx_encode_trace(buf.data_ptr())
                batch.pack_batch_varlen(t, flat, ln, "rudp7", reuse=res, check=False)
                lib.rudpx_encode_trace(None)
                torch.cuda.synchronize()
                rec = buf.view(-1, 12).cpu().numpy()
                if args.save:
                    np.save(Path(args.save) / f"vtile_{name}_{form}_{k}.npy", rec[rec[:, 0] != 0])
                runs.append(analyse(rec))
            res.check()
            out[f"{name}/{form}"] = {"call_ms_median": statistics.median(ts), "traced": runs}
            print(f"{name}/{form} done", file=sys.stderr, flush=True)
        del buf
    for k, v in defaults.items():
        lib.rudpx_tune(k, v)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
