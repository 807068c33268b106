"""Timeline of one fixed-length encode launch, tile by tile (rudpx_encode_trace).

Every tile records its start and end (100 MHz wall clock), its XCD and CU.
From one traced launch per shape this prints:
  span_us            first start to last end
  per_xcd            tiles, first start / last end (us from the launch start),
                     mean tile time
  ramp_us / tail_us  time until the resident tile count first reaches 90 %
                     of its median, and from its last time there to the end
  tile_us            mean tile time in the first / middle / last tenth of the span
  phases             per-tile percentiles: phase-1 loads (start to landed), sums and
                     headers (landed to the second barrier), phase-2 stores (to the end)
  untraced_ms        the same launch without the trace, median of events
  stamp_to_first_tile_us / last_tile_to_stamp_us
                     a one-lane kernel stamps the wall clock on the stream just
                     before and just after the traced launch: the launch's time
                     outside its tiles (plus two kernel boundaries)
Shapes: the headline (1M x 1472 B in buffers of its own) and a 16M launch;
any --L (tiles of T packets as encode_tile_geometry picks them: 16 from 512 B,
128 at 64 B).  --sets K rotates K buffer sets (as the bench does below 1 GiB
per set, so the traced launch does not find its inputs in the Infinity Cache).

usage: python tools/tile_timeline.py [--L 1472] [--no-16m] [--sets 8]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402

TICK_US = 0.01  # wall_clock64 runs at 100 MHz


def pct(x):
    return {p: round(float(np.percentile(x, p)), 3) for p in (10, 50, 90)}


def analyse(rec: np.ndarray) -> dict:
    t0 = rec[:, 0].astype(np.int64)
    t1 = rec[:, 1].astype(np.int64)
    xcc = rec[:, 2].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) * TICK_US, (t1 - base) * TICK_US
    span = float(e.max())
    per = {}
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        per[int(x)] = {"tiles": int(m.sum()), "first_start_us": float(s[m].min()),
                       "last_end_us": float(e[m].max()), "mean_tile_us": float((e[m] - s[m]).mean())}
    # resident tiles over time, 1-us bins
    nb = int(span) + 2
    conc = np.zeros(nb + 1)
    np.add.at(conc, np.floor(s).astype(int), 1)
    np.add.at(conc, np.floor(e).astype(int), -1)
    conc = np.cumsum(conc)[:nb]
    med = float(np.median(conc[: max(1, int(span))]))
    hi = np.nonzero(conc >= 0.9 * med)[0]
    ramp = float(hi[0]) if len(hi) else span
    tail = float(span - hi[-1]) if len(hi) else span
    d = e - s
    tenth = span / 10
    first = d[s < tenth].mean()
    mid = d[(s >= 4.5 * tenth) & (s < 5.5 * tenth)].mean()
    last = d[s >= 9 * tenth].mean()
    t_ld = (rec[:, 4].astype(np.int64) - t0) * TICK_US
    t_sm = (rec[:, 5].astype(np.int64) - t0) * TICK_US
    phases = {"load_us": pct(t_ld), "sum_us": pct(t_sm - t_ld), "store_us": pct(d - t_sm)}
    return {"span_us": span, "tiles": int(len(rec)), "median_resident_tiles": med, "phases": phases,
            "ramp_us": ramp, "tail_us": tail,
            "tile_us": {"first_tenth": float(first), "middle": float(mid), "last_tenth": float(last)},
            "xcd_last_end_spread_us": float(max(v["last_end_us"] for v in per.values())
                                            - min(v["last_end_us"] for v in per.values())),
            "per_xcd": per}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--no-16m", action="store_true")
    ap.add_argument("--save", default="", help="directory for the raw 1M traces (.npy)")
    ap.add_argument("--percu", default="", help="also trace 1M under these tiles-per-CU caps (rudpx_tune 6)")
    ap.add_argument("--early", action="store_true", help="also trace 1M with the header-table loads before phase 1 (rudpx_tune 30)")
    ap.add_argument("--sets", type=int, default=1, help="rotating buffer sets (the traced launch uses the next one)")
    ap.add_argument("--tune", default="", help="rudpx_tune knobs for every shape, key=value[,key=value]")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.tools_lib()
    lib.rudpx_encode_trace.argtypes = [ctypes.c_void_p]
    lib.rudpx_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    stamps = torch.zeros((4,), dtype=torch.int64, device=dev)
    L, M = args.L, 1 << 20
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    shapes = {"own_1M": (M, -1)}
    for c in filter(None, args.percu.split(",")):
        shapes[f"own_1M_percu{c}"] = (M, int(c))
    if args.early:
        shapes["own_1M_early_table"] = (M, -1)
    if not args.no_16m:
        shapes["launch_16M"] = (16 * M, -1)
    tune = {}
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        tune[int(k)] = int(v)
        lib.rudpx_tune(int(k), int(v))
    # packets per tile, as encode_tile_geometry (capi.hip) picks them
    T = 16
    while T * 2 <= min(8192 // L, 256):
        T *= 2
    out = {"L": L, "packets_per_tile": T, "buffer_sets": args.sets, "tune": args.tune}
    for name, (n, percu) in shapes.items():
        lib.rudpx_tune(6, percu)
        lib.rudpx_tune(30, 1 if name.endswith("early_table") else -1)
        sets = []
        for _ in range(args.sets if n == M else 1):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
        cur = [0]

        def enc():
            tab, pay, fr = sets[cur[0] % len(sets)]
            cur[0] += 1
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        for _ in range(3):
            enc()
        ts = []
        for _ in range(8):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            enc()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        tiles = (n + T - 1) // T
        buf = torch.zeros((tiles * 6,), dtype=torch.int64, device=dev)
        res = {"untraced_ms": statistics.median(ts)}
        runs = []
        for k in range(3):
            enc()  # back to back with the traced launch, as in the bench
            lib.rudpx_stamp(stamps.data_ptr(), stream)
            lib.rudpx_encode_trace(buf.data_ptr())
            enc()
            lib.rudpx_encode_trace(None)
            lib.rudpx_stamp(stamps[2:].data_ptr(), stream)
            enc()
            torch.cuda.synchronize()
            rec = buf.view(-1, 6).cpu().numpy()
            if (rec[:, 1] == 0).any():
                raise RuntimeError(f"trace incomplete: tile geometry is not T = {T}")
            r = analyse(rec)
            if args.save and n == M:
                np.save(Path(args.save) / f"tile_trace_{name}_{k}.npy", rec)
            st = stamps.cpu().numpy()
            r["stamp_to_first_tile_us"] = float((rec[:, 0].min() - st[0]) * TICK_US)
            r["last_tile_to_stamp_us"] = float((st[2] - rec[:, 1].max()) * TICK_US)
            runs.append(r)
        res["traced"] = runs
        out[name] = res
        del sets, buf
        torch.cuda.empty_cache()
        print(f"{name} done", file=sys.stderr, flush=True)
    lib.rudpx_tune(6, -1)
    lib.rudpx_tune(30, -1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
