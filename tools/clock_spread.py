"""Per-dispatch duration against the effective shader clock of one kernel.

Reads a rocprofv3 counter-collection CSV taken with GRBM_COUNT and
GRBM_GUI_ACTIVE (plus any SQ counters) and prints, per dispatch of the named
kernel, its duration (End - Start timestamps), the clock GRBM_COUNT implies
(GRBM_COUNT / XCDs / duration: the counter is summed over the 8 XCDs), and
SQ_WAVE_CYCLES per dispatch when present; then the correlation of duration
with clock and with dispatch order, so a spread of launch times can be put
down to the clock (power / thermal state) or to the work (tile order, data).

usage: python tools/clock_spread.py CSV --kernel decode_tile_kernel [--xcds 8] [--json out.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    by = collections.defaultdict(dict)
    span = {}
    for r in csv.DictReader(open(args.csv)):
        if args.kernel not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        by[d][r["Counter_Name"]] = float(r["Counter_Value"])
        span[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    rows = []
    for i, d in enumerate(sorted(by)):
        t0, t1 = span[d]
        us = (t1 - t0) / 1e3
        ghz = by[d].get("GRBM_COUNT", float("nan")) / args.xcds / (t1 - t0)
        busy = by[d].get("GRBM_GUI_ACTIVE", float("nan")) / max(by[d].get("GRBM_COUNT", 1.0), 1.0)
        rows.append({"dispatch": d, "order": i, "us": us, "ghz": ghz, "gui_active_share": busy,
                     "sq_wave_cycles": by[d].get("SQ_WAVE_CYCLES")})

    def corr(a, b):
        ma, mb = statistics.fmean(a), statistics.fmean(b)
        va = sum((x - ma) ** 2 for x in a)
        vb = sum((y - mb) ** 2 for y in b)
        return sum((x - ma) * (y - mb) for x, y in zip(a, b)) / (va * vb) ** 0.5 if va and vb else float("nan")

    us = [r["us"] for r in rows]
    ghz = [r["ghz"] for r in rows]
    out = {"kernel": args.kernel, "dispatches": len(rows),
           "us": {"min": min(us), "median": statistics.median(us), "max": max(us), "stdev": statistics.pstdev(us)},
           "ghz": {"min": min(ghz), "median": statistics.median(ghz), "max": max(ghz)},
           "corr_us_vs_ghz": corr(us, ghz), "corr_us_vs_order": corr(us, [r["order"] for r in rows]),
           "us_times_ghz": {"min": min(u * g for u, g in zip(us, ghz)), "max": max(u * g for u, g in zip(us, ghz))},
           "rows": rows}
    if rows and rows[0]["sq_wave_cycles"] is not None:
        wc = [r["sq_wave_cycles"] for r in rows]
        out["corr_us_vs_sq_wave_cycles"] = corr(us, wc)
    text = json.dumps(out, indent=1)
    if args.json:
        open(args.json, "w").write(text)
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}, indent=1))


if __name__ == "__main__":
    main()
