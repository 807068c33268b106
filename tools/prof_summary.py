"""Summarise rocprofv3 output into profiles/ (committed evidence).

usage: python tools/prof_summary.py --round r01 --tag encode_1Mx1472 \
          --kt gpurun_out/prof_kt --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write \
          --kernel encode_tile_kernel --n 1048576 --L 1472 --alg-bytes-per-unit 2956

--kernel takes a comma-separated list for a call that is a chain of launches
(e.g. the varlen encode: scan passes + tile kernel): the summary's avg_us is
then the sum of the kernels' averages (each runs once per call) and the HBM
bytes the sum of their medians; per-kernel entries are listed under "chain".

Writes profiles/<round>/<tag>_kernel_stats.csv (the rocprofv3 --stats table),
profiles/<round>/<tag>_summary.json, and (with --pmc-out) the per-launch HBM
traffic bench.py reads.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE
and WRITE_SIZE come from separate --pmc passes, are in KiB, and FETCH_SIZE is
doubled on gfx950 (it counts 128-B streaming reads at 64 B).
"""
from __future__ import annotations

import argparse
import csv
import json
import shutil
import statistics
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def _one(d: Path, suffix: str) -> Path:
    hits = sorted(d.rglob(f"*{suffix}"))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def counter_values(d: Path, kernel: str, counter: str):
    vals = []
    with open(_one(d, "counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def kernel_stats(d: Path, kernel: str):
    with open(_one(d, "kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                st = {"name": row["Name"], "calls": int(row["Calls"]),
                      "avg_ns": float(row["AverageNs"]), "min_ns": float(row["MinNs"]),
                      "max_ns": float(row["MaxNs"])}
                break
        else:
            raise SystemExit(f"kernel {kernel} not in stats")
    # per-dispatch durations from the trace: the median is robust to the
    # first, cold launches and to launches the tracer's own gaps slowed
    hits = sorted(d.rglob("*kernel_trace.csv"))
    if hits:
        durs = []
        with open(hits[0]) as f:
            for row in csv.DictReader(f):
                if row.get("Kernel_Name") == st["name"]:
                    durs.append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
        if durs:
            st["median_ns"] = statistics.median(durs)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kt", type=Path, required=True)
    ap.add_argument("--fetch", type=Path)
    ap.add_argument("--write", type=Path)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--L", type=int, required=True)
    ap.add_argument("--alg-bytes-per-unit", type=float, required=True)
    ap.add_argument("--pmc-out", type=Path, help="write the traffic record bench.py reads")
    ap.add_argument("--event-ms", type=float, help="run_kernel's HIP-event time per call under the tracer")
    args = ap.parse_args()

    out_dir = REPO / "profiles" / args.round
    out_dir.mkdir(parents=True, exist_ok=True)
    shutil.copy(_one(args.kt, "kernel_stats.csv"), out_dir / f"{args.tag}_kernel_stats.csv")
    # (a "|"-separated list when a kernel's template arguments hold commas)
    names = [k for k in args.kernel.split("|" if "|" in args.kernel else ",") if k]
    stats = [kernel_stats(args.kt, k) for k in names]
    avg_ns = sum(st["avg_ns"] for st in stats)
    alg = args.n * args.alg_bytes_per_unit
    summary = {
        "kernel": stats[0]["name"], "calls": stats[0]["calls"], "avg_us": avg_ns / 1e3,
        "min_us": sum(st["min_ns"] for st in stats) / 1e3, "max_us": sum(st["max_ns"] for st in stats) / 1e3,
        "units_per_launch": args.n, "payload_bytes": args.L,
        "algorithmic_bytes_per_unit": args.alg_bytes_per_unit,
        "algorithmic_bytes_per_launch": alg,
        "achieved_GBs_at_avg": alg / (avg_ns * 1e-9) / 1e9,
        "hbm_peak_GBs": 8000.0,
    }
    if all("median_ns" in st for st in stats):
        med_ns = sum(st["median_ns"] for st in stats)
        summary["median_us"] = med_ns / 1e3
        summary["achieved_GBs_at_median"] = alg / (med_ns * 1e-9) / 1e9
        summary["roofline_frac_at_median"] = summary["achieved_GBs_at_median"] / 8000.0
    if args.event_ms is not None:
        summary["hip_event_ms_per_call"] = args.event_ms
    if len(stats) > 1:
        summary["chain"] = [{"kernel": st["name"], "calls": st["calls"], "avg_us": st["avg_ns"] / 1e3,
                             **({"median_us": st["median_ns"] / 1e3} if "median_ns" in st else {})}
                            for st in stats]
        summary["chain_note"] = "avg_us/min_us/max_us are sums over the chain's kernels (one launch each per call)"
    summary["roofline_frac_at_avg"] = summary["achieved_GBs_at_avg"] / 8000.0
    if args.fetch and args.write:
        rd = wr = 0.0
        nf = nw = 0
        for k, st in zip(names, stats):
            fetch = counter_values(args.fetch, k, "FETCH_SIZE")
            write = counter_values(args.write, k, "WRITE_SIZE")
            rd += statistics.median(fetch) * 1024 * 2   # KiB; x2 gfx950 FETCH_SIZE correction
            wr += statistics.median(write) * 1024
            nf, nw = nf + len(fetch), nw + len(write)
        summary.update({
            "pmc_launches": [nf, nw],
            "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": rd + wr,
            "traffic_over_algorithmic": (rd + wr) / alg,
            "pmc_note": "median over launches; FETCH_SIZE*1024*2 + WRITE_SIZE*1024 "
                        "(MI355X_MICROARCH.md §HBM gfx950 correction), separate --pmc passes",
        })
        if args.pmc_out:
            args.pmc_out.write_text(json.dumps({
                "L": args.L, "n": args.n, "kernel": stats[0]["name"],
                "hbm_bytes_per_launch": rd + wr, "source": f"profiles/{args.round}/{args.tag}_summary.json",
            }, indent=1) + "\n")
    (out_dir / f"{args.tag}_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
