"""Per-kernel median / mean durations of rocprofv3 kernel traces under gpurun_out/.

usage: python tools/trace_stats.py TAG [TAG ...]   (directories gpurun_out/TAG/run_kernel_trace.csv)
       python tools/trace_stats.py --counters TAG_sq [...]   (gpurun_out/TAG_sq/run_counter_collection.csv:
                                                            per kernel, the median of each counter over dispatches)
Prints, per tag, each kernel with at least --min dispatches and the run's HIP-event
ms_per_launch from gpurun_out/TAG.log (tools/run_kernel.py's line).
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics as st
from pathlib import Path

OUT = Path(__file__).resolve().parent.parent / "gpurun_out"


def kernel_durations(tag: str) -> dict:
    by = {}
    with open(OUT / tag / "run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            by.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return by


def counters(tag: str) -> dict:
    """{kernel: {counter: median over dispatches}} of a --pmc run (values summed over a dispatch's rows)."""
    per = {}
    with open(OUT / tag / "run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            key = (r["Kernel_Name"], r["Dispatch_Id"])
            per.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    by = {}
    for (k, _), cs in per.items():
        for c, v in cs.items():
            by.setdefault(k, {}).setdefault(c, []).append(v)
    return {k: {c: st.median(v) for c, v in cs.items()} for k, cs in by.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--min", type=int, default=20)
    ap.add_argument("--counters", action="store_true")
    args = ap.parse_args()
    if args.counters:
        print(json.dumps({t: counters(t) for t in args.tags}, indent=1))
        return
    for tag in args.tags:
        line = ""
        log = OUT / f"{tag}.log"
        if log.exists():
            for ln in log.read_text().splitlines():
                if ln.startswith("{"):
                    line = f"  events {json.loads(ln)['ms_per_launch'] * 1e3:.1f} us/launch"
        print(f"== {tag}{line}")
        for k, v in sorted(kernel_durations(tag).items(), key=lambda kv: -sum(kv[1])):
            if len(v) >= args.min:
                print(f"  {len(v):5d}  median {st.median(v):9.2f} us  mean {st.mean(v):9.2f}  {k[:100]}")


if __name__ == "__main__":
    main()
