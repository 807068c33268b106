"""Why does the bench's fixed-decode leg (1M x 1472 B, rudp7) time slower than
the raw ABI call in tools/lib_ab.py?  Times, in one process on the same frames:
bench.time_loop over Workload.decode (the bench leg), the same loop over the raw
rudp_decode with fixed output buffers, and per-launch HIP events of both.

usage: python tools/decode_probe.py [--steps 20]
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

import bench  # noqa: E402
from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = bench.Workload(torch, batch, 1 << 20, 1472, "rudp7", 0, bench.SEEDS[1472], dev)
    for i in range(len(w.sets)):
        w.encode(batch, i)
    n, F = 1 << 20, 1479
    fr = w.sets[0][2]
    outs = [torch.empty((n,), dtype=dt, device=dev) for dt in (torch.uint16, torch.uint16, torch.uint8,
                                                               torch.uint8, torch.uint16)]
    lib = _native.lib()
    stream = torch.cuda.current_stream().cuda_stream

    def raw(i):
        lib.rudp_decode(fr.data_ptr(), None, F, n, None, *[t.data_ptr() for t in outs], None, 7, 0, stream)

    def py(i):
        w.decode(batch, i)

    def py_keep(i, keep=[]):
        keep.append(w.decode(batch, i))
        if len(keep) > 4:
            keep.pop(0)

    res = {}
    for rep in range(3):
        for name, fn in (("bench_py", py), ("raw", raw), ("py_keep", py_keep)):
            ms = bench.time_loop(torch, fn, args.steps, 3) / args.steps
            ev = bench.time_events(torch, fn, args.steps, 3)
            res.setdefault(name, []).append({"loop_ms": ms, "event_median_ms": statistics.median(ev),
                                             "event_min_ms": min(ev), "event_max_ms": max(ev)})
            print(name, rep, res[name][-1], file=sys.stderr, flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
