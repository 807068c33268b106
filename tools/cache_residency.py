"""Does the 256 MiB Infinity Cache (MALL) flatter the 1M x 1472 B headline?

The headline re-encodes one buffer set (1.55 GB in, 1.55 GB out) back to
back; C5's 16M set is 16x larger and ran ~3% slower per packet while PMC
traffic and UTCL1 translation misses per packet stayed equal.  Here, per
launch (median of HIP-event pairs), interleaved round by round:
  one_set     the headline: the same input and output every launch
  two_sets    two sets alternating (6.2 GB working set)
  four_sets   four sets rotating
  flushed     one set, a 1 GiB scratch write between launches (outside the events)
  n16M        the C5 shape, one set, per 2^20 packets
  n16M_split  the same 16M buffers encoded as 16 launches of 2^20 packets each
              (launch size vs address-space size)
  n4M         one 4M-packet launch (12.4 GB in + out)

usage: python tools/cache_residency.py [--reps 20] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-16m", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L, n = 1472, 1 << 20
    sets = []
    for k in range(4):
        tab, pay = batch.synth_batch(n, L, 0x5EED0004, first_index=k * n, device=dev)
        sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
    scratch = torch.empty((1 << 30,), dtype=torch.uint8, device=dev)
    big = None
    if not args.no_16m:
        tab16, pay16 = batch.synth_batch(16 * n, L, 0x5EED0005, device=dev)
        big = (tab16, pay16, torch.empty((16 * n, L + 7), dtype=torch.uint8, device=dev))

    def enc(s):
        batch.pack_batch(s[0], s[1], 7, out=s[2], want_csum=False)

    def timed(pick, reps, flush=False, scale=1.0):
        ts = []
        for i in range(reps):
            if flush:
                scratch.fill_(i & 0xFF)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            enc(pick(i))
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        return [x.elapsed_time(y) / scale for x, y in ts]

    forms = {
        "one_set": lambda: timed(lambda i: sets[0], args.reps),
        "two_sets": lambda: timed(lambda i: sets[i % 2], args.reps),
        "four_sets": lambda: timed(lambda i: sets[i % 4], args.reps),
        "flushed": lambda: timed(lambda i: sets[0], args.reps, flush=True),
    }
    if big is not None:
        forms["n16M"] = lambda: timed(lambda i: big, max(4, args.reps // 4), scale=16.0)
        parts = [(type(big[0])(big[0].seq[k * n:(k + 1) * n], big[0].ack[k * n:(k + 1) * n],
                               big[0].flags[k * n:(k + 1) * n]), big[1][k * n:(k + 1) * n],
                  big[2][k * n:(k + 1) * n]) for k in range(16)]
        forms["n16M_split"] = lambda: timed(lambda i: parts[i % 16], 16 * max(2, args.reps // 8))
        forms["n4M"] = lambda: timed(lambda i: (type(big[0])(big[0].seq[:4 * n], big[0].ack[:4 * n],
                                                             big[0].flags[:4 * n]), big[1][:4 * n],
                                                big[2][:4 * n]), max(4, args.reps // 2), scale=4.0)
    for f in forms.values():  # warm every form once
        f()
    per = {k: [] for k in forms}
    for _ in range(args.rounds):
        for k, f in forms.items():
            per[k] += f()
    out = {k: {"ms_per_2^20_packets": statistics.median(v), "min": min(v), "max": max(v),
               "frac": n * (2 * L + 12) / statistics.median(v) / 1e9 / 8.0, "launches": len(v)}
           for k, v in per.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
