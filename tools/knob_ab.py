"""Interleaved A/B of one rudpx_tune knob (tools build) on the codec's BASELINE shapes.

For every shape, each knob value's launches run in rotation (median of
--reps rounds of --inner back-to-back calls, HIP events), and every value's
output is compared byte for byte with the first value's.

shapes: encode:L (fixed-length, 1M x L, rotating sets below 1 GiB), decode:L, u8:L (decode + UTF-8),
u8text:L (the same on valid multi-byte text), u8mix:L (mostly-ASCII text with a few
multi-byte characters in every payload), varlen:L
(packed, equal lengths), ragged (lengths uniform in [0, 2944]), decode:L,
vdec:L (varlen decode, equal lengths; vdec:L+u with the UTF-8 check), rdec (varlen
decode, ragged ASCII lengths; rdec:+u; rdec:sort sorts each run of 16 lengths,
rdec:perm makes each run of 16 a permutation of one even spread), dedup (1M one-character datagrams, window 500).

usage: python tools/knob_ab.py --knob 58 --values 0,1 --shapes encode:1472,encode:64,varlen:1472,ragged
       python tools/knob_ab.py --variants "base:;t256b512:2=256,10=512" --shapes encode:64
         (named variants of several knobs each; knobs a variant does not name keep their defaults)
"""
from __future__ import annotations

import argparse
import json
import math
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def make_shape(spec, dev):
    n = 1 << 20
    kind, _, arg = spec.partition(":")
    if kind in ("encode", "decode", "u8", "u8text", "u8mix"):
        L = int(arg)
        nsets = max(1, min(8, math.ceil((1 << 30) / (n * (2 * L + 12)))))
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            if kind == "u8text":  # valid multi-byte text in every payload (bench decode_utf8_*_multibyte_text)
                from run_kernel import text_payloads
                pay = text_payloads(n, L, dev)
            elif kind == "u8mix":  # mostly-ASCII text, a few multi-byte characters in every payload
                from run_kernel import mixed_text_payloads
                pay = mixed_text_payloads(n, L, dev)
            fr, _ = batch.pack_batch(tab, pay, 7)
            sets.append((tab, pay, fr))
        cur = [0]

        def run():
            tab, pay, fr = sets[cur[0] % len(sets)]
            cur[0] += 1
            if kind == "encode":
                batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
                return fr
            if kind.startswith("u8"):  # decode + strict UTF-8 in one pass
                d = batch.unpack_batch(fr, 7, utf8=True)
                return torch.cat([d.ok, d.valid])
            return batch.unpack_batch(fr, 7).ok
        return run
    g = torch.Generator(device=dev).manual_seed(0x5EED0004)
    if kind == "dedup":  # the proxy's check over 1M one-character rudp5 datagrams, window 500
        tab, pay = batch.synth_batch(n, 1, 0x5EED0004, device=dev)
        res = batch.pack_batch_varlen(tab, pay.view(-1), torch.ones(n, dtype=torch.int32, device=dev), 5)

        def run():
            return batch.detect_retransmissions(res.frames, frame_off=res.frame_off, window=500, check=False)
        return run
    if kind in ("vdec", "rdec"):  # varlen decode (vdec:L equal lengths, rdec: lengths uniform in [0, 2944])
        if kind == "vdec":
            L = int(arg.split("+")[0])
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            flat, lens = pay.view(-1), torch.full((n,), L, dtype=torch.int32, device=dev)
        else:
            lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev, generator=g)
            if arg.startswith("sort"):  # sorted within each run of 16 frames: same tile runs, even waves
                lens = lens.view(-1, 16).sort(dim=1).values.reshape(-1).contiguous()
            elif arg.startswith("perm"):  # every run of 16 a permutation of one spread: equal tile runs
                base = (torch.arange(16, device=dev, dtype=torch.int32) * 2944 + 1472) // 16
                idx = torch.rand((n // 16, 16), device=dev, generator=g).argsort(dim=1)
                lens = base[idx].reshape(-1).to(torch.int32).contiguous()
            tab, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
            flat = torch.randint(0, 128, (int(lens.sum().item()),), dtype=torch.uint8, device=dev, generator=g)
        res = batch.pack_batch_varlen(tab, flat, lens, 7)
        utf8 = spec.endswith("+u")
        dec = batch.unpack_batch_varlen(res.frames, res.frame_off, 7, utf8=utf8)

        def run():
            batch.unpack_batch_varlen(res.frames, res.frame_off, 7, reuse=dec, check=False, utf8=utf8)
            return dec._buf
        return run
    if kind == "varlen":
        L = int(arg)
        tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
        flat, lens = pay.view(-1), torch.full((n,), L, dtype=torch.int32, device=dev)
    else:  # ragged
        lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev, generator=g)
        tab, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
        flat = torch.randint(0, 256, (int(lens.sum().item()),), dtype=torch.uint8, device=dev, generator=g)
    res = batch.pack_batch_varlen(tab, flat, lens, 7)

    def run():
        batch.pack_batch_varlen(tab, flat, lens, 7, reuse=res, check=False)
        return res.frames
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", type=int)
    ap.add_argument("--values")
    ap.add_argument("--variants", help="name:key=value,key=value;name:...")
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--inner", type=int, default=10)
    args = ap.parse_args()
    lib = _native.tools_lib()
    dev = torch.device("cuda", 0)
    if args.variants:
        variants = {}
        for item in args.variants.split(";"):
            name, _, kvs = item.partition(":")
            variants[name] = {int(k): int(v) for k, v in (kv.split("=") for kv in kvs.split(",") if kv)}
    else:
        variants = {str(v): {args.knob: int(v)} for v in args.values.split(",")}
    keys = sorted({k for kv in variants.values() for k in kv})
    defaults = {k: lib.rudpx_tune(k, 0) for k in keys}
    for k, v in defaults.items():
        lib.rudpx_tune(k, v)

    def apply(name):
        for k in keys:
            lib.rudpx_tune(k, variants[name].get(k, defaults[k]))

    def restore():
        for k, v in defaults.items():
            lib.rudpx_tune(k, v)
    values = list(variants)
    out = {"variants": variants, "shapes": {}}
    for spec in args.shapes.split(","):
        # every shape's inputs (frames, offsets a decode shape encodes first) are built
        # under the default knobs, whatever variant timed the shape before
        restore()
        run = make_shape(spec, dev)
        ref = None
        exact = {}
        for v in values:
            apply(v)
            got = run().clone()
            torch.cuda.synchronize()
            if ref is None:
                ref = got
            exact[v] = bool(torch.equal(got, ref))
        times = {v: [] for v in values}
        for _ in range(args.reps):
            for v in values:
                apply(v)
                run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.inner):
                    run()
                e.record()
                e.synchronize()
                times[v].append(s.elapsed_time(e) / args.inner)
        out["shapes"][spec] = {"ms": {v: statistics.median(t) for v, t in times.items()}, "exact": exact}
        print(spec, out["shapes"][spec], file=sys.stderr, flush=True)
        del run
        torch.cuda.empty_cache()
    restore()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
