"""Run one codec op repeatedly on one shape, for rocprofv3 captures.

usage: python tools/run_kernel.py --op encode|decode|roundtrip|encode_varlen|decode_varlen|utf8|dedup
          [--L 1472] [--n 1048576]
          [--layout rudp7] [--steps 20] [--ragged] [--tune 51=1,52=2]
Prints the HIP-event time per launch so it can be set beside the profiler's
kernel-trace average.  Runs librudp.so (the product) unless --tune is given,
which needs the diagnostics build librudp_tools.so.
"""
from __future__ import annotations

import argparse
import json
import math
import time
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import batch  # noqa: E402


def text_payloads(n, L, dev):
    """n copies of one L-byte payload of valid 1-4 byte UTF-8 characters, as bench.py's
    decode_utf8_1Mx1472_multibyte_text leg frames them."""
    text = ("\u00e9\u4e2d\U0001f600a\u00df\u0416\u20ac\U0001d11e" * (L // 8 + 8)).encode()[:L]
    while True:
        try:
            text.decode()
            break
        except UnicodeDecodeError:
            text = text[:-1]
    text += b"x" * (L - len(text))
    return torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev).expand(n, L).contiguous()


def mixed_text_payloads(n, L, dev):
    """n copies of one L-byte payload of mostly-ASCII text with a few multi-byte characters
    (about one 16-B chunk in two holds a high bit): every frame holds a high bit, most chunks
    do not."""
    text = ("Reliable UDP delivers each datagram in order; the proxy drops some \u2014 caf\u00e9. "
            * (L // 40 + 2)).encode()[:L]
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
    ap.add_argument("--op", choices=["encode", "decode", "decode_copy", "roundtrip", "encode_varlen",
                                     "decode_varlen", "utf8", "dedup"], default="encode",
                    help="utf8: strict UTF-8 check of the fixed-stride frames (bench leg "
                         "utf8_validate_1Mx1472); dedup: the proxy's 500-deep retransmission check "
                         "over packed frames of L-byte payloads (bench leg proxy_dedup_1M_window500, L = 1)")
    ap.add_argument("--L", type=int, default=1472)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--layout", default="rudp7")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ragged", action="store_true",
                    help="varlen ops: lengths uniform in [0, 2L] (mean L) instead of all L")
    ap.add_argument("--utf8", action="store_true",
                    help="decode ops: strict UTF-8 of each payload in the same pass (rudp_decode_utf8)")
    ap.add_argument("--text", action="store_true",
                    help="fixed-length ops: every payload valid multi-byte UTF-8 text of 1-4 byte "
                         "characters (bench leg decode_utf8_1Mx1472_multibyte_text)")
    ap.add_argument("--tune", default="",
                    help="rudpx_tune knobs to set first, as key=value[,key=value...]")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="idle time between launches (synchronize, then sleep): separates a "
                         "per-launch effect from one of sustained back-to-back HBM load")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    H = batch.layout_header_len(args.layout)
    per_set = args.n * (2 * args.L + H + 5)
    nsets = max(1, min(8, math.ceil((1 << 30) / per_set)))
    sets = []
    for _ in range(nsets):
        tab, pay = batch.synth_batch(args.n, args.L, 0x5EED0004, device=dev)
        if args.text:
            pay = text_payloads(args.n, args.L, dev)
        fr, _ = batch.pack_batch(tab, pay, args.layout)
        sets.append((tab, pay, fr))
    import ctypes
    from rudp import _native
    # the product library unless knobs are asked for (they live in the diagnostics build only)
    lib = _native.tools_lib() if args.tune else _native.lib()
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        lib.rudpx_tune(int(k), int(v))
    scratch = [torch.empty(args.n, dtype=torch.uint16, device=dev) for _ in range(2)] + \
              [torch.empty(args.n, dtype=torch.uint8, device=dev) for _ in range(2)]

    def decode_copy(tab, pay, fr):
        # copy-out decode into the payload buffer (aligned), preallocated outputs
        _native.check(lib.rudp_decode(fr.data_ptr(), None, args.L + H, args.n, None,
                                      scratch[0].data_ptr(), scratch[1].data_ptr(),
                                      scratch[2].data_ptr(), scratch[3].data_ptr(), None,
                                      pay.data_ptr(), H, 0, torch.cuda.current_stream().cuda_stream))
    del ctypes

    vsets = []
    if args.op.endswith("varlen") or args.op == "dedup":
        for tab, pay, fr in sets:
            if args.ragged:
                g = torch.Generator(device=dev).manual_seed(7)
                lens = torch.randint(0, 2 * args.L + 1, (args.n,), dtype=torch.int32, device=dev, generator=g)
                tab, big = batch.synth_batch(args.n, 2 * args.L, 0x5EED0004, device=dev)
                flat = big.view(-1)[: int(lens.sum().item())].contiguous()
                del big
            else:
                lens = torch.full((args.n,), args.L, dtype=torch.int32, device=dev)
                flat = pay.view(-1)
            res = batch.pack_batch_varlen(tab, flat, lens, "rudp5" if args.op == "dedup" else args.layout)
            dec = batch.unpack_batch_varlen(res.frames, res.frame_off, "rudp5" if args.op == "dedup" else args.layout,
                                            csum=res.csum, utf8=args.utf8)
            vsets.append((tab, flat, lens, res, dec))

    def step(i):
        if vsets:
            # the sync-free forms with the outputs reused, as the bench's *_reuse forms:
            # the call is its kernels only
            tab, flat, lens, res, dec = vsets[i % nsets]
            if args.op == "encode_varlen":
                batch.pack_batch_varlen(tab, flat, lens, args.layout, reuse=res, check=False)
            elif args.op == "dedup":
                batch.detect_retransmissions(res.frames, frame_off=res.frame_off, window=500)
            else:
                batch.unpack_batch_varlen(res.frames, res.frame_off, args.layout, csum=res.csum, reuse=dec,
                                          check=False, utf8=args.utf8)
            return
        tab, pay, fr = sets[i % nsets]
        if args.op in ("encode", "roundtrip"):
            batch.pack_batch(tab, pay, args.layout, out=fr, want_csum=False)
        if args.op in ("decode", "roundtrip"):
            batch.unpack_batch(fr, args.layout, utf8=args.utf8)
        if args.op == "decode_copy":
            decode_copy(tab, pay, fr)
        if args.op == "utf8":
            batch.validate_utf8(fr, args.layout)

    # warm the launch for ~30 ms before the clock, as bench.py's legs do (a
    # launch after an idle gap runs slow: profiles/r03/sweeps/c2_probe.json)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.03
    i = 0
    while time.perf_counter() < t_end:
        step(i)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(args.steps):
        step(i)
        if args.gap_ms:
            torch.cuda.synchronize()
            time.sleep(args.gap_ms / 1e3)
    e.record()
    e.synchronize()
    payload_bytes = int(vsets[0][1].numel()) if vsets else args.n * args.L
    print(json.dumps({"op": args.op, "utf8": args.utf8, "text": args.text, "L": args.L, "n": args.n, "layout": args.layout, "tune": args.tune,
                      "ragged": args.ragged, "payload_bytes": payload_bytes,
                      "buffer_sets": nsets, "ms_per_launch": s.elapsed_time(e) / args.steps}))


if __name__ == "__main__":
    main()
