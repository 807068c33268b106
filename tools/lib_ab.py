"""Interleaved A/B of the fixed-length encode across library builds.

Loads several builds of librudp (the product, the diagnostics build, an older
tree's build) side by side through ctypes and times rudp_encode of each on the
same buffers, round by round (median of --reps rounds of 10 launches), with
every build's frames compared byte for byte with the first's.

usage: python tools/lib_ab.py --libs name=path,... [--L 1472,1024,64]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--L", default="1472,1024,64")
    ap.add_argument("--reps", type=int, default=11)
    ap.add_argument("--op", default="encode", choices=["encode", "decode", "varlen", "vdecode", "vu8", "vval", "u8text",
                                                       "u8ascii", "u8val", "u8valtext"],
                    help="decode: verify-only fixed-length rudp_decode of the encoded frames; varlen: "
                         "rudp_encode_varlen_checked of packed payloads, --L lengths or 'ragged' "
                         "(uniform in [0, 2944]); a 'u' suffix (1472u) times the unchecked rudp_encode_varlen; "
                         "vdecode: rudp_decode_varlen_checked (no status word) of such frames, rudp5 with the "
                         "sideband checksums below 16-B payloads, else rudp7; u8text: rudp_decode_utf8 of "
                         "frames whose payload is valid multi-byte UTF-8 text (1-4 byte characters); u8ascii: "
                         "rudp_decode_utf8 of the ASCII synthetic frames; u8val / u8valtext: rudp_validate_utf8 (the check alone) of the ASCII / text frames")
    args = ap.parse_args()
    _native.lib()  # torch's HIP runtime first
    libs = {}
    for item in args.libs.split(","):
        name, path = item.split("=")
        h = ctypes.CDLL(str(REPO / path))
        h.rudp_encode.argtypes = [ctypes.POINTER(_native.RudpBatch), ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_encode.restype = ctypes.c_int
        h.rudp_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_decode.restype = ctypes.c_int
        if hasattr(h, "rudp_decode_utf8"):  # ABI 6 on (older trees lack it)
            h.rudp_decode_utf8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64] + \
                [ctypes.c_void_p] * 8 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            h.rudp_decode_utf8.restype = ctypes.c_int
        h.rudp_encode_varlen_checked.argtypes = [ctypes.POINTER(_native.RudpBatch), ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_encode_varlen_checked.restype = ctypes.c_int
        h.rudp_encode_varlen.argtypes = [ctypes.POINTER(_native.RudpBatch), ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_encode_varlen.restype = ctypes.c_int
        h.rudp_decode_varlen_checked.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p] + [ctypes.c_void_p] * 6 + \
                                                [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        h.rudp_decode_varlen_checked.restype = ctypes.c_int
        if hasattr(h, "rudp_decode_varlen_utf8"):
            h.rudp_decode_varlen_utf8.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_uint64] + [ctypes.c_void_p] * 8 + \
                                                 [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            h.rudp_decode_varlen_utf8.restype = ctypes.c_int
        if hasattr(h, "rudp_validate_utf8"):
            h.rudp_validate_utf8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            h.rudp_validate_utf8.restype = ctypes.c_int
        libs[name] = h
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    if args.op in ("varlen", "vdecode", "vu8", "vval"):
        for spec in args.L.split(","):
            fn = varlen_ab if args.op == "varlen" else vdecode_ab if args.op == "vdecode" else vu8_ab
            out[spec] = fn(libs, spec, args.reps, dev, stream, **({"validate": True} if args.op == "vval" else {}))
            print(spec, out[spec], file=sys.stderr, flush=True)
        print(json.dumps(out, indent=1))
        return
    for L in (int(x) for x in args.L.split(",")):
        n = 1 << 20
        nsets = max(1, min(8, math.ceil((1 << 30) / (n * (2 * L + 12)))))
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            if args.op in ("u8text", "u8valtext"):
                text = ("é中😀aßЖ€𝄞" * (L // 8 + 8)).encode()[:L]
                while True:
                    try:
                        text.decode()
                        break
                    except UnicodeDecodeError:
                        text = text[:-1]
                text += b"x" * (L - len(text))
                pay = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev).expand(n, L).contiguous()
            fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
            b = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                                  flags=tab.flags.data_ptr(), payload=pay.data_ptr(), len=None, payload_off=None)
            sets.append((tab, pay, fr, b))
            libs[next(iter(libs))].rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, stream)
        outs = [torch.empty((n,), dtype=dt, device=dev) for dt in (torch.uint16, torch.uint16, torch.uint8,
                                                                     torch.uint8, torch.uint16)]
        valid = torch.empty((n,), dtype=torch.uint8, device=dev)

        def call(h, fr, b):
            if args.op == "encode":
                return h.rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, stream)
            if args.op in ("u8val", "u8valtext"):
                return h.rudp_validate_utf8(fr.data_ptr(), None, L + 7, n, 7, valid.data_ptr(), 0, stream)
            if args.op in ("u8text", "u8ascii"):
                return h.rudp_decode_utf8(fr.data_ptr(), None, L + 7, n, None, *[t.data_ptr() for t in outs], None,
                                          valid.data_ptr(), 7, 0, stream)
            return h.rudp_decode(fr.data_ptr(), None, L + 7, n, None, *[t.data_ptr() for t in outs], None, 7, 0,
                                 stream)
        ref = None
        exact = {}
        for name, h in libs.items():
            _, _, fr, b = sets[0]
            if args.op == "encode":
                fr.zero_()
            for t in outs:
                t.zero_()
            assert call(h, fr, b) == 0
            got = fr.clone() if args.op == "encode" else torch.cat([t.view(torch.uint8) for t in outs] + [valid])
            ref = got if ref is None else ref
            exact[name] = bool(torch.equal(got, ref))
        times = {k: [] for k in libs}
        for _ in range(args.reps):
            for name, h in libs.items():
                for i in range(2):
                    _, _, fr, b = sets[i % nsets]
                    call(h, fr, b)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(10):
                    _, _, fr, b = sets[i % nsets]
                    call(h, fr, b)
                e.record()
                e.synchronize()
                times[name].append(s.elapsed_time(e) / 10)
        out[L] = {"ms": {k: statistics.median(v) for k, v in times.items()}, "exact": exact}
        print(L, out[L], file=sys.stderr, flush=True)
        del sets
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


def varlen_ab(libs, spec, reps, dev, stream):
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(0x5EED0004)
    unchecked = spec.endswith("u")
    spec = spec.rstrip("u")
    if spec == "ragged":
        lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev, generator=g)
        hint = 1472
    else:
        hint = int(spec)
        lens = torch.full((n,), hint, dtype=torch.int32, device=dev)
    tab, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
    pbytes = int(lens.sum().item())
    pay = torch.randint(0, 256, (pbytes,), dtype=torch.uint8, device=dev, generator=g)
    fcap = pbytes + 7 * n
    frames = torch.empty((fcap,), dtype=torch.uint8, device=dev)
    fo = torch.empty((n + 1,), dtype=torch.int64, device=dev)
    st = torch.zeros((1,), dtype=torch.int32, device=dev)
    b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                          flags=tab.flags.data_ptr(), payload=pay.data_ptr(), len=lens.data_ptr(), payload_off=None)

    def call(h):
        if unchecked:
            return h.rudp_encode_varlen(ctypes.byref(b), frames.data_ptr(), fo.data_ptr(), None, 7, 0, stream)
        return h.rudp_encode_varlen_checked(ctypes.byref(b), pbytes, frames.data_ptr(), fcap, fo.data_ptr(), None,
                                            st.data_ptr(), 7, 0, stream)
    ref, exact = None, {}
    for name, h in libs.items():
        frames.zero_()
        assert call(h) == 0
        assert int(st.item()) == 0
        got = frames.clone()
        ref = got if ref is None else ref
        exact[name] = bool(torch.equal(got, ref))
    times = {k: [] for k in libs}
    for _ in range(reps):
        for name, h in libs.items():
            for _ in range(2):
                call(h)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                call(h)
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / 10)
    return {"ms": {k: statistics.median(v) for k, v in times.items()}, "exact": exact, "payload_bytes": pbytes}


def vdecode_ab(libs, spec, reps, dev, stream):
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(0x5EED0004)
    if spec == "ragged":
        lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev, generator=g)
        hint = 1472
    else:
        hint = int(spec)
        lens = torch.full((n,), hint, dtype=torch.int32, device=dev)
    layout = 5 if hint < 16 else 7
    tab, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
    pay = torch.randint(0, 256, (int(lens.sum().item()),), dtype=torch.uint8, device=dev, generator=g)
    enc = batch.pack_batch_varlen(tab, pay, lens, layout, want_csum=layout == 5)
    cs = enc.csum if layout == 5 else None
    outs = [torch.empty((n,), dtype=dt, device=dev) for dt in (torch.uint16, torch.uint16, torch.uint8, torch.uint8,
                                                                 torch.uint16)]

    def call(h):
        return h.rudp_decode_varlen_checked(enc.frames.data_ptr(), enc.frames.numel(), enc.frame_off.data_ptr(),
                                            hint + layout, n, cs.data_ptr() if cs is not None else None,
                                            *[t.data_ptr() for t in outs], None, layout, 0, stream)
    ref, exact = None, {}
    for name, h in libs.items():
        for t in outs:
            t.zero_()
        assert call(h) == 0
        got = torch.cat([t.view(torch.uint8) for t in outs])
        ref = got if ref is None else ref
        exact[name] = bool(torch.equal(got, ref))
    times = {k: [] for k in libs}
    for _ in range(reps):
        for name, h in libs.items():
            for _ in range(2):
                call(h)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                call(h)
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / 10)
    return {"ms": {k: statistics.median(v) for k, v in times.items()}, "exact": exact, "layout": layout}


def text_flat(lens, dev):
    """Packed payloads of valid multi-byte text: payload i is the longest
    character-aligned prefix of one text of at most lens[i] bytes, padded with
    ASCII to lens[i]."""
    t = ("é中😀aßЖ€𝄞" * 400).encode()
    vl = torch.tensor([len(t[:k].decode("utf-8", "ignore").encode()) for k in range(int(lens.max().item()) + 1)],
                      dtype=torch.int64, device=dev)
    tt = torch.frombuffer(bytearray(t), dtype=torch.uint8).to(dev)
    l64 = lens.to(torch.int64)
    starts = torch.cumsum(l64, 0) - l64
    total = int(l64.sum().item())
    pos = torch.arange(total, device=dev, dtype=torch.int64) - torch.repeat_interleave(starts, l64)
    keep = torch.repeat_interleave(vl[l64], l64)
    return torch.where(pos < keep, tt[pos.clamp(max=tt.numel() - 1)], torch.full_like(pos, 0x78).to(torch.uint8))


def vu8_ab(libs, spec, reps, dev, stream, validate=False):
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(0x5EED0004)
    text = spec.endswith("t")
    spec = spec.rstrip("t")
    if spec == "ragged":
        lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev, generator=g)
        hint = 1472
    else:
        hint = int(spec)
        lens = torch.full((n,), hint, dtype=torch.int32, device=dev)
    tab, _ = batch.synth_batch(n, 0, 0x5EED0004, device=dev)
    if text:
        pay = text_flat(lens, dev)
    else:
        pay = torch.randint(0x20, 0x7F, (int(lens.sum().item()),), dtype=torch.uint8, device=dev, generator=g)
    enc = batch.pack_batch_varlen(tab, pay, lens, 7)
    outs = [torch.empty((n,), dtype=dt, device=dev) for dt in (torch.uint16, torch.uint16, torch.uint8, torch.uint8,
                                                                 torch.uint16, torch.uint8)]

    def call(h):
        if validate:
            return h.rudp_validate_utf8(enc.frames.data_ptr(), enc.frame_off.data_ptr(), hint + 7, n, 7,
                                        outs[5].data_ptr(), 0, stream)
        return h.rudp_decode_varlen_utf8(enc.frames.data_ptr(), enc.frames.numel(), enc.frame_off.data_ptr(),
                                         hint + 7, n, None, *[t.data_ptr() for t in outs], None, 7, 0, stream)
    ref, exact = None, {}
    for name, h in libs.items():
        for t in outs:
            t.zero_()
        assert call(h) == 0
        got = torch.cat([t.view(torch.uint8) for t in outs])
        ref = got if ref is None else ref
        exact[name] = bool(torch.equal(got, ref))
    all_valid = bool((outs[5] == 1).all().item()) and (validate or bool((outs[3] == 1).all().item()))
    times = {k: [] for k in libs}
    for _ in range(reps):
        for name, h in libs.items():
            for _ in range(2):
                call(h)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                call(h)
            e.record()
            e.synchronize()
            times[name].append(s.elapsed_time(e) / 10)
    return {"ms": {k: statistics.median(v) for k, v in times.items()}, "exact": exact, "all_valid_verified": all_valid}


if __name__ == "__main__":
    main()
