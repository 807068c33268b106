"""Kernel variant sweep on one GPU (interleaved A/B, median of repeats).

Times encode launch-policy variants (rudpx_tune), decode paths, and the
streaming-copy ceiling, on the BASELINE shapes.  Output: one JSON object.
usage: python tools/sweep.py [--reps 15] [--only encode|decode|copy]
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

from rudp import _native, batch  # noqa: E402

lib = _native.tools_lib()
lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
lib.rudpx_tune.restype = ctypes.c_int
lib.rudpx_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                           ctypes.c_void_p]
lib.rudpx_copy.restype = ctypes.c_int
lib.rudpx_copy_vpt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                               ctypes.c_int, ctypes.c_void_p]
lib.rudpx_copy_vpt.restype = ctypes.c_int
lib.rudpx_copy_tile.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_void_p]
lib.rudpx_copy_tile.restype = ctypes.c_int
lib.rudpx_copy_tile_pipe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
lib.rudpx_copy_tile_pipe.restype = ctypes.c_int
lib.rudpx_copy_tile_dma.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
lib.rudpx_copy_tile_dma.restype = ctypes.c_int


def event_ms(fn, reps=1):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def interleaved(variants, reps):
    """variants: name -> (setup, fn).  Returns name -> median ms."""
    times = {k: [] for k in variants}
    for _ in range(reps):
        for k, (setup, fn) in variants.items():
            setup()
            fn()  # warm (and re-apply the setting's kernel)
            times[k].append(event_ms(fn, 3))
    return {k: statistics.median(v) for k, v in times.items()}


BLOCKS_OVERRIDE = None
ENCODE_LS = None
PERCU_OVERRIDE = None      # encode: tiles-per-CU caps to try (256-thread blocks)
TILES_OVERRIDE = None      # encode: packets per tile to try
VDEC_CAP_PCTS = ()         # vdec: extra varlen-decode tile LDS budgets (% of the hinted run)
GEOMETRY_VARIANTS = False


def encode_sweep(reps):
    out = {}
    dev = torch.device("cuda", 0)
    shapes = ((1472, (0, 4, 8, 16)), (1024, (0, 4, 8, 16)), (64, (0, 16, 32, 64, 128)))
    for L, tiles in (s for s in shapes if not ENCODE_LS or s[0] in ENCODE_LS):
        n = 1 << 20
        nsets = 1 if L > 512 else 7
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
        it = [0]

        def run():
            tab, pay, fr = sets[it[0] % nsets]
            it[0] += 1
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)

        variants = {}
        blocks = BLOCKS_OVERRIDE or (64, 128, 256)
        for block in blocks:
            for tile in (TILES_OVERRIDE or tiles):
                if tile > block:
                    continue
                for per_cu in ((PERCU_OVERRIDE or (-1, 0, 5)) if block == 256 else (0, 16, 24) if block < 256 else (0, 2, 3)):
                    def setup(tile=tile, per_cu=per_cu, block=block):
                        lib.rudpx_tune(10, block)
                        lib.rudpx_tune(2, tile)
                        lib.rudpx_tune(6, per_cu)
                    variants[f"L{L}_b{block}_tile{tile}_percu{per_cu}"] = (setup, run)
        res = interleaved(variants, reps)
        alg = n * (2 * L + 12)
        # every variant must produce the default kernel's frames bit for bit
        tab0, pay0, _ = sets[0]
        lib.rudpx_tune(3, 8), lib.rudpx_tune(6, -1), lib.rudpx_tune(10, 256), lib.rudpx_tune(2, 0)
        want, _ = batch.pack_batch(tab0, pay0, 7)  # the default kernel
        for k, (setup, _) in variants.items():
            setup()
            got, _ = batch.pack_batch(tab0, pay0, 7)
            res[k] = (res[k], bool(torch.equal(got, want)))
        for k, (ms, same) in res.items():
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0, "exact": same}
        del sets
        torch.cuda.empty_cache()
    lib.rudpx_tune(0, 1)
    lib.rudpx_tune(1, 1)
    lib.rudpx_tune(2, 0)
    lib.rudpx_tune(3, 8)
    lib.rudpx_tune(5, -1)
    lib.rudpx_tune(6, -1)
    lib.rudpx_tune(10, 256)
    return out


def align_sweep(reps, key=23, values=(1, 0), names=("align64", "align16")):
    """Encode / verify / copy-out decode / varlen encode under one rudpx_tune knob:
    by default phase-2 wave stores on 64-B sector boundaries (key 23) or not."""
    out = {}
    dev = torch.device("cuda", 0)
    for L in (ENCODE_LS or (1472, 1024, 64)):
        n = 1 << 20
        nsets = 1 if L > 512 else 7
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
        it = [0]

        def run():
            tab, pay, fr = sets[it[0] % nsets]
            it[0] += 1
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        pay_out = torch.empty((n, L), dtype=torch.uint8, device=dev)
        o16 = torch.empty(n, dtype=torch.uint16, device=dev)
        o8 = torch.empty(n, dtype=torch.uint8, device=dev)
        for tab, pay, fr in sets:
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)

        def verify():  # raw ABI, preallocated outputs (the Python entry's allocations hide small L)
            fr = sets[it[0] % nsets][2]
            it[0] += 1
            _native.check(lib.rudp_decode(fr.data_ptr(), None, L + 7, n, None, o16.data_ptr(),
                                          o16.data_ptr(), o8.data_ptr(), o8.data_ptr(), o16.data_ptr(),
                                          None, 7, 0, torch.cuda.current_stream().cuda_stream))

        def copyout():
            fr = sets[it[0] % nsets][2]
            it[0] += 1
            _native.check(lib.rudp_decode(fr.data_ptr(), None, L + 7, n, None, o16.data_ptr(),
                                          o16.data_ptr(), o8.data_ptr(), o8.data_ptr(), None,
                                          pay_out.data_ptr(), 7, 0, torch.cuda.current_stream().cuda_stream))
        lens = torch.full((n,), L, dtype=torch.int32, device=dev)

        def venc():
            tab, pay, _ = sets[it[0] % nsets]
            it[0] += 1
            batch.pack_batch_varlen(tab, pay.view(-1), lens, 7)
        algs = {"encode": n * (2 * L + 12), "verify": n * (L + 13), "copyout": n * (2 * L + 13),
                "varlen_encode": n * (2 * L + 24)}
        variants = {}
        old = lib.rudpx_tune(key, values[0])
        lib.rudpx_tune(key, old)
        for op, fn in (("encode", run), ("verify", verify), ("copyout", copyout), ("varlen_encode", venc)):
            for v, nm in zip(values, names):
                variants[f"L{L}_{op}_{nm}"] = (lambda v=v: lib.rudpx_tune(key, v), fn)
        res = interleaved(variants, reps)
        lib.rudpx_tune(key, old)
        for k, ms in res.items():
            alg = algs[k.split("_", 1)[1].rsplit("_", 1)[0]]
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del sets
        torch.cuda.empty_cache()
    return out


def knob_sweep(reps, key, values, pre=()):
    """Encode with one rudpx_tune knob at each of `values` (bit-exact check against the first);
    `pre`: (key, value) settings held for the whole sweep."""
    out = {}
    for k, v in pre:
        lib.rudpx_tune(k, v)
    dev = torch.device("cuda", 0)
    for L in (ENCODE_LS or (1472, 1024, 64)):
        n = 1 << 20
        nsets = 1 if L > 512 else 7
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
        it = [0]

        def run():
            tab, pay, fr = sets[it[0] % nsets]
            it[0] += 1
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        old = lib.rudpx_tune(key, values[0])
        lib.rudpx_tune(key, old)
        variants = {f"L{L}_key{key}_{v}": ((lambda v=v: lib.rudpx_tune(key, v)), run) for v in values}
        res = interleaved(variants, reps)
        tab0, pay0, _ = sets[0]
        lib.rudpx_tune(key, values[0])
        want, _ = batch.pack_batch(tab0, pay0, 7)
        alg = n * (2 * L + 12)
        for v in values:
            lib.rudpx_tune(key, v)
            got, _ = batch.pack_batch(tab0, pay0, 7)
            k = f"L{L}_key{key}_{v}"
            ms = res[k]
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0,
                      "exact": bool(torch.equal(got, want))}
        lib.rudpx_tune(key, old)
        del sets
        torch.cuda.empty_cache()
    return out


def multi_sweep(reps, specs):
    """Encode under named settings: specs = [(name, [(key, value), ...])]; the
    first is the reference for the bit-exact check.  Knobs are restored after."""
    out = {}
    dev = torch.device("cuda", 0)
    keys = sorted({k for _, kv in specs for k, _ in kv})
    for L in (ENCODE_LS or (1472, 1024, 64)):
        n = 1 << 20
        nsets = 1 if L > 512 else 7
        sets = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            sets.append((tab, pay, torch.empty((n, L + 7), dtype=torch.uint8, device=dev)))
        it = [0]

        def run():
            tab, pay, fr = sets[it[0] % nsets]
            it[0] += 1
            batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
        defaults = {}
        for k in keys:  # read each knob's default (set returns the old value)
            defaults[k] = lib.rudpx_tune(k, 0)
            lib.rudpx_tune(k, defaults[k])

        def apply(kv):
            for k in keys:
                lib.rudpx_tune(k, defaults[k])
            for k, v in kv:
                lib.rudpx_tune(k, v)
        variants = {f"L{L}_{name}": ((lambda kv=kv: apply(kv)), run) for name, kv in specs}
        res = interleaved(variants, reps)
        tab0, pay0, _ = sets[0]
        alg = n * (2 * L + 12)
        want = None
        for name, kv in specs:
            apply(kv)
            got, _ = batch.pack_batch(tab0, pay0, 7)
            want = got if want is None else want
            ms = res[f"L{L}_{name}"]
            out[f"L{L}_{name}"] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0,
                                   "exact": bool(torch.equal(got, want))}
        apply([])
        del sets
        torch.cuda.empty_cache()
    return out


def vdec_sweep(reps):
    """Varlen decode through the raw ABI (preallocated outputs, hint = mean frame
    length): LDS-tile kernel (rudpx_tune 33 = 1) vs per-frame vector kernel (0)."""
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    for L in (1, 64, 256, 1024, 1472, -1):  # -1: lengths uniform in [0, 2944]
        n = 1 << 20
        tab, pay = batch.synth_batch(n, max(L, 2944), 0x5EED0007, device=dev)
        if L >= 0:
            lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        else:
            lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev)
        mean = int(lens.double().mean().item()) + 7
        flat = pay.view(-1)[: int(lens.sum().item())] if L < 0 else pay[:, :max(L, 0)].contiguous().view(-1)
        nsets = max(1, min(8, -(-(1 << 30) // (n * mean))))
        sets = []
        for _ in range(nsets):
            r = batch.pack_batch_varlen(tab, flat, lens, 7)
            sets.append((r.frames, r.frame_off))
        o16 = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(3)]
        o8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        it = [0]

        def run():
            frames, off = sets[it[0] % nsets]
            it[0] += 1
            _native.check(lib.rudp_decode(frames.data_ptr(), off.data_ptr(), mean, n, None,
                                          o16[0].data_ptr(), o16[1].data_ptr(), o8[0].data_ptr(),
                                          o8[1].data_ptr(), o16[2].data_ptr(), None, 7, 0, stream))
        name = f"L{L}" if L >= 0 else "U0-2944"
        variants = {f"{name}_tile": (lambda: (lib.rudpx_tune(33, 2), lib.rudpx_tune(38, 110)), run),
                    f"{name}_vec": (lambda: lib.rudpx_tune(33, 0), run)}
        for pct in VDEC_CAP_PCTS:
            variants[f"{name}_tile_cap{pct}"] = (lambda pct=pct: (lib.rudpx_tune(33, 2), lib.rudpx_tune(38, pct)), run)
        res = interleaved(variants, reps)
        lib.rudpx_tune(33, 1)
        lib.rudpx_tune(38, 110)
        alg = n * (mean + 8 + 8)  # frames + offsets read, seq/ack/flags/ok/csum written
        for k, ms in res.items():
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del sets, tab, pay, flat, lens
        torch.cuda.empty_cache()
    return out


def vknob_sweep(reps, key, values, pre=()):
    """Varlen encode (Python entry: bounds check, offset scan, tile kernel) and
    varlen decode-verify (raw ABI, preallocated outputs) with one rudpx_tune
    knob at each of `values`; outputs checked bit-exact against the first."""
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    held = [(k, lib.rudpx_tune(k, v)) for k, v in pre]  # settings held for the whole sweep
    old = lib.rudpx_tune(key, values[0])
    lib.rudpx_tune(key, old)
    for L in (1472, 1024, 512, 256, -1):  # -1: lengths uniform in [0, 2944]
        n = 1 << 20
        tab, pay = batch.synth_batch(n, max(L, 2944), 0x5EED0009, device=dev)
        if L >= 0:
            lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        else:
            lens = torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev)
        flat = pay.view(-1)[: int(lens.sum().item())] if L < 0 else pay[:, :L].contiguous().view(-1)
        del pay
        mean = int(lens.double().mean().item()) + 7
        ref = batch.pack_batch_varlen(tab, flat, lens, 7)
        o16 = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(3)]
        o8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]

        def enc():
            batch.pack_batch_varlen(tab, flat, lens, 7)

        def dec():
            _native.check(lib.rudp_decode(ref.frames.data_ptr(), ref.frame_off.data_ptr(), mean, n, None,
                                          o16[0].data_ptr(), o16[1].data_ptr(), o8[0].data_ptr(),
                                          o8[1].data_ptr(), o16[2].data_ptr(), None, 7, 0, stream))
        def utf():
            batch.validate_utf8(ref.frames, "rudp7", frame_off=ref.frame_off)
        name = f"L{L}" if L >= 0 else "U0-2944"
        variants = {}
        for v in values:
            variants[f"{name}_enc_key{key}_{v}"] = ((lambda v=v: lib.rudpx_tune(key, v)), enc)
            variants[f"{name}_dec_key{key}_{v}"] = ((lambda v=v: lib.rudpx_tune(key, v)), dec)
            variants[f"{name}_utf_key{key}_{v}"] = ((lambda v=v: lib.rudpx_tune(key, v)), utf)
        res = interleaved(variants, reps)
        exact = {}
        for v in values:
            lib.rudpx_tune(key, v)
            r = batch.pack_batch_varlen(tab, flat, lens, 7)
            dec()
            ok_all = bool((o8[1] == 1).all().item())
            u = batch.validate_utf8(ref.frames, "rudp7", frame_off=ref.frame_off)
            if v == values[0]:
                u0 = u.clone()
            exact[v] = bool(torch.equal(r.frames, ref.frames)) and ok_all and bool(torch.equal(u, u0))
        lib.rudpx_tune(key, old)
        alg_e = n * (2 * mean + 12)
        alg_d = n * (mean + 8 + 8)
        for k, ms in res.items():
            alg = alg_e if "_enc_" in k else alg_d  # utf: frames + offsets read, as decode
            out[k] = {"ms": ms, "frac": alg / ms / 1e9 / 8.0, "exact": exact[int(k.rsplit("_", 1)[1])]}
        del ref, tab, flat, lens
        torch.cuda.empty_cache()
    for k, v in reversed(held):
        lib.rudpx_tune(k, v)
    return out


def small_sweep(reps):
    """Small frames (the reference's one-character datagrams and a few other
    tiny shapes): varlen encode and decode-verify through the sync-free C ABI
    (preallocated outputs), with the small-frame tile kernels at 1/2/4/8
    packets per thread (keys 46/47), two or three launches (key 50), against
    the per-packet vector kernels.
    Every variant is checked bit-exact against the vector kernels."""
    import ctypes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    specs = {"vec": ((46, 0), (50, 1)), "fpt1": ((46, 16), (47, 1), (50, 1)), "fpt2": ((46, 16), (47, 2), (50, 1)),
             "fpt4": ((46, 16), (47, 4), (50, 1)), "fpt8": ((46, 16), (47, 8), (50, 1)),
             "auto": ((46, 16), (47, 0), (50, 1)), "auto_3launch": ((46, 16), (47, 0), (50, 0))}
    old = {k: lib.rudpx_tune(k, 0) for k in (46, 47, 50)}
    for k, v in old.items():
        lib.rudpx_tune(k, v)
    for shape in ("L1", "L4", "U1-4", "L9", "L15"):
        n = 1 << 20
        if shape.startswith("U"):
            lens = torch.randint(1, 5, (n,), dtype=torch.int32, device=dev)
        else:
            lens = torch.full((n,), int(shape[1:]), dtype=torch.int32, device=dev)
        total = int(lens.sum().item())
        tab, pay = batch.synth_batch(n, 16, 0x5EED000B, device=dev)
        flat = pay.view(-1)[:total].contiguous()
        del pay
        H = 7
        hint = total // n
        frames = torch.empty(total + n * H, dtype=torch.uint8, device=dev)
        off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        st = torch.empty(1, dtype=torch.int32, device=dev)
        o16 = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(3)]
        o8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                              flags=tab.flags.data_ptr(), payload=flat.data_ptr(), len=lens.data_ptr(),
                              payload_off=None)

        def enc():
            _native.check(lib.rudp_encode_varlen_checked(ctypes.byref(b), total, frames.data_ptr(), frames.numel(),
                                                         off.data_ptr(), None, st.data_ptr(), H, 0, stream))

        def dec():
            _native.check(lib.rudp_decode_varlen_checked(frames.data_ptr(), frames.numel(), off.data_ptr(),
                                                         frames.numel() // n, n, None, o16[0].data_ptr(),
                                                         o16[1].data_ptr(), o8[0].data_ptr(), o8[1].data_ptr(),
                                                         o16[2].data_ptr(), st.data_ptr(), H, 0, stream))

        def setter(kv):
            return lambda: [lib.rudpx_tune(k, v) for k, v in kv]
        variants = {}
        for name, kv in specs.items():
            variants[f"{shape}_enc_{name}"] = (setter(kv), enc)
            variants[f"{shape}_dec_{name}"] = (setter(kv), dec)
        res = interleaved(variants, reps)
        ref = None
        exact = {}
        for name, kv in specs.items():
            setter(kv)()
            enc()
            dec()
            got = (frames.clone(), off.clone(), [o.clone() for o in o16 + o8])
            if ref is None:
                ref = got
            exact[name] = (torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
                           and all(torch.equal(x, y) for x, y in zip(got[2], ref[2]))
                           and bool((o8[1] == 1).all().item()) and int(st.item()) == 0)
        for k, v in old.items():
            lib.rudpx_tune(k, v)
        mean_f = (total + n * H) / n
        alg_e = n * (4 + total / n + 5 + mean_f + 8)      # len, payload, table in; frames, offsets out
        alg_d = n * (mean_f + 8 + 8)                      # frames, offsets in; seq/ack/flags/ok/csum out
        for k, ms in res.items():
            alg = alg_e if "_enc_" in k else alg_d
            out[k] = {"ms": ms, "frac": alg / ms / 1e9 / 8.0, "exact": exact[k.split("_", 2)[2]]}
        del tab, flat, lens, frames, off
        torch.cuda.empty_cache()
    return out


def ragged_sweep(reps):
    """Where ragged varlen encode loses (lengths uniform in [0, 2944], mean
    1472, against equal 1472-B lengths): stage ablations of the tile kernel
    (key 35: 2 = no sum pass, 4 = overflowing tiles skipped; wrong output, so
    not checked) and LDS budgets (key 39), through the sync-free C ABI.
    Also counts the tiles whose payload run exceeds the default budget."""
    import ctypes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    n, H = 1 << 20, 7
    out = {}
    torch.manual_seed(11)
    for shape in ("U0-2944", "L1472"):
        lens = (torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev) if shape[0] == "U"
                else torch.full((n,), 1472, dtype=torch.int32, device=dev))
        total = int(lens.sum().item())
        tab, pay = batch.synth_batch(n, 2944, 0x5EED000C, device=dev)
        flat = pay.view(-1)[:total].contiguous()
        del pay
        frames = torch.empty(total + n * H, dtype=torch.uint8, device=dev)
        off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        st = torch.empty(1, dtype=torch.int32, device=dev)
        b = _native.RudpBatch(n=n, payload_len=total // n, reserved=0, seq=tab.seq.data_ptr(),
                              ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(), payload=flat.data_ptr(),
                              len=lens.data_ptr(), payload_off=None)

        def enc():
            _native.check(lib.rudp_encode_varlen_checked(ctypes.byref(b), total, frames.data_ptr(),
                                                         frames.numel(), off.data_ptr(), None, st.data_ptr(),
                                                         H, 0, stream))
        specs = {"default": (), "no_sums": ((35, 2),), "skip_overflow": ((35, 4),),
                 "no_sums_skip_overflow": ((35, 6),), "cap125": ((39, 125),), "cap150": ((39, 150),),
                 "cap200": ((39, 200),), "no_hchunk": ((36, 0),), "btile": ((51, 2),),
                 "btile_no_sums": ((51, 2), (35, 2)), "chunksums": ((52, 0),), "packet": ((51, 0),)}
        variants = {}
        for name, kv in specs.items():
            def setup(kv=kv):
                for k, v in ((35, 0), (39, 110), (36, 2), (51, 1), (52, 2)):
                    lib.rudpx_tune(k, v)
                for k, v in kv:
                    lib.rudpx_tune(k, v)
            variants[f"{shape}_{name}"] = (setup, enc)
        res = interleaved(variants, reps)
        exact = {}
        ref = None
        for name, kv in specs.items():
            if "no_" in name or "skip" in name:
                continue
            variants[f"{shape}_{name}"][0]()
            enc()
            if ref is None:
                ref = (frames.clone(), off.clone())
            exact[name] = bool(torch.equal(frames, ref[0]) and torch.equal(off, ref[1]) and int(st.item()) == 0)
        for k, v in ((35, 0), (39, 110), (36, 2), (51, 1), (52, 2)):
            lib.rudpx_tune(k, v)
        # tiles of 16 packets whose payload run exceeds 1.1x the hinted run (+ alignment slack)
        runs = lens[: (n // 16) * 16].view(-1, 16).sum(1)
        over = float((runs > (16 * (total // n) * 110 // 100 + 256 - 32)).float().mean().item())
        alg = n * (2 * (total / n + H) + 12)
        for k, ms in res.items():
            out[k] = {"ms": ms, "frac": alg / ms / 1e9 / 8.0, "exact": exact.get(k.split("_", 1)[1])}
        out[f"{shape}_overflow_tile_fraction"] = over
        del tab, flat, lens, frames, off
        torch.cuda.empty_cache()
    return out


def decode_sweep(reps):
    dev = torch.device("cuda", 0)
    out = {}
    for L in (1472, 1024, 256, 64):
        n = 1 << 20
        nsets = 1 if L > 512 else 7
        frs = []
        for _ in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
            fr, _ = batch.pack_batch(tab, pay, 7)
            frs.append(fr)
        pay_out = torch.empty((n, L), dtype=torch.uint8, device=dev)
        it = [0]

        def verify():
            batch.unpack_batch(frs[it[0] % nsets], 7)
            it[0] += 1

        def copy():
            f = frs[it[0] % nsets]
            it[0] += 1
            # copy-out path through the raw ABI with a preallocated output
            seq = torch.empty(n, dtype=torch.uint16, device=dev)
            ok = torch.empty(n, dtype=torch.uint8, device=dev)
            _native.check(lib.rudp_decode(f.data_ptr(), None, L + 7, n, None, seq.data_ptr(),
                                          seq.data_ptr(), ok.data_ptr(), ok.data_ptr(), None,
                                          pay_out.data_ptr(), 7, 0,
                                          torch.cuda.current_stream().cuda_stream))
        variants = {f"L{L}_copyout_tile": (lambda: (lib.rudpx_tune(4, -1), lib.rudpx_tune(11, 1)), copy),
                    f"L{L}_copyout_regs": (lambda: (lib.rudpx_tune(4, -1), lib.rudpx_tune(11, 0)), copy)}
        variants[f"L{L}_verify_chunks"] = (lambda: (lib.rudpx_tune(4, -1), lib.rudpx_tune(12, 0)), verify)
        variants[f"L{L}_verify_tile"] = (lambda: (lib.rudpx_tune(4, -1), lib.rudpx_tune(12, 1)), verify)
        if L <= 256:
            for lg in (0, 1, 2):
                variants[f"L{L}_verify_tile_glog{lg}"] = (
                    lambda lg=lg: (lib.rudpx_tune(12, 1), lib.rudpx_tune(4, lg)), verify)
                variants[f"L{L}_copyout_tile_glog{lg}"] = (
                    lambda lg=lg: (lib.rudpx_tune(11, 1), lib.rudpx_tune(4, lg)), copy)
        res = interleaved(variants, reps)
        lib.rudpx_tune(4, -1)
        lib.rudpx_tune(11, 1)
        lib.rudpx_tune(12, 1)
        for k, ms in res.items():
            alg = n * (L + 13) if "verify" in k else n * (2 * L + 13)
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del frs
        torch.cuda.empty_cache()
    return out


def copy_sweep(reps):
    dev = torch.device("cuda", 0)
    nbytes = 1 << 20 << 10 >> 0  # placeholder, replaced below
    nbytes = (1 << 20) * 1472
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(7)
    stream = torch.cuda.current_stream().cuda_stream
    variants = {}
    for blocks in (65536,):
        variants[f"copy_blocks{blocks}"] = (
            lambda: None,
            lambda blocks=blocks: lib.rudpx_copy(a.data_ptr(), b.data_ptr(), nbytes // 16, blocks, stream))
    variants["torch_copy_"] = (lambda: None, lambda: b.copy_(a))
    for vpt in (1, 4):
        for pol in (0, 1):
            variants[f"copy_vpt{vpt}_nt{pol}"] = (
                lambda: None,
                lambda vpt=vpt, pol=pol: lib.rudpx_copy_vpt(a.data_ptr(), b.data_ptr(), nbytes // 16,
                                                            vpt, pol, stream))
    for kb in (4, 8, 12, 24):
        for per_cu in (0, 5):
            lds = (160 * 1024 // per_cu) & ~15 if per_cu else 0
            variants[f"copy_tile{kb}k_percu{per_cu}"] = (
                lambda: None,
                lambda kb=kb, lds=lds: lib.rudpx_copy_tile(a.data_ptr(), b.data_ptr(), nbytes // 16,
                                                           kb * 64, lds, stream))
    for kb in (8, 12, 24):
        for per_cu in (2, 4, 6, 8):
            variants[f"copy_pipe{kb}k_blocks{per_cu}x256"] = (
                lambda: None,
                lambda kb=kb, per_cu=per_cu: lib.rudpx_copy_tile_pipe(
                    a.data_ptr(), b.data_ptr(), nbytes // 16, kb * 64, per_cu * 256, 0, stream))
    res = interleaved(variants, reps)
    return {k: {"ms": ms, "TBs": 2 * nbytes / ms / 1e9} for k, ms in res.items()}


def copydma_sweep(reps):
    """Tiled copies staged by LDS-DMA, one tile per block or persistent double-buffered."""
    dev = torch.device("cuda", 0)
    nbytes = (1 << 20) * 1472
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(7)
    stream = torch.cuda.current_stream().cuda_stream
    n16 = nbytes // 16
    variants = {"copy_vpt1_nt1": (lambda: None, lambda: lib.rudpx_copy_vpt(a.data_ptr(), b.data_ptr(), n16, 1, 1, stream))}
    for kb in (8, 24):
        for per_cu in (0, 5):
            lds = (160 * 1024 // per_cu) & ~15 if per_cu else 0
            variants[f"regs_tile{kb}k_percu{per_cu}"] = (
                lambda: None, lambda kb=kb, lds=lds: lib.rudpx_copy_tile(a.data_ptr(), b.data_ptr(), n16, kb * 64, lds, stream))
            variants[f"dma_tile{kb}k_percu{per_cu}"] = (
                lambda: None, lambda kb=kb, lds=lds: lib.rudpx_copy_tile_dma(a.data_ptr(), b.data_ptr(), n16, kb * 64, 0, lds, 0, stream))
    for kb in (8, 12, 24):
        for per_cu in (1, 2, 3, 4, 6):
            if 2 * kb * per_cu > 160:
                continue
            variants[f"dma_pipe{kb}k_blocks{per_cu}x256"] = (
                lambda: None, lambda kb=kb, per_cu=per_cu: lib.rudpx_copy_tile_dma(
                    a.data_ptr(), b.data_ptr(), n16, kb * 64, per_cu * 256, (160 * 1024 // per_cu) & ~15, 1, stream))
    res = interleaved(variants, reps)
    torch.cuda.synchronize()
    assert torch.equal(a, b), "copy mismatch"
    return {k: {"ms": ms, "TBs": 2 * nbytes / ms / 1e9} for k, ms in res.items()}


ABLATE_L = 1472


def ablate_sweep(reps):
    """Encode with stages switched off (inexact on purpose) beside LDS-tiled copies."""
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, ABLATE_L
    tab, pay = batch.synth_batch(n, L, 0x5EED0004, device=dev)
    fr = torch.empty((n, L + 7), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    variants = {}
    for tile in ((8, 16) if L >= 1024 else (128, 256)):
        for abl in range(8):
            def setup(tile=tile, abl=abl):
                lib.rudpx_tune(2, tile)
                lib.rudpx_tune(13, abl)
            variants[f"tile{tile}_ablate{abl}"] = (
                setup, lambda: batch.pack_batch(tab, pay, 7, out=fr, want_csum=False))
    a = pay.view(-1)
    b = fr.view(-1)[: a.numel()]
    for kb in ((12, 24) if L >= 1024 else (8, 16)):
        t16 = (kb * 1024 * 23 // 24) // 16 if kb == 24 else (kb * 1024 // 16)
        variants[f"copy_tile{kb}k"] = (lambda: None, lambda t16=t16: lib.rudpx_copy_tile(
            a.data_ptr(), b.data_ptr(), a.numel() // 16, t16, 0, stream))
    res = interleaved(variants, reps)
    lib.rudpx_tune(2, 0)
    lib.rudpx_tune(13, 0)
    alg = n * (2 * L + 12)
    return {k: {"ms": ms, "TBs": (alg if "tile" in k and "copy" not in k else 2 * a.numel()) / ms / 1e9}
            for k, ms in res.items()}


def varlen_sweep(reps):
    """Varlen decode (raw ABI, preallocated outputs): vector kernel vs byte kernel."""
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    for L in (1, 64, 1024, 1472):
        n = 1 << 20
        tab, pay = batch.synth_batch(n, L, 0x5EED0007, device=dev)
        lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        res = batch.pack_batch_varlen(tab, pay.view(-1), lens, 7)
        frames, off = res.frames, res.frame_off
        o16 = [torch.empty(n, dtype=torch.uint16, device=dev) for _ in range(3)]
        o8 = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]

        def run(hint):
            _native.check(lib.rudp_decode(frames.data_ptr(), off.data_ptr(), hint, n, None,
                                          o16[0].data_ptr(), o16[1].data_ptr(), o8[0].data_ptr(),
                                          o8[1].data_ptr(), o16[2].data_ptr(), None, 7, 0, stream))
        fr2 = torch.empty_like(frames)
        off2 = torch.empty_like(off)
        flat = pay.view(-1)

        def enc(hint):
            b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab.seq.data_ptr(),
                                  ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(),
                                  payload=flat.data_ptr(), len=lens.data_ptr(), payload_off=None)
            _native.check(lib.rudp_encode_varlen(ctypes.byref(b), fr2.data_ptr(), off2.data_ptr(),
                                                 None, 7, 0, stream))
        variants = {f"L{L}_bytes": (lambda: (lib.rudpx_tune(15, -1), lib.rudpx_tune(14, 0)), lambda: run(L + 7)),
                    f"L{L}_enc_bytes": (lambda: (lib.rudpx_tune(15, -1), lib.rudpx_tune(14, 0)), lambda: enc(L))}
        for lg in (range(2, 7) if L >= 1024 else ()):
            variants[f"L{L}_vec_glog{lg}"] = (lambda lg=lg: (lib.rudpx_tune(14, 1), lib.rudpx_tune(15, lg)),
                                              lambda: run(L + 7))
            variants[f"L{L}_enc_vec_glog{lg}"] = (lambda lg=lg: (lib.rudpx_tune(14, 1), lib.rudpx_tune(15, lg)),
                                                  lambda: enc(L))
        for hint in sorted({0, L + 7, 64, 1479}):
            variants[f"L{L}_vec_hint{hint}"] = (lambda: (lib.rudpx_tune(15, -1), lib.rudpx_tune(14, 1)),
                                                lambda hint=hint: run(hint))
            variants[f"L{L}_enc_vec_hint{hint}"] = (lambda: (lib.rudpx_tune(15, -1), lib.rudpx_tune(14, 1)),
                                                    lambda hint=hint: enc(hint))
        res_t = interleaved(variants, reps)
        lib.rudpx_tune(14, 1)
        lib.rudpx_tune(15, -1)
        for k, ms in res_t.items():
            # decode: frames + offsets read, seq/ack/flags/ok/csum written;
            # encode: payload + len + header table read, frames + offsets written
            alg = n * (2 * L + 7 + 9 + 8) if "_enc_" in k else n * (L + 7 + 8 + 8)
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del fr2, off2, flat
        del frames, off, res, tab, pay
        torch.cuda.empty_cache()
    return out


def varlen_enc_sweep(reps):
    """Varlen encode of packed payloads: LDS-tile kernel vs per-packet vector kernel."""
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    n = 1 << 20
    for name in ("L1", "L64", "L1024", "L1472", "U0-2944"):
        if name.startswith("U"):
            g = torch.Generator(device=dev)
            g.manual_seed(7)
            lens = torch.randint(0, 2945, (n,), device=dev, generator=g, dtype=torch.int32)
        else:
            lens = torch.full((n,), int(name[1:]), dtype=torch.int32, device=dev)
        total = int(lens.sum().item())
        flat = torch.randint(0, 128, (total,), dtype=torch.uint8, device=dev)
        tab, _ = batch.synth_batch(n, 0, 0x5EED0007, device=dev)
        hint = total // n
        fr = torch.empty(total + 7 * n, dtype=torch.uint8, device=dev)
        off = torch.empty(n + 1, dtype=torch.int64, device=dev)

        def enc(hint=hint, flat=flat, lens=lens, fr=fr, off=off, tab=tab):
            b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab.seq.data_ptr(),
                                  ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(),
                                  payload=flat.data_ptr(), len=lens.data_ptr(), payload_off=None)
            _native.check(lib.rudp_encode_varlen(ctypes.byref(b), fr.data_ptr(), off.data_ptr(),
                                                 None, 7, 0, stream))
        def cfg(tile, maxT=256, nbytes=0):  # nbytes 0: the automatic tile size
            return lambda: (lib.rudpx_tune(16, tile), lib.rudpx_tune(17, maxT), lib.rudpx_tune(18, nbytes))
        variants = {f"{name}_tile": (cfg(1), enc), f"{name}_vec": (cfg(0), enc),
                    f"{name}_tile_hipcub": (lambda: (cfg(1)(), lib.rudpx_tune(24, 0)), enc)}
        variants[f"{name}_tile"] = (lambda: (cfg(1)(), lib.rudpx_tune(24, 1)), enc)
        variants[f"{name}_vec"] = (lambda: (cfg(0)(), lib.rudpx_tune(24, 1)), enc)
        if GEOMETRY_VARIANTS:
            for maxT in (64, 128):
                variants[f"{name}_tile_maxT{maxT}"] = (cfg(1, maxT), enc)
            for nbytes in (8192, 12288, 16384, 32768):
                variants[f"{name}_tile_bytes{nbytes}"] = (cfg(1, 256, nbytes), enc)
        res = interleaved(variants, reps)
        cfg(1)()
        lib.rudpx_tune(24, 1)
        # payload + len + header table read; frames + offsets written (scan included)
        alg = 2 * total + n * (7 + 9 + 8)
        for k, ms in res.items():
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del flat, fr, off, lens, tab
        torch.cuda.empty_cache()
    return out


def utf8_sweep(reps):
    """Strict UTF-8 validation over fixed-length frames (ASCII and random payloads),
    LDS-tile kernel (rudpx_tune 31 = 1) against the per-frame vector kernel (0);
    buffer sets rotate so every launch streams from HBM."""
    dev = torch.device("cuda", 0)
    out = {}
    for L in (ENCODE_LS or (1472, 1024, 256, 64)):
        n = 1 << 20
        nsets = max(1, min(8, -(-(1 << 30) // (n * (L + 7)))))
        variants = {}
        for ascii in (True, False):
            frs = []
            for i in range(nsets):
                tab, pay = batch.synth_batch(n, L, 0x5EED0009 + i, ascii=ascii, device=dev)
                frs.append(batch.pack_batch(tab, pay, 7)[0])
            it = [0]

            def run(frs=frs, it=it):
                batch.validate_utf8(frs[it[0] % len(frs)], 7)
                it[0] += 1
            for tile in (1, 0):
                variants[f"L{L}_{'ascii' if ascii else 'random'}_tile{tile}"] = (
                    lambda tile=tile: lib.rudpx_tune(31, tile), run)
        res = interleaved(variants, reps)
        lib.rudpx_tune(31, 1)
        for k, ms in res.items():
            alg = n * (L + 7 + 1)
            out[k] = {"ms": ms, "TBs": alg / ms / 1e9, "frac": alg / ms / 1e9 / 8.0}
        del variants
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--L", type=int, default=1472, help="payload length for --only ablate")
    ap.add_argument("--only", choices=["encode", "decode", "copy", "ablate", "varlen", "varlen_enc", "utf8", "small", "ragged", "align", "knob", "copydma", "multi", "opsknob", "vdec", "vknob"])
    ap.add_argument("--blocks", type=str, default="", help="encode sweep: workgroup sizes, e.g. 256,512,1024")
    ap.add_argument("--encode-L", type=str, default="", help="encode sweep: payload lengths, e.g. 1472")
    ap.add_argument("--percu", type=str, default="", help="encode sweep: tiles-per-CU caps, e.g. 3,4,5")
    ap.add_argument("--key", type=int, default=25, help="--only knob: rudpx_tune key")
    ap.add_argument("--values", type=str, default="0,1", help="--only knob: values (first = reference)")
    ap.add_argument("--pre", type=str, default="", help="--only knob: held settings, e.g. 26=1,6=4")
    ap.add_argument("--specs", type=str, default="",
                    help="--only multi: name:key=val,key=val;name2:... (first = reference)")
    ap.add_argument("--tiles", type=str, default="", help="encode sweep: packets per tile, e.g. 8,16")
    args = ap.parse_args()
    global BLOCKS_OVERRIDE, ENCODE_LS, PERCU_OVERRIDE, TILES_OVERRIDE
    if args.percu:
        PERCU_OVERRIDE = tuple(int(x) for x in args.percu.split(","))
    if args.tiles:
        TILES_OVERRIDE = tuple(int(x) for x in args.tiles.split(","))
    if args.blocks:
        BLOCKS_OVERRIDE = tuple(int(b) for b in args.blocks.split(","))
    if args.encode_L:
        ENCODE_LS = tuple(int(x) for x in args.encode_L.split(","))
    result = {}
    if args.only in (None, "copy"):
        result["copy"] = copy_sweep(args.reps)
    if args.only in (None, "decode"):
        result["decode"] = decode_sweep(args.reps)
    if args.only == "ragged":
        result["ragged"] = ragged_sweep(args.reps)
    if args.only == "small":
        result["small"] = small_sweep(args.reps)
    if args.only == "utf8":
        result["utf8"] = utf8_sweep(args.reps)
    if args.only == "varlen":
        result["varlen"] = varlen_sweep(args.reps)
    if args.only == "copydma":
        result["copydma"] = copydma_sweep(args.reps)
    if args.only == "multi":
        specs = []
        for part in args.specs.split(";"):
            name, _, kvs = part.partition(":")
            specs.append((name, [tuple(int(y) for y in x.split("=")) for x in kvs.split(",") if x]))
        result["multi"] = multi_sweep(args.reps, specs)
    if args.only == "vdec":
        global VDEC_CAP_PCTS
        VDEC_CAP_PCTS = (105, 125)
        result["vdec"] = vdec_sweep(args.reps)
    if args.only == "vknob":
        pre = [tuple(int(y) for y in x.split("=")) for x in args.pre.split(",") if x]
        result["vknob"] = vknob_sweep(args.reps, args.key, [int(x) for x in args.values.split(",")], pre)
    if args.only == "knob":
        pre = [tuple(int(y) for y in x.split("=")) for x in args.pre.split(",") if x]
        result["knob"] = knob_sweep(args.reps, args.key, [int(x) for x in args.values.split(",")], pre)
    if args.only == "align":
        result["align"] = align_sweep(args.reps)
    if args.only == "opsknob":  # every tile op under --key at --values (names v<value>)
        vals = tuple(int(x) for x in args.values.split(","))
        result["opsknob"] = align_sweep(args.reps, args.key, vals, tuple(f"v{v}" for v in vals))
    if args.only == "varlen_enc":
        result["varlen_enc"] = varlen_enc_sweep(args.reps)
    if args.only == "ablate":
        global ABLATE_L
        ABLATE_L = args.L
        result["ablate"] = ablate_sweep(args.reps)
    if args.only in (None, "encode"):
        result["encode"] = encode_sweep(args.reps)
    print(json.dumps(result, indent=1))


if __name__ == "__main__":
    main()
