"""Where the one-character host varlen calls' time goes: the raw C entries
(pinned outputs) of the diagnostics build under host_min_chunks (knob 71) and
host_slots (knob 8) values, interleaved, beside plain pinned copies of the same
byte counts (the link's floor for the call's traffic).

usage: RUDP_LIB=reliable-udp_amd/rudp/librudp_tools.so python tools/host_chunks_ab.py [--reps 7]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("RUDP_LIB", str(REPO / "reliable-udp_amd" / "rudp" / "librudp_tools.so"))
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402


def pinned(k, dt):
    return torch.empty(k, dtype=dt, pin_memory=True).numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--chunks", default="1,2,4,8,16")
    ap.add_argument("--slots", default="3")
    ap.add_argument("--direct", default="1",
                    help="knob 73 values: 1 = the kernels store the per-frame outputs into the pinned arrays, "
                         "0 = slot + D2H copies")
    ap.add_argument("--zero-copy", default="0",
                    help="knob 75 values: 1 = one launch reading and writing the pinned arrays over PCIe "
                         "(then chunks / slots / direct do not apply), 0 = the slot pipeline")
    args = ap.parse_args()
    lib = _native.lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    m = 1 << 20
    rng = np.random.default_rng(1)
    seq, ack, flg = pinned(m, torch.uint16), pinned(m, torch.uint16), pinned(m, torch.uint8)
    seq[:] = np.arange(m, dtype=np.uint16)
    ack[:] = rng.integers(0, 1 << 16, m, dtype=np.uint16)
    flg[:] = 0x40
    pay = pinned(m, torch.uint8)
    pay[:] = rng.integers(0x20, 0x7F, m, dtype=np.uint8)
    lens = pinned(m, torch.int32)
    lens[:] = 1
    enc = batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True)
    fr, fo, cs = pinned(enc.frames.size, torch.uint8), pinned(m + 1, torch.int64), pinned(m, torch.uint16)
    fr[:], fo[:], cs[:] = enc.frames, enc.frame_off, enc.csum
    outs = [pinned(m, torch.uint16), pinned(m, torch.uint16), pinned(m, torch.uint8), pinned(m, torch.uint8),
            pinned(m, torch.uint16), pinned(m, torch.uint8)]
    st = np.zeros(1, np.uint32)
    fo_out, cs_out = pinned(m + 1, torch.int64), pinned(m, torch.uint16)
    fr_out = pinned(fr.size, torch.uint8)
    b = _native.RudpBatch(n=m, payload_len=1, reserved=0, seq=seq.ctypes.data, ack=ack.ctypes.data,
                          flags=flg.ctypes.data, payload=pay.ctypes.data, len=lens.ctypes.data, payload_off=None)

    def dec():
        _native.check(lib.rudp_decode_varlen_host(fr.ctypes.data, fr.size, fo.ctypes.data, 6, m, cs.ctypes.data,
                                                  *[a.ctypes.data for a in outs], st.ctypes.data, 5, 0))

    def encf():
        _native.check(lib.rudp_encode_varlen_host(ctypes.byref(b), m, fr_out.ctypes.data, fr_out.size,
                                                  fo_out.ctypes.data, cs_out.ctypes.data, 5, 0))

    # the link floor: the same bytes as plain pinned copies, one each way, not overlapped
    up = torch.from_numpy(pinned(16 << 20, torch.uint8))
    dn = torch.from_numpy(pinned(16 << 20, torch.uint8))
    dbuf = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")

    def copies(nu, nd):
        def f():
            dbuf[:nu].copy_(up[:nu], non_blocking=True)
            dn[:nd].copy_(dbuf[:nd], non_blocking=True)
            torch.cuda.synchronize()
        return f

    variants = [(c, s, d, 0) for d in map(int, args.direct.split(",")) for s in map(int, args.slots.split(","))
                for c in map(int, args.chunks.split(","))]
    if "1" in args.zero_copy.split(","):
        variants.append((4, 3, 1, 1))
    old_c, old_s, old_d, old_z = lib.rudpx_tune(71, 4), lib.rudpx_tune(8, 3), lib.rudpx_tune(73, 1), lib.rudpx_tune(75, 0)
    lib.rudpx_tune(71, old_c)
    lib.rudpx_tune(8, old_s)
    lib.rudpx_tune(73, old_d)
    lib.rudpx_tune(75, old_z)
    jobs = {"copy_dec_16MBup_9MBdown": copies(16 << 20, 9 << 20), "copy_enc_10MBup_16MBdown": copies(10 << 20, 16 << 20)}
    for c, s, d, z in variants:
        for name, fn in (("dec", dec), ("enc", encf)):
            def run(c=c, s=s, d=d, z=z, fn=fn):
                lib.rudpx_tune(71, c)
                lib.rudpx_tune(8, s)
                lib.rudpx_tune(73, d)
                lib.rudpx_tune(75, z)
                fn()
            jobs[f"{name}_zero_copy" if z else f"{name}_chunks{c}_slots{s}_direct{d}"] = run
    times = {k: [] for k in jobs}
    for f in jobs.values():
        f()
    for _ in range(args.reps):
        for k, f in jobs.items():
            t0 = time.perf_counter()
            f()
            times[k].append(time.perf_counter() - t0)
    lib.rudpx_tune(71, old_c)
    lib.rudpx_tune(8, old_s)
    lib.rudpx_tune(73, old_d)
    lib.rudpx_tune(75, old_z)
    out = {k: round(sorted(v)[len(v) // 2] * 1e3, 4) for k, v in times.items()}
    print(json.dumps({"ms_median": out, "reps": args.reps}, indent=1))


if __name__ == "__main__":
    main()
