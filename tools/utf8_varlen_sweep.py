"""Packed-frame UTF-8 validation: LDS-tile kernel (rudpx_tune 41 = 1) vs
per-frame vector kernel (0), 1M ASCII frames of 1472 B and of uniform
0-2944 B, rotating buffer sets.  usage: python tools/utf8_varlen_sweep.py"""
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
dev = torch.device("cuda", 0)
n = 1 << 20
out = {}
for name in ("L1472", "U0-2944"):
    tab, pay = batch.synth_batch(n, 2944, 0x5EED0009, device=dev)
    lens = (torch.full((n,), 1472, dtype=torch.int32, device=dev) if name == "L1472"
            else torch.randint(0, 2945, (n,), dtype=torch.int32, device=dev))
    flat = pay.view(-1)[: int(lens.sum().item())]
    r = batch.pack_batch_varlen(tab, flat, lens, 7)
    fr, off = r.frames, r.frame_off
    res = {}
    for vt in ((1, 110), (0, 110), (1, 130), (1, 150), (1, 110), (0, 110), (1, 130), (1, 150)):
        lib.rudpx_tune(41, vt[0])
        lib.rudpx_tune(42, vt[1])
        v = batch.validate_utf8(fr, 7, frame_off=off)
        assert bool((v == 1).all())
        times = []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                batch.validate_utf8(fr, 7, frame_off=off)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b) / 3)
        res.setdefault(vt, []).append(statistics.median(times))
    lib.rudpx_tune(41, 1)
    lib.rudpx_tune(42, 110)
    out[name] = {f"tile{c}_ms" if t else "vector_ms": min(v) for (t, c), v in res.items()}
    del tab, pay, lens, flat, r, fr, off
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
