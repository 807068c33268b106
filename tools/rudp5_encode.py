"""rudp5 encode (5-B header + u16 checksum sideband) vs rudp7 (in-band), 1M
packets through pack_batch with preallocated outputs, rotating buffer sets.
usage: python tools/rudp5_encode.py"""
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

from rudp import batch  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 20
for L in (1472, 256, 64):
    res = {}
    for H, want in ((7, False), (7, True), (5, True)):
        nsets = max(1, min(8, -(-(1 << 30) // (n * (2 * L + H)))))
        sets = []
        for i in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004 + i, device=dev)
            out = torch.empty((n, L + H), dtype=torch.uint8, device=dev)
            cs = torch.empty(n, dtype=torch.uint16, device=dev) if want else None
            sets.append((tab, pay, out, cs))

        def run(i):
            tab, pay, out, cs = sets[i % nsets]
            batch.pack_batch(tab, pay, H, out=out, csum_out=cs, want_csum=want)
        for i in range(nsets):
            run(i)
        torch.cuda.synchronize()
        times = []
        for r in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(nsets):
                run(i)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b) / nsets)
        res[(H, want)] = statistics.median(times)
    print(f"L={L}: rudp7 {res[(7, False)]*1e3:.1f} us, rudp7+csum {res[(7, True)]*1e3:.1f} us, "
          f"rudp5+sideband {res[(5, True)]*1e3:.1f} us")
