"""rudp5 (5-B header + u16 sideband) vs rudp7 verify-only decode through the raw
ABI, 1M packets, rotating buffer sets.  usage: python tools/rudp5_decode.py"""
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402

lib = _native.lib()
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream().cuda_stream
n = 1 << 20
for L in (1472, 256, 64):
    res = {}
    for H in (7, 5):
        nsets = max(1, min(8, -(-(1 << 30) // (n * (L + H)))))
        sets = []
        for i in range(nsets):
            tab, pay = batch.synth_batch(n, L, 0x5EED0004 + i, device=dev)
            fr, cs = batch.pack_batch(tab, pay, H, want_csum=True)
            sets.append((fr, cs))
        o16 = torch.empty(n, dtype=torch.uint16, device=dev)
        o8 = torch.empty(n, dtype=torch.uint8, device=dev)
        okb = torch.empty(n, dtype=torch.uint8, device=dev)

        def run(i):
            fr, cs = sets[i % nsets]
            _native.check(lib.rudp_decode(fr.data_ptr(), None, L + H, n, cs.data_ptr() if H == 5 else None,
                                          o16.data_ptr(), o16.data_ptr(), o8.data_ptr(), okb.data_ptr(),
                                          None, None, H, 0, stream))
        for i in range(nsets):
            run(i)
        torch.cuda.synchronize()
        assert bool((okb == 1).all()), (L, H)
        times = []
        for r in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(nsets):
                run(i)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b) / nsets)
        res[H] = statistics.median(times)
    print(f"L={L}: rudp7 {res[7]*1e3:.1f} us, rudp5+sideband {res[5]*1e3:.1f} us")
