"""Host cost (us per call) of the ways the Python entries can allocate their
one output buffer, and of the whole sync-free varlen encode entry with and
without reuse=, for 1M one-character packets.

usage: python tools/alloc_probe.py
"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

from rudp import batch  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 20
size = 34 * n


def t(fn, k=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    us = (time.perf_counter() - t0) / k * 1e6
    torch.cuda.synchronize()
    return us


pay = torch.zeros((n,), dtype=torch.uint8, device=dev)
out = {
    "torch.empty(dtype, device=torch.device)": t(lambda: torch.empty((size,), dtype=torch.uint8, device=dev)),
    "torch.empty(dtype, device=int)": t(lambda: torch.empty((size,), dtype=torch.uint8, device=0)),
    "torch.empty(size int, device=int)": t(lambda: torch.empty(size, dtype=torch.uint8, device=0)),
    "payload.new_empty": t(lambda: pay.new_empty((size,))),
    "payload.new_empty(int)": t(lambda: pay.new_empty(size)),
}
tab, p1 = batch.synth_batch(n, 1, 0x5EED0004, device=dev)
lens = torch.ones(n, dtype=torch.int32, device=dev)
flat = p1.view(-1)
res = batch.pack_batch_varlen(tab, flat, lens, "rudp5", want_csum=True)
out["pack_batch_varlen host us (no reuse)"] = t(lambda: batch.pack_batch_varlen(tab, flat, lens, "rudp5", want_csum=True, check=False), 200)
out["pack_batch_varlen host us (reuse)"] = t(lambda: batch.pack_batch_varlen(tab, flat, lens, "rudp5", want_csum=True, check=False, reuse=res), 200)
print(json.dumps(out, indent=1))
