"""Host-side cost of the Python decode entry's output allocations (us per call).

usage: python tools/py_overhead.py
"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 20


def t(fn, k=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) / k * 1e6


def five():
    return [torch.empty((n,), dtype=d, device=dev) for d in
            (torch.uint16, torch.uint16, torch.uint8, torch.uint8, torch.uint16)]


def one_split():
    s2 = (2 * n + 255) & ~255
    s1 = (n + 255) & ~255
    buf = torch.empty((3 * s2 + 2 * s1,), dtype=torch.uint8, device=dev)
    a, b, c, d, e = torch.split(buf, (s2, s2, s2, s1, s1))
    return a[:2 * n].view(torch.uint16), b[:2 * n].view(torch.uint16), d[:n], e[:n], c[:2 * n].view(torch.uint16)


def one_empty():
    return torch.empty((8 * n,), dtype=torch.uint8, device=dev)


off = torch.arange(n + 1, device=dev, dtype=torch.int64) * 8
print("five empties us", t(five))
print("one empty + split/views us", t(one_split))
print("one empty us", t(one_empty))
print("start/end (minimum, add) us", t(lambda: torch.minimum(off[:-1] + 5, off[1:])))
print("start/end (clamp) us", t(lambda: (off[:-1] + 5).clamp_(max=off[1:])))
