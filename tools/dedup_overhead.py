"""Proxy dedup over 1M one-character datagrams: Python entry vs bare ABI call
vs the offset bounds check alone (microseconds per call)."""
import ctypes
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

from rudp import _native, batch  # noqa: E402
dev = torch.device('cuda', 0)
n = 1 << 20
tab, pay = batch.synth_batch(n, 1, 0x5EED0007, device=dev)
lens = torch.ones(n, dtype=torch.int32, device=dev)
enc = batch.pack_batch_varlen(tab, pay.view(-1), lens, 7)
lib = _native.lib()
def t(fn, k=30):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6
st = torch.cuda.current_stream().cuda_stream
dup = torch.empty(n, dtype=torch.uint8, device=dev)
print('python entry us', t(lambda: batch.detect_retransmissions(enc.frames, frame_off=enc.frame_off, window=500)))
print('abi only us', t(lambda: lib.rudp_dedup_window(enc.frames.data_ptr(), enc.frame_off.data_ptr(), 0, n, 500, dup.data_ptr(), 0, st)))
out = (ctypes.c_int64 * 3)()
print('bounds us', t(lambda: lib.rudp_frame_off_bounds(enc.frame_off.data_ptr(), n, out, 0, st)))
print('dups', int(dup.sum()))
