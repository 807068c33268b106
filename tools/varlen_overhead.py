"""Where the time of the Python varlen entry points goes, 1M one-character
datagrams (the reference's traffic): whole calls, the bounds checks, the
bare ABI encode, and an empty stream sync.  Prints microseconds per call."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402
from rudp import batch  # noqa: E402
dev = torch.device('cuda', 0)
n = 1 << 20
tab, pay = batch.synth_batch(n, 1, 0x5EED0007, device=dev)
lens = torch.ones(n, dtype=torch.int32, device=dev)
flat = pay.view(-1)
def t(fn, k=50):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6
lens64 = lens.to(torch.int64)
print('pack_batch_varlen us', t(lambda: batch.pack_batch_varlen(tab, flat, lens, 7)))
print('stats block us', t(lambda: torch.stack([lens.to(torch.int64).min(), lens.to(torch.int64).max(), lens.to(torch.int64).sum()]).tolist()))
print('to int64 us', t(lambda: lens.to(torch.int64)))
res = batch.pack_batch_varlen(tab, flat, lens, 7)
print('unpack_batch_varlen us', t(lambda: batch.unpack_batch_varlen(res.frames, res.frame_off, 7)))
import ctypes
from rudp import _native
lib = _native.lib()
out = (ctypes.c_int64 * 5)()
st = torch.cuda.current_stream().cuda_stream
print('rudp_varlen_bounds us', t(lambda: lib.rudp_varlen_bounds(lens.data_ptr(), None, n, out, 0, st)))
print('rudp_frame_off_bounds us', t(lambda: lib.rudp_frame_off_bounds(res.frame_off.data_ptr(), n, out, 0, st)))
print('empty sync us', t(lambda: torch.cuda.current_stream().synchronize()))
print('encode_varlen (ABI only) us', t(lambda: lib.rudp_encode_varlen(ctypes.byref(_native.RudpBatch(
    n=n, payload_len=1, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(),
    payload=flat.data_ptr(), len=lens.data_ptr(), payload_off=None)), res.frames.data_ptr(), res.frame_off.data_ptr(),
    None, 7, 0, st)))
