"""Probe: the bench's C2 leg (1M x 1024 B encode through the Python entry, after the
headline workload) beside the raw C-ABI launch on the same buffers, on one box."""
import ctypes
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rudp import _native, batch  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
out = {}
w = bench.Workload(torch, batch, 1 << 20, 1472, "rudp7", 0, bench.SEEDS[1472], dev)
out["headline_ms"] = bench.time_loop(torch, lambda i: w.encode(batch, i), 50, 5) / 50
if "--digest" in sys.argv:  # as bench.main does: the headline frames hashed against the C4 digests
    out["digest"] = bench.verify_digests(w, "C4", 0, 1 << 20)
del w
torch.cuda.empty_cache()
for rep in range(3):
    w = bench.Workload(torch, batch, 1 << 20, 1024, "rudp7", 0, bench.SEEDS[1024], dev)
    py = bench.time_loop(torch, lambda i: w.encode(batch, i), 25, 3) / 25
    tab, pay, fr = w.sets[0]
    b = _native.RudpBatch(n=1 << 20, payload_len=1024, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                          flags=tab.flags.data_ptr(), payload=pay.data_ptr(), len=None, payload_off=None)
    lib = _native.lib()
    s = torch.cuda.current_stream().cuda_stream
    raw = bench.time_loop(torch, lambda i: lib.rudp_encode(ctypes.byref(b), fr.data_ptr(), None, 7, 0, s), 25, 3) / 25
    # host time of one Python-entry call
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        batch.pack_batch(tab, pay, 7, out=fr, want_csum=False)
    host = (time.perf_counter() - t0) / 200
    torch.cuda.synchronize()
    out[f"rep{rep}"] = {"python_entry_ms": py, "raw_abi_ms": raw, "host_submit_ms_per_call": host * 1e3}
    del w, tab, pay, fr
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
