"""UTF-8 bench-leg timing check: the bench's own buffers and time_loop, tile
kernel (rudpx_tune 31 = 1) against the vector kernel (0), twice each.

usage: python tools/utf8_diag.py
"""
import ctypes
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch
from rudp import batch, _native
import bench
lib = _native.tools_lib(); lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
dev = torch.device("cuda", 0)
w = bench.Workload(torch, batch, 1 << 20, 1472, "rudp7", 0, bench.SEEDS.get(1472, 0x5EED0004), dev)
for i in range(3): w.encode(batch, i)
fr = w.sets[0][2]
for tile in (1, 0, 1, 0):
    lib.rudpx_tune(31, tile)
    ms = bench.time_loop(torch, lambda i: batch.validate_utf8(fr, "rudp7"), 25, 3) / 25
    print("bench-style tile", tile, round(ms, 4), "valid", int(batch.validate_utf8(fr, "rudp7").sum()))
tab, pay = batch.synth_batch(1 << 20, 1472, 0x5EED0009, ascii=True, device=dev)
fr2 = batch.pack_batch(tab, pay, 7)[0]
for tile in (1, 0):
    lib.rudpx_tune(31, tile)
    ms = bench.time_loop(torch, lambda i: batch.validate_utf8(fr2, 7), 25, 3) / 25
    print("sweep-data tile", tile, round(ms, 4))
print(fr.shape, fr.stride(), fr.data_ptr() % 256, fr[0, :12].tolist())
