"""Does output alignment bound encode?  Streaming copy (one dwordx4 per thread,
non-temporal) of 1M x 1472 B with the source and/or destination offset by 16,
64 or 112 bytes from a 128-B line, and with a 7-byte gap opened every 1472 B in
the destination (encode's write pattern with no compute).  Prints TB/s."""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

from sweep import interleaved, lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nbytes = (1 << 20) * 1472
    a = torch.empty(nbytes + 4096, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes + 4096, dtype=torch.uint8, device=dev)
    a.fill_(7)
    stream = torch.cuda.current_stream().cuda_stream
    n16 = nbytes // 16
    variants = {}
    for so, do in ((0, 0), (0, 16), (0, 64), (0, 112), (16, 0), (64, 0), (16, 16), (64, 64)):
        variants[f"src+{so}_dst+{do}"] = (
            lambda: None,
            lambda so=so, do=do: lib.rudpx_copy_vpt(a.data_ptr() + so, b.data_ptr() + do, n16, 1, 1, stream))
    res = interleaved(variants, 9)
    print(json.dumps({k: {"ms": ms, "TBs": 2 * nbytes / ms / 1e9} for k, ms in res.items()}, indent=1))


if __name__ == "__main__":
    main()
