"""SHA-256 of device-resident frame batches, chunk by chunk (parity evidence).

tests/golden/digests.json holds, per BASELINE config, the SHA-256 of every
2^20-packet chunk of the frames utils/packet.py produced for that config's
synthetic batch (tests/golden/make_golden.py).  This hashes the same chunks
of a batch framed on the GPU, so a full 16M-packet launch, or any rank's
slice of one, can be compared with the reference chunk by chunk.

Chunks move device -> host through a small ring of pinned slots and are hashed
by a thread pool (hashlib releases the GIL on large buffers), so the copy of
chunk k + 1 overlaps the hashing of chunk k.  Host-side only: no codec work.
"""
from __future__ import annotations

import hashlib
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Tuple


def chunk_sha256(frames, csum=None, chunk: int = 1 << 20, workers: int = 8
                 ) -> List[Tuple[str, Optional[str]]]:
    """[(sha256(frames rows of chunk k), sha256(csum of chunk k as LE u16) or None)]
    for k over the rows of ``frames`` (a 2-D uint8 device tensor) in ``chunk`` steps."""
    import torch
    n = frames.shape[0]
    nchunks = (n + chunk - 1) // chunk
    if nchunks == 0:
        return []
    slots = min(workers, nchunks)
    row = frames.shape[1]
    bufs = [torch.empty((min(chunk, n), row), dtype=torch.uint8, pin_memory=True) for _ in range(slots)]
    busy = [None] * slots

    def _hash(buf, m):
        return hashlib.sha256(memoryview(buf[:m].numpy()).cast("B")).hexdigest()

    out_frames = [None] * nchunks
    with ThreadPoolExecutor(slots) as ex:
        for k in range(nchunks):
            s = k % slots
            if busy[s] is not None:
                j, fut = busy[s]
                out_frames[j] = fut.result()
            m = min(chunk, n - k * chunk)
            bufs[s][:m].copy_(frames[k * chunk:k * chunk + m])
            busy[s] = (k, ex.submit(_hash, bufs[s], m))
        for item in busy:
            if item is not None:
                out_frames[item[0]] = item[1].result()
    del bufs
    # hand the pinned slots back to the OS: kept in torch's host cache, GBs of
    # pinned pages slowed later pinned copies in the same process (bench e2e leg)
    empty = getattr(torch._C, "_host_emptyCache", None)
    if empty is not None:
        empty()
    out_cs: List[Optional[str]] = [None] * nchunks
    if csum is not None:
        cs = csum.cpu().numpy().astype("<u2")
        for k in range(nchunks):
            out_cs[k] = hashlib.sha256(cs[k * chunk:(k + 1) * chunk].tobytes()).hexdigest()
    return list(zip(out_frames, out_cs))
