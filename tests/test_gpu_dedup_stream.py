"""librudp's dedup stream (rudp_dedup_stream_*, ABI 6): the reference proxy's
retransmission count over a datagram stream (proxy.py:79-94; the 500-deep
history of proxy.py:17, :92-94; Packet.__eq__, utils/packet.py:83-86) with
the history kept on the device between batches.  Checked against a direct
restatement of the proxy's list scan with per-side counters."""
import ctypes

import numpy as np
import pytest

from rudp import _native

pytestmark = pytest.mark.gpu


def _proxy_counts(seq, sides, window):
    hist, flags, counts = [], [], [0, 0]
    for data, side in zip(seq, sides):
        key = data if data else bytes(5)  # Packet(b"") is the 40-bit zero header
        dup = key in hist[-window:] if window else False
        flags.append(int(dup))
        counts[side] += int(dup)
        hist.append(key)
    return flags, counts


@pytest.mark.parametrize("window", [1, 500, 4096])
def test_dedup_stream_matches_proxy_list_scan(cuda, window):
    import torch
    rng = np.random.default_rng(window)
    pool = [b"", bytes(5), b"\x00"] + [bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
                                       for _ in range(300)]
    seq = [pool[int(k)] for k in rng.integers(0, len(pool), 9000)]
    sides = [int(s) for s in rng.integers(0, 2, len(seq))]
    want_flags, want_counts = _proxy_counts(seq, sides, window)
    lib = _native.lib()
    s = torch.cuda.Stream(device=cuda)
    h = ctypes.c_void_p()
    _native.check(lib.rudp_dedup_stream_create(window, 1024, 64, 0, s.cuda_stream, ctypes.byref(h)))
    try:
        got = torch.empty(len(seq), dtype=torch.uint8, device=cuda)
        pos = 0
        while pos < len(seq):
            k = min(int(rng.integers(1, 1025)), len(seq) - pos)
            part = seq[pos:pos + k]
            fr = np.frombuffer(b"".join(part) + b"\x00", np.uint8)
            off = np.concatenate([[0], np.cumsum([len(p) for p in part])]).astype(np.uint64)
            side = np.array(sides[pos:pos + k], np.uint8)
            _native.check(lib.rudp_dedup_stream_push(h, fr.ctypes.data, off.ctypes.data, k, side.ctypes.data,
                                                     got.data_ptr() + pos))
            pos += k
        counts = (ctypes.c_uint64 * 2)()
        _native.check(lib.rudp_dedup_stream_counts(h, counts))
        assert [int(counts[0]), int(counts[1])] == want_counts
        assert got.cpu().numpy().tolist() == want_flags
    finally:
        lib.rudp_dedup_stream_destroy(h)


def test_dedup_stream_rejects_bad_batches(cuda):
    import torch
    lib = _native.lib()
    h = ctypes.c_void_p()
    _native.check(lib.rudp_dedup_stream_create(500, 8, 16, 0, torch.cuda.current_stream().cuda_stream,
                                               ctypes.byref(h)))
    try:
        fr = np.zeros(64, np.uint8)
        too_many = np.arange(10, dtype=np.uint64)
        assert lib.rudp_dedup_stream_push(h, fr.ctypes.data, too_many.ctypes.data, 9, None, None) == _native.EINVAL
        too_long = np.array([0, 17], np.uint64)
        assert lib.rudp_dedup_stream_push(h, fr.ctypes.data, too_long.ctypes.data, 1, None, None) == _native.EINVAL
        back = np.array([0, 5, 3], np.uint64)
        assert lib.rudp_dedup_stream_push(h, fr.ctypes.data, back.ctypes.data, 2, None, None) == _native.EINVAL
    finally:
        lib.rudp_dedup_stream_destroy(h)
    assert lib.rudp_dedup_stream_create(5000, 8, 16, 0, None, ctypes.byref(h)) == _native.EINVAL
