"""Call temporaries (scan sums, tile records, dedup hashes, offset-check
partials) kept per (device, stream) by librudp, not per host thread.

The reference proxy parses datagrams on ThreadPoolExecutor workers
(proxy.py:127, :154); a caller with short-lived threads, or one that makes a
stream per call, must not grow the library's device footprint.  Measured
through the diagnostics build's rudpx_scratch_stats (its pool's
hipMemPoolAttrUsedMemCurrent and the number of scratch sets).
"""
import ctypes
import threading

import numpy as np
import pytest

from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu


class _RawStreams:
    """Distinct HIP streams (hipStreamCreate), as torch ExternalStreams: torch.cuda.Stream()
    hands out its pool's 32 streams round robin, so it cannot make 65+ distinct ones."""

    def __init__(self, k, cuda):
        import torch
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        self.raw = []
        for _ in range(k):
            h = ctypes.c_void_p()
            assert self.hip.hipStreamCreate(ctypes.byref(h)) == 0
            self.raw.append(h)
        self.streams = [torch.cuda.ExternalStream(h.value, device=cuda) for h in self.raw]

    def close(self):
        import torch
        torch.cuda.synchronize()
        for h in self.raw:
            self.hip.hipStreamDestroy(h)


def _stats(lib):
    out = (ctypes.c_uint64 * 2)()
    _native.check(lib.rudpx_scratch_stats(0, out))
    return int(out[0]), int(out[1])


def _work(cuda, n, seed, own_stream, errors):
    """One request's worth: varlen encode (scan + tiles), decode, dedup; checked."""
    import torch
    try:
        s = torch.cuda.Stream(device=cuda) if own_stream else torch.cuda.current_stream(cuda)
        rng = np.random.default_rng(seed)
        lens = rng.integers(0, 300 if seed % 2 else 3, n).astype(np.int32)
        pay = rng.integers(0, 128, int(lens.sum()), dtype=np.uint8)
        seq, ack, flags, _ = synth.synth(seed, 0, n, 0)
        with torch.cuda.stream(s):
            tab = tuple(torch.from_numpy(a).to(cuda) for a in (seq, ack, flags))
            res = batch.pack_batch_varlen(tab, torch.from_numpy(pay).to(cuda),
                                          torch.from_numpy(lens).to(cuda), "rudp7")
            dec = batch.unpack_batch_varlen(res.frames, res.frame_off, "rudp7", utf8=True)
            dup = batch.detect_retransmissions(res.frames, frame_off=res.frame_off, window=500)
            s.synchronize()
        pays = [bytes(pay[o:o + k]) for o, k in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)]
        want, off, _ = codec_np.encode_varlen(seq, ack, flags, pays, 7)
        assert np.array_equal(res.frames.cpu().numpy(), want)
        assert bool((dec.ok == 1).all()) and bool((dec.valid == 1).all())
        assert int(dup.sum().item()) >= 0
    except BaseException as e:  # noqa: BLE001 -- reported by the main thread
        errors.append(e)


def _wave(cuda, k, n, base_seed):
    errors = []
    threads = [threading.Thread(target=_work, args=(cuda, n, base_seed + i, i % 4 == 0, errors))
               for i in range(k)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]


def test_short_lived_threads_keep_footprint_bounded(cuda):
    """Two waves of 64 short-lived threads (a quarter on streams of their own):
    every result correct, and the second wave adds no memory and no sets."""
    import torch
    lib = _native.tools_lib()
    _wave(cuda, 64, 3000, 1000)
    torch.cuda.synchronize()
    used1, sets1 = _stats(lib)
    _wave(cuda, 64, 3000, 2000)
    torch.cuda.synchronize()
    used2, sets2 = _stats(lib)
    assert 0 < sets1 <= 64 and sets2 <= 64
    # new streams may map onto released handles or new sets, never past the cap,
    # and the pool does not grow by a thread's worth per thread
    assert used2 <= used1 + 16 * (1 << 20), (used1, used2)


def test_stream_per_call_is_capped(cuda):
    """A caller that makes a fresh stream per call (80 live streams at once):
    at most 64 scratch sets, results still exact (an evicted set is reused
    only after the device is idle)."""
    import torch
    lib = _native.tools_lib()
    n = 2000
    seq, ack, flags, _ = synth.synth(5, 0, n, 0)
    lens = np.full(n, 40, np.int32)
    pay = np.random.default_rng(5).integers(0, 256, int(lens.sum()), dtype=np.uint8)
    want, off, _ = codec_np.encode_varlen(seq, ack, flags, [bytes(pay[40 * i:40 * i + 40]) for i in range(n)], 7)
    tab = tuple(torch.from_numpy(a).to(cuda) for a in (seq, ack, flags))
    d_pay, d_len = torch.from_numpy(pay).to(cuda), torch.from_numpy(lens).to(cuda)
    raw = _RawStreams(80, cuda)
    outs = []
    try:
        for s in raw.streams:
            s.wait_stream(torch.cuda.current_stream(cuda))
            with torch.cuda.stream(s):
                outs.append(batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False))
        torch.cuda.synchronize()
        for r in outs:
            r.check()
            assert np.array_equal(r.frames.cpu().numpy(), want)
        assert _stats(lib)[1] <= 64
    finally:
        raw.close()


def test_scratch_under_graph_capture(cuda):
    """A varlen encode captured into a HIP graph allocates its temporaries inside
    the capture; replays give the same frames, and eager calls on the capture
    stream afterwards still do (no pointer the graph owns is cached)."""
    import torch
    n = 5000
    rng = np.random.default_rng(77)
    lens = rng.integers(0, 200, n).astype(np.int32)
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(77, 0, n, 0)
    pays = [bytes(pay[o:o + k]) for o, k in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)]
    want, _, _ = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    tab = tuple(torch.from_numpy(a).to(cuda) for a in (seq, ack, flags))
    d_pay, d_len = torch.from_numpy(pay).to(cuda), torch.from_numpy(lens).to(cuda)
    s = torch.cuda.Stream(device=cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        warm = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        cap = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(cap.frames.cpu().numpy(), want)
    with torch.cuda.stream(s):
        again = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False)
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(again.frames.cpu().numpy(), want)
    assert np.array_equal(warm.frames.cpu().numpy(), want)


def test_eviction_while_another_thread_captures(cuda):
    """with every scratch set taken (64 streams), a call on a new
    stream must neither synchronize the device while another thread holds a
    graph capture open (torch.cuda.graph's default global mode refuses that,
    or breaks the capture) nor reuse a set whose work may still run.  Sets are
    taken over only when their last call's end event has fired, else the call
    allocates its temporaries in stream order.  Under another thread's
    global-mode capture the HIP runtime refuses those queries and allocations
    (hipErrorStreamCaptureUnsupported): such a call fails cleanly with that
    error, the capture stays valid and replays exactly, and once the capture
    has ended every call succeeds with exact results."""
    import torch
    lib = _native.tools_lib()  # the batch API runs the diagnostics build: its sets are the ones counted
    n = 3000
    seq, ack, flags, _ = synth.synth(9, 0, n, 0)
    lens = np.full(n, 24, np.int32)
    pay = np.random.default_rng(9).integers(0, 256, int(lens.sum()), dtype=np.uint8)
    want, _, _ = codec_np.encode_varlen(seq, ack, flags, [bytes(pay[24 * i:24 * i + 24]) for i in range(n)], 7)
    tab = tuple(torch.from_numpy(a).to(cuda) for a in (seq, ack, flags))
    d_pay, d_len = torch.from_numpy(pay).to(cuda), torch.from_numpy(lens).to(cuda)
    # fill the device's sets (earlier tests may have made some); a second round on
    # them after the device is full records their end events
    raw = _RawStreams(80, cuda)
    streams, late = raw.streams[:72], raw.streams[72:]
    warm = []
    for rnd in range(2):
        for k, s in enumerate(streams):
            s.wait_stream(torch.cuda.current_stream(cuda))
            with torch.cuda.stream(s):
                r = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False,
                                            reuse=warm[k] if rnd else None)
                if not rnd:
                    warm.append(r)
    torch.cuda.synchronize()
    assert _stats(lib)[1] == 64
    for r in warm:
        r.check()
        assert np.array_equal(r.frames.cpu().numpy(), want)
    cap_stream = torch.cuda.Stream(device=cuda)
    cap_stream.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(cap_stream):
        cap_warm = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    inside, done, errors, cap = threading.Event(), threading.Event(), [], {}

    def capture():
        try:
            with torch.cuda.graph(g, stream=cap_stream):
                cap["r"] = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False, reuse=cap_warm)
                inside.set()
                done.wait(60)
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
            inside.set()

    t = threading.Thread(target=capture)
    t.start()
    inside.wait(60)
    # new streams while the capture is open: each needs a set (the eviction path)
    outs, refused = [], 0
    try:
        for k, s in enumerate(late):
            with torch.cuda.stream(s):
                try:
                    outs.append(batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False, reuse=warm[k]))
                except _native.RudpError as e:
                    assert "capturing" in str(e) or "capture" in str(e), e
                    refused += 1
    finally:
        done.set()
        t.join()
    if errors:
        raise errors[0]
    torch.cuda.synchronize()
    for r in outs:
        r.check()
        assert np.array_equal(r.frames.cpu().numpy(), want)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(cap["r"].frames.cpu().numpy(), want)
    # after the capture: every new stream's call goes through
    for k, s in enumerate(late):
        with torch.cuda.stream(s):
            r = batch.pack_batch_varlen(tab, d_pay, d_len, "rudp7", check=False, reuse=warm[k])
        torch.cuda.synchronize()
        r.check()
        assert np.array_equal(r.frames.cpu().numpy(), want)
    assert _stats(lib)[1] <= 64
    raw.close()
