"""Variable-length batches and strict UTF-8 validation on the GPU.

Pinned by tests/golden/varlen.npz: mixed-width UTF-8 strings framed one per
packet by the reference utils/packet.py, and the reference get_payload()
outcome (value or UnicodeDecodeError) on hand-picked and random byte bodies.
"""
import numpy as np
import pytest

from conftest import split_by_lengths
from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).to(cuda)


def host(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("layout", [5, 7])
def test_varlen_encode_matches_reference(cuda, golden_varlen, layout):
    g = golden_varlen
    res = batch.pack_batch_varlen((dev(g["seq"], cuda), dev(g["ack"], cuda), dev(g["flags"], cuda)),
                                  dev(g["payload"], cuda), dev(g["lengths"], cuda), layout,
                                  want_csum=True)
    assert np.array_equal(host(res.frames), g[f"frames{layout}"])
    assert np.array_equal(host(res.csum), g["csum"])
    off = host(res.frame_off)
    assert off[0] == 0 and np.array_equal(np.diff(off), g["lengths"] + layout)
    d = batch.unpack_batch_varlen(res.frames, res.frame_off, layout,
                                  csum=res.csum if layout == 5 else None)
    assert (host(d.ok) == 1).all()
    assert np.array_equal(host(d.seq), g["seq"]) and np.array_equal(host(d.ack), g["ack"])
    assert np.array_equal(host(d.flags), g["flags"]) and np.array_equal(host(d.csum), g["csum"])
    start, end = host(d.payload[0]), host(d.payload[1])
    fr = g[f"frames{layout}"]
    pays, _ = split_by_lengths(g["payload"], g["lengths"])
    assert all(bytes(fr[start[i]:end[i]]) == pays[i] for i in range(len(pays)))


def test_varlen_gather_offsets(cuda):
    rng = np.random.default_rng(3)
    n = 5000
    lens = rng.integers(0, 40, n).astype(np.int32)
    buf = rng.integers(0, 256, int(lens.sum()) + 100, dtype=np.uint8)
    # payloads taken from arbitrary places of the buffer (not packed, not in order)
    starts = rng.integers(0, len(buf) - 40, n).astype(np.int64)
    seq, ack, flags, _ = synth.synth(9, 0, n, 0)
    res = batch.pack_batch_varlen((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(buf, cuda),
                                  dev(lens, cuda), 7, payload_off=dev(starts, cuda))
    pays = [bytes(buf[s:s + l]) for s, l in zip(starts, lens)]
    want, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    assert np.array_equal(host(res.frames), want) and np.array_equal(host(res.frame_off), off)


def test_varlen_reference_traffic_roundtrip(cuda):
    """1M one-character datagrams (utils/reliableUDP.py:11): encode -> decode on device."""
    import torch
    n = 1 << 20
    rng = np.random.default_rng(11)
    chars = np.array(list("test\n"), dtype="<U1")
    text = "".join(rng.choice(chars, n))
    pay = np.frombuffer(text.encode(), np.uint8)
    lens = np.ones(n, np.int32)
    seq, ack, flags, _ = synth.synth(0x5EED0001, 0, n, 0)
    res = batch.pack_batch_varlen((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda),
                                  dev(lens, cuda), 5, want_csum=True)
    assert res.frames.numel() == 6 * n
    # spot-check against the oracle on a prefix, then a full device round trip
    pref = 4096
    want, _, cs = codec_np.encode_varlen(seq[:pref], ack[:pref], flags[:pref],
                                         [bytes([b]) for b in pay[:pref]], 5)
    assert np.array_equal(host(res.frames[:6 * pref]), want)
    d = batch.unpack_batch_varlen(res.frames, res.frame_off, 5, csum=res.csum)
    assert bool((d.ok == 1).all())
    assert torch.equal(d.flags, dev(flags, cuda))
    assert torch.equal(res.frames.view(n, 6)[:, 5], dev(pay, cuda))
    assert bool((batch.validate_utf8(res.frames, 5, frame_off=res.frame_off) == 1).all())


def test_varlen_short_and_empty_frames(cuda):
    # hand-built frames of every length 0..9, decoded with offsets
    frames = [bytes(range(1, 1 + k)) for k in range(10)]
    flat = np.frombuffer(b"".join(frames), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    for layout in (5, 7):
        d = batch.unpack_batch_varlen(dev(flat, cuda), dev(off, cuda), layout)
        want = codec_np.decode_varlen(flat, off, layout)
        for got, exp in zip((d.seq, d.ack, d.flags, d.ok, d.csum), want):
            assert np.array_equal(host(got), exp), layout


def test_utf8_matches_reference_get_payload(cuda, golden_varlen):
    g = golden_varlen
    bodies, _ = split_by_lengths(g["utf8_bodies"], g["utf8_lengths"])
    frames = [b"\x00\x01\x00\x02\x40" + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    v = batch.validate_utf8(dev(flat, cuda), 5, frame_off=dev(off, cuda))
    assert np.array_equal(host(v), g["utf8_valid"])


def test_utf8_fixed_length(cuda, golden_small):
    for L in (1, 16, 64, 1472):
        fr = golden_small[f"L{L}_full_frames7"]
        off = np.arange(fr.shape[0] + 1, dtype=np.int64) * fr.shape[1]
        want = codec_np.utf8_valid(fr.reshape(-1), off, 7)
        assert np.array_equal(host(batch.validate_utf8(dev(fr, cuda), 7)), want)
        ascii_fr = golden_small[f"L{L}_frames7"]
        assert (host(batch.validate_utf8(dev(ascii_fr, cuda), 7)) == 1).all()


def test_varlen_rejects_out_of_bounds(cuda):
    z16 = dev(np.zeros(2, np.uint16), cuda)
    z8 = dev(np.zeros(2, np.uint8), cuda)
    with pytest.raises(ValueError, match="sum"):
        batch.pack_batch_varlen((z16, z16, z8), dev(np.zeros(3, np.uint8), cuda),
                                dev(np.array([2, 2], np.int32), cuda))
    with pytest.raises(ValueError, match="inside"):
        batch.unpack_batch_varlen(dev(np.zeros(8, np.uint8), cuda),
                                  dev(np.array([0, 5, 12], np.int64), cuda))


def _near_utf8(rng, n):
    """Mostly-valid UTF-8 strings with a few random byte edits (hits every DFA edge)."""
    chars = [chr(c) for c in (0x41, 0x7F, 0x80, 0x7FF, 0x800, 0xD7FF, 0xE000, 0xFFFD, 0xFFFF,
                               0x10000, 0x1F600, 0x10FFFF, 0xE9, 0x4E2D)]
    out = []
    for _ in range(n):
        s = "".join(chars[i] for i in rng.integers(0, len(chars), rng.integers(0, 12))).encode()
        b = bytearray(s)
        for _ in range(rng.integers(0, 3)):
            if b and rng.random() < 0.7:
                b[rng.integers(0, len(b))] = int(rng.integers(0, 256))
            elif rng.random() < 0.5 and b:
                del b[rng.integers(0, len(b))]
            else:
                b.insert(int(rng.integers(0, len(b) + 1)), int(rng.choice([0x80, 0xBF, 0xC0, 0xE0, 0xED, 0xF0, 0xF4, 0xF5])))
        out.append(bytes(b))
    return out


def test_utf8_random_vs_python_decoder(cuda):
    rng = np.random.default_rng(1234)
    bodies = _near_utf8(rng, 20000)
    frames = [b"\x12\x34\x00\x00\x80" + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    want = codec_np.utf8_valid(flat, off, 5)
    assert 0.2 < want.mean() < 0.9  # both outcomes well represented
    got = host(batch.validate_utf8(dev(flat, cuda), 5, frame_off=dev(off, cuda)))
    assert np.array_equal(got, want)


def _dedup_form(table):
    """Context: the dedup window pass by LDS hash table (1) or by window scan (0)."""
    import contextlib
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int

    @contextlib.contextmanager
    def ctx():
        old = lib.rudpx_tune(32, table)
        try:
            yield
        finally:
            lib.rudpx_tune(32, old)
    return ctx()


@pytest.mark.parametrize("table", [1, 0])
def test_dedup_matches_reference_proxy(cuda, golden_dedup, table):
    g = golden_dedup
    off = np.concatenate([[0], np.cumsum(g["lengths"])]).astype(np.int64)
    with _dedup_form(table):
        dup = batch.detect_retransmissions(dev(g["frames"], cuda), frame_off=dev(off, cuda), window=500)
    assert np.array_equal(host(dup), g["dup"])


@pytest.mark.parametrize("table", [1, 0])
@pytest.mark.parametrize("window", [1, 7, 500, 4096])
def test_dedup_fixed_length_vs_oracle(cuda, window, table):
    from oracle.bitstring_packet import proxy_retransmitted
    rng = np.random.default_rng(window)
    base = rng.integers(0, 256, (300, 40), dtype=np.uint8)
    idx = rng.integers(0, 300, 2500)
    fr = np.ascontiguousarray(base[idx])
    want = proxy_retransmitted([r.tobytes() for r in fr], window) if window < 4096 else None
    with _dedup_form(table):
        got = host(batch.detect_retransmissions(dev(fr, cuda), window=window))
    last, ref = {}, []  # last occurrence of each frame: dup iff it lies inside the window
    for i, r in enumerate(fr):
        k = r.tobytes()
        ref.append(int(k in last and last[k] >= i - window))
        last[k] = i
    if want is None:
        want = ref
    assert list(want) == ref
    assert got.tolist() == list(want)


def test_utf8_misaligned_buffer_uses_fallback(cuda):
    import torch
    rng = np.random.default_rng(77)
    bodies = _near_utf8(rng, 3000)
    frames = [b"\x12\x34\x00\x00\x80" + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    raw = torch.zeros(len(flat) + 16, dtype=torch.uint8, device=cuda)
    view = raw[3:3 + len(flat)]
    view.copy_(dev(flat, cuda))
    got = host(batch.validate_utf8(view, 5, frame_off=dev(off, cuda)))
    assert np.array_equal(got, codec_np.utf8_valid(flat, off, 5))


def test_socket_ring_to_gpu_decode(cuda):
    """Datagrams from a UDP socket (recvmmsg into a pinned ring) decoded on the GPU."""
    import socket
    import threading

    from rudp import netio
    n = 30000
    rng = np.random.default_rng(21)
    seq, ack, flags, _ = synth.synth(21, 0, n, 0)
    pays = [bytes([int(c)]) for c in rng.integers(32, 127, n)]  # one character each (reliableUDP.py:11)
    fr, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 25)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    t = threading.Thread(target=lambda: netio.send_batch(tx, fr, off, "127.0.0.1", rx.getsockname()[1]))
    t.start()
    recv = netio.BatchReceiver(rx, max_msgs=n, slot_bytes=64)
    seen = []
    while len(seen) < n:
        k = recv.recv(timeout_ms=2000)
        assert k > 0
        dec, _, _ = recv.decode("rudp7", cuda)
        seen += list(zip(host(dec.seq), host(dec.ok)))
    t.join()
    assert [s for s, _ in seen] == seq.tolist()
    assert all(o == 1 for _, o in seen)
    rx.close()
    tx.close()


def _varlen_frames(rng, n, lo, hi, layout):
    """Frames of payload length in [lo, hi], some short / corrupted, after a ragged prefix."""
    lens = rng.integers(lo, hi + 1, n)
    pays = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
    seq, ack, flags, _ = synth.synth(int(rng.integers(1 << 30)), 0, n, 0)
    frames, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
    parts = [frames[off[i]:off[i + 1]].tobytes() for i in range(n)]
    for i in rng.choice(n, n // 20, replace=False):   # short frames, header cut
        parts[i] = parts[i][: int(rng.integers(0, layout))]
    for i in rng.choice(n, n // 20, replace=False):   # one flipped byte
        if parts[i]:
            b = bytearray(parts[i])
            b[int(rng.integers(len(b)))] ^= 1 << int(rng.integers(8))
            parts[i] = bytes(b)
    prefix = int(rng.integers(0, 16))
    buf = bytes(prefix) + b"".join(parts)
    off = np.cumsum([prefix] + [len(p) for p in parts]).astype(np.int64)
    return np.frombuffer(buf, np.uint8), off, cs


@pytest.mark.parametrize("lo,hi", [(0, 9), (0, 1500), (1400, 1472), (3000, 9000)])
@pytest.mark.parametrize("layout", [5, 7])
def test_varlen_decode_kernels_vs_oracle(cuda, lo, hi, layout):
    """LDS-tile and vector varlen decode (any lanes-per-frame hint; tiles past
    their budget take the per-frame path) == byte kernel == oracle."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(lo * 7 + hi + layout)
    n = 1500 if hi < 2000 else 300
    buf, off, cs = _varlen_frames(rng, n, lo, hi, layout)
    csum_in = cs if layout == 5 else None
    want = codec_np.decode_varlen(buf, off, layout, csum_in)
    d_buf, d_off = dev(buf, cuda), dev(off, cuda)
    d_cs = dev(cs, cuda) if layout == 5 else None
    outs = [torch.empty(n, dtype=dt, device=cuda)
            for dt in (torch.uint16, torch.uint16, torch.uint8, torch.uint8, torch.uint16)]
    runs = [("python", None, 1, 1)] + [("abi", h, v, t) for v in (1, 0) for h in (0, 8, 64, 263, 519, 1031, 1472, 65535)
                                         for t in ((2, 0) if v else (1,))]
    for kind, hint, vec, tile in runs:
        lib.rudpx_tune(14, vec)
        lib.rudpx_tune(33, tile)
        try:
            if kind == "python":
                d = batch.unpack_batch_varlen(d_buf, d_off, layout, csum=d_cs)
                got = [host(x) for x in (d.seq, d.ack, d.flags, d.ok, d.csum)]
            else:
                for o in outs:
                    o.fill_(0xAB)
                _native.check(lib.rudp_decode(
                    d_buf.data_ptr(), d_off.data_ptr(), hint, n,
                    d_cs.data_ptr() if d_cs is not None else None,
                    *[o.data_ptr() for o in outs], None, layout, 0,
                    torch.cuda.current_stream().cuda_stream))
                got = [host(o) for o in outs]
        finally:
            lib.rudpx_tune(14, 1)
            lib.rudpx_tune(33, 1)
        for name, g, w in zip(("seq", "ack", "flags", "ok", "csum"), got, want):
            assert np.array_equal(g, w), (lo, hi, layout, kind, hint, vec, tile, name)
    assert (want[3] == 2).any() and (want[3] == 0).any() and (want[3] == 1).any()


@pytest.mark.parametrize("lo,hi", [(0, 3), (0, 100), (20, 40), (1400, 1472), (5000, 20000)])
@pytest.mark.parametrize("layout", [5, 7])
def test_varlen_encode_kernels_vs_oracle(cuda, lo, hi, layout):
    """Vector varlen encode (any lanes-per-packet hint, packed or gathered
    payloads) == byte kernel == oracle, frames and offsets bit for bit."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(lo + 3 * hi + layout)
    n = 2000 if hi < 2000 else 120
    lens = rng.integers(lo, hi + 1, n).astype(np.int32)
    seq, ack, flags, _ = synth.synth(int(rng.integers(1 << 30)), 0, n, 0)
    packed = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    pays, _ = split_by_lengths(packed, lens)
    want_fr, want_off, want_cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
    # the same payloads scattered through a bigger buffer at arbitrary offsets
    gaps = rng.integers(0, 40, n)
    starts = (np.cumsum(gaps + lens) - lens).astype(np.int64)  # disjoint, ragged alignment
    big = rng.integers(0, 256, int(starts[-1] + lens[-1]) + 64, dtype=np.uint8)
    for i in range(n):
        big[starts[i]:starts[i] + lens[i]] = np.frombuffer(pays[i], np.uint8)
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    d_lens = dev(lens, cuda)
    for vec, vhc in ((1, 0), (1, 1), (1, 2), (0, 0)):
        lib.rudpx_tune(14, vec)
        old_vhc = lib.rudpx_tune(36, vhc)  # varlen tile: prebuilt header chunks, fast phase 2
        try:
            for payload, off in ((dev(packed, cuda), None), (dev(big, cuda), dev(starts, cuda))):
                res = batch.pack_batch_varlen(tab, payload, d_lens, layout, payload_off=off,
                                              want_csum=True)
                assert np.array_equal(host(res.frames), want_fr), (lo, hi, layout, vec, vhc, off is None)
                assert np.array_equal(host(res.frame_off), want_off)
                assert np.array_equal(host(res.csum), want_cs)
            # any hint gives the same frames (raw ABI)
            frames = torch.empty(len(want_fr), dtype=torch.uint8, device=cuda)
            frame_off = torch.empty(n + 1, dtype=torch.int64, device=cuda)
            p = dev(packed, cuda)
            for hint in (0, 7, 1000, 1472, 65535):
                frames.fill_(0xCD)
                b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab[0].data_ptr(),
                                      ack=tab[1].data_ptr(), flags=tab[2].data_ptr(),
                                      payload=p.data_ptr() if p.numel() else 16,
                                      len=d_lens.data_ptr(), payload_off=None)
                _native.check(lib.rudp_encode_varlen(ctypes.byref(b), frames.data_ptr(),
                                                     frame_off.data_ptr(), None, layout, 0,
                                                     torch.cuda.current_stream().cuda_stream))
                assert np.array_equal(host(frames), want_fr), (lo, hi, layout, vec, vhc, hint)
        finally:
            lib.rudpx_tune(14, 1)
            lib.rudpx_tune(36, old_vhc)


@pytest.mark.parametrize("dist", ["uniform2944", "bursty", "empty", "tiny", "mtu"])
@pytest.mark.parametrize("layout", [5, 7])
def test_varlen_encode_tile_kernel_vs_oracle(cuda, dist, layout):
    """The LDS-tile varlen encode (packed payloads) == per-packet vector kernel
    == oracle, at every tile size the hint can pick, including tiles whose run
    overflows the LDS budget (bursts far above the hint: per-packet path)."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(sum(map(ord, dist)) * 10 + layout)
    n = 20011
    if dist == "uniform2944":
        lens = rng.integers(0, 2945, n)
    elif dist == "bursty":   # mostly one character, runs of MTU payloads
        lens = np.where(rng.random(n) < 0.9, 1, 1472)
        lens[5000:5300] = 4000
    elif dist == "empty":
        lens = np.zeros(n, np.int64)
    elif dist == "tiny":
        lens = rng.integers(0, 4, n)
    else:
        lens = np.full(n, 1472)
    lens = lens.astype(np.int32)
    seq, ack, flags, _ = synth.synth(int(rng.integers(1 << 30)), 0, n, 0)
    packed = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    pays, _ = split_by_lengths(packed, lens)
    want_fr, want_off, want_cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    d_lens = dev(lens, cuda)
    p = dev(packed, cuda)
    frames = torch.empty(len(want_fr), dtype=torch.uint8, device=cuda)
    frame_off = torch.empty(n + 1, dtype=torch.int64, device=cuda)
    csum = torch.empty(n, dtype=torch.uint16, device=cuda)
    old_vhc = lib.rudpx_tune(36, 1)
    try:
        for tile, vhc in ((1, 0), (1, 1), (1, 2), (0, 0)):
            lib.rudpx_tune(16, tile)
            lib.rudpx_tune(36, vhc)  # prebuilt header chunks, fast phase 2 (tiles of frames >= 32 B)
            for hint in (0, 1, 16, 100, 800, 1024, 1472, 3000, 6144):
                frames.fill_(0xCD)
                csum.fill_(0)
                b = _native.RudpBatch(n=n, payload_len=hint, reserved=0, seq=tab[0].data_ptr(),
                                      ack=tab[1].data_ptr(), flags=tab[2].data_ptr(),
                                      payload=p.data_ptr() if p.numel() else 16,
                                      len=d_lens.data_ptr(), payload_off=None)
                frame_off.fill_(-1)
                _native.check(lib.rudp_encode_varlen(ctypes.byref(b), frames.data_ptr(),
                                                     frame_off.data_ptr(), csum.data_ptr(), layout, 0,
                                                     torch.cuda.current_stream().cuda_stream))
                assert np.array_equal(host(frames), want_fr), (dist, layout, tile, hint)
                assert np.array_equal(host(frame_off), want_off), (dist, layout, tile, hint)
                assert np.array_equal(host(csum), want_cs), (dist, layout, tile, hint)
    finally:
        lib.rudpx_tune(16, 1)
        lib.rudpx_tune(36, old_vhc)


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 4099, 1 << 20])
def test_device_bounds_match_numpy(cuda, n):
    """rudp_varlen_bounds / rudp_frame_off_bounds == numpy on the same arrays
    (negative int32 lengths show as > 65535; decreasing offsets counted)."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.lib()
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 70000, n).astype(np.int32)
    lens[rng.integers(n)] = -3
    off = rng.integers(-5, 1 << 40, n).astype(np.int64)
    stream = torch.cuda.current_stream().cuda_stream
    out = (ctypes.c_int64 * 5)()
    d_lens, d_off = dev(lens, cuda), dev(off, cuda)  # keep them alive across the calls
    _native.check(lib.rudp_varlen_bounds(d_lens.data_ptr(), d_off.data_ptr(), n, out, 0, stream))
    u = lens.astype(np.uint32).astype(np.int64)
    assert list(out) == [u.min(), u.max(), u.sum(), off.min(), (off + u).max()]
    _native.check(lib.rudp_varlen_bounds(d_lens.data_ptr(), None, n, out, 0, stream))
    assert list(out) == [u.min(), u.max(), u.sum(), 0, u.sum()]
    fo = np.concatenate([[0], np.cumsum(rng.integers(0, 9, n))]).astype(np.int64)
    out3 = (ctypes.c_int64 * 3)()
    d_fo = dev(fo, cuda)
    _native.check(lib.rudp_frame_off_bounds(d_fo.data_ptr(), n, out3, 0, stream))
    assert list(out3) == [fo[0], fo[-1], 0]
    bad = fo.copy()
    k = rng.integers(1, n + 1, 3)
    bad[k] -= 1000
    want_bad = int((bad[1:] < bad[:-1]).sum())
    d_bad = dev(bad, cuda)
    _native.check(lib.rudp_frame_off_bounds(d_bad.data_ptr(), n, out3, 0, stream))
    assert list(out3) == [bad.min(), bad.max(), want_bad]


def test_device_bounds_concurrent_callers(cuda):
    """Eight threads, each on its own stream, take bounds of their own arrays
    at once (the scratch free list hands each call its own slot)."""
    import ctypes
    import threading
    import torch
    from rudp import _native
    lib = _native.lib()
    rng = np.random.default_rng(11)
    arrays = [rng.integers(0, 60000, 50000 + 977 * k).astype(np.int32) for k in range(8)]
    errors = []

    def work(k):
        try:
            s = torch.cuda.Stream(device=cuda)
            with torch.cuda.stream(s):
                d = dev(arrays[k], cuda)
                for _ in range(20):
                    out = (ctypes.c_int64 * 5)()
                    _native.check(lib.rudp_varlen_bounds(d.data_ptr(), None, d.numel(), out, 0,
                                                         s.cuda_stream))
                    a = arrays[k].astype(np.int64)
                    assert list(out) == [a.min(), a.max(), a.sum(), 0, a.sum()], k
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    threads = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("n", [1, 2047, 2048, 2049, 4096 * 1024 + 5])
def test_frame_offset_scans_agree(cuda, n):
    """The three-pass frame-offset scan (default) == hipcub == numpy cumsum."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 65536, n).astype(np.int32) if n < 10000 else \
        rng.integers(0, 3, n).astype(np.int32)
    want = np.concatenate([[0], np.cumsum(lens.astype(np.int64) + 7)])
    d_lens = dev(lens, cuda)
    tab = (torch.zeros(n, dtype=torch.uint16, device=cuda), torch.zeros(n, dtype=torch.uint16, device=cuda),
           torch.zeros(n, dtype=torch.uint8, device=cuda))
    pay = torch.zeros(int(lens.sum()), dtype=torch.uint8, device=cuda)
    try:
        for scan in (1, 0):
            lib.rudpx_tune(24, scan)
            res = batch.pack_batch_varlen(tab, pay, d_lens, 7)
            assert np.array_equal(host(res.frame_off), want), (n, scan)
    finally:
        lib.rudpx_tune(24, 1)


@pytest.mark.parametrize("L", [1, 5, 16, 17, 64, 100, 256, 1472, 4096])
def test_utf8_fixed_stride_tile_and_vector_kernels(cuda, L):
    """Fixed-stride frames: the LDS-tile validator (default) and the per-frame
    vector kernel (rudpx_tune 31 = 0) both equal Python's strict decoder, on
    near-UTF-8 bodies cut or padded to L bytes (multibyte characters cross
    16-B chunk and tile boundaries; both outcomes well represented)."""
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int
    rng = np.random.default_rng(4321 + L)
    n = 3001
    bodies = []
    for b in _near_utf8(rng, n):
        reps = b * (L // max(1, len(b)) + 1) if b else b"A" * L
        bodies.append((reps + b"A" * L)[:L])
    for H in (5, 7):
        hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
        fr = np.frombuffer(b"".join(hdr + x for x in bodies), np.uint8).reshape(n, L + H)
        off = np.arange(n + 1, dtype=np.int64) * (L + H)
        want = codec_np.utf8_valid(fr.reshape(-1), off, H)
        if L >= 16:
            assert 0.05 < want.mean() < 0.95, want.mean()
        for tile in (1, 0):
            old = lib.rudpx_tune(31, tile)
            try:
                got = host(batch.validate_utf8(dev(fr, cuda), H))
            finally:
                lib.rudpx_tune(31, old)
            assert np.array_equal(got, want), (L, H, tile)


@pytest.mark.parametrize("window", [1, 500, 4096])
def test_dedup_table_heavy_repeats_and_collisions(cuda, window):
    """Long chains: few distinct frames (every bucket chain holds many equal
    hashes, most outside the window), empty datagrams (equal to the 40-bit zero
    header), and 20K frames so windows cross many workgroups."""
    rng = np.random.default_rng(99 + window)
    pool = [b"", bytes(5), b"\x01", b"\x00\x00\x00\x00\x00\x00"] + \
           [bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)) for _ in range(60)]
    seq = [pool[int(k)] for k in rng.integers(0, len(pool), 20000)]
    off = np.concatenate([[0], np.cumsum([len(f) for f in seq])]).astype(np.int64)
    flat = np.frombuffer(b"".join(seq) + b"\x00", np.uint8)[:-1] if off[-1] else np.zeros(0, np.uint8)
    canon = [f if f else bytes(5) for f in seq]  # Packet(b"") equals the zero header
    last, want = {}, []
    for i, k in enumerate(canon):
        want.append(int(k in last and last[k] >= i - window))
        last[k] = i
    for table in (1, 0):
        with _dedup_form(table):
            got = host(batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(off, cuda),
                                                    window=window))
        assert got.tolist() == want, table


@pytest.mark.parametrize("mean_len", [6, 40, 200, 1500])
def test_dedup_lanes_per_frame_and_bad_offsets(cuda, mean_len):
    """The hash pass takes 1-8 lanes per frame from the mean frame length: same
    flags at every length; a frame whose offsets are decreasing or past the
    buffer gets 2 (RUDP_DUP_BAD_OFFSETS), equals nothing, and check=True raises."""
    rng = np.random.default_rng(mean_len)
    pool = [bytes(rng.integers(0, 256, max(0, int(rng.normal(mean_len, mean_len / 4))), dtype=np.uint8))
            for _ in range(300)]
    seq = [pool[int(k)] for k in rng.integers(0, len(pool), 5000)]
    off = np.concatenate([[0], np.cumsum([len(f) for f in seq])]).astype(np.int64)
    flat = np.frombuffer(b"".join(seq) + b"\x00", np.uint8)[:-1]
    canon = [f if f else bytes(5) for f in seq]
    last, want = {}, []
    for i, k in enumerate(canon):
        want.append(int(k in last and last[k] >= i - 500))
        last[k] = i
    got = host(batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(off, cuda), window=500))
    assert got.tolist() == want
    bad = off.copy()
    bad[100] = bad[101] + 1           # frame 100 decreasing
    bad[-1] = len(flat) + 7           # the last frame past the buffer
    d = host(batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(bad, cuda), window=500, check=False))
    assert d[100] == _native.DUP_BAD_OFFSETS and d[-1] == _native.DUP_BAD_OFFSETS
    assert int((d == _native.DUP_BAD_OFFSETS).sum()) == 2
    with pytest.raises(ValueError, match="non-decreasing"):
        batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(bad, cuda), window=500)


def test_utf8_packed_tile_vs_python_decoder(cuda):
    """Packed frames of 0.3-3 KB (mean-length hint >= 128 B: the LDS-tile
    validator; a low hint: every tile overflows its budget and checks its
    frames from HBM) == per-frame vector kernel == Python's strict decoder."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int
    rng = np.random.default_rng(2468)
    bodies = []
    for b in _near_utf8(rng, 3000):
        L = int(rng.integers(300, 3000))
        bodies.append(((b or b"A") * (L // max(1, len(b)) + 1))[:L])
    frames = [b"\x12\x34\x00\x00\x80" + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    want = codec_np.utf8_valid(flat, off, 5)
    assert 0.05 < want.mean() < 0.95
    d_flat, d_off = dev(flat, cuda), dev(off, cuda)
    out = torch.empty(len(frames), dtype=torch.uint8, device=cuda)
    for vtile in (1, 0):
        old = lib.rudpx_tune(41, vtile)
        try:
            got = host(batch.validate_utf8(d_flat, 5, frame_off=d_off))
            assert np.array_equal(got, want), vtile
            for hint in (200, 512, 1600, 4000):  # 200/512: runs overflow the tile budget
                out.fill_(7)
                _native.check(lib.rudp_validate_utf8(d_flat.data_ptr(), d_off.data_ptr(), hint,
                                                     len(frames), 5, out.data_ptr(), 0,
                                                     torch.cuda.current_stream().cuda_stream))
                assert np.array_equal(host(out), want), (vtile, hint)
        finally:
            lib.rudpx_tune(41, old)


# ------------------------------------------------ sync-free (device-checked) entries
def test_varlen_sync_free_matches_checked(cuda):
    """check=False never waits for the device and gives the same frames / fields."""
    import torch
    rng = np.random.default_rng(41)
    n = 20011
    lens = rng.integers(0, 300, n).astype(np.int32)
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(41, 0, n, 0)
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    for layout in (5, 7):
        a = batch.pack_batch_varlen(tab, dev(pay, cuda), dev(lens, cuda), layout, want_csum=True)
        b = batch.pack_batch_varlen(tab, dev(pay, cuda), dev(lens, cuda), layout, want_csum=True, check=False)
        b.check()
        assert int(b.status.item()) == 0
        assert torch.equal(a.frames, b.frames) and torch.equal(a.frame_off, b.frame_off)
        want, off, cs = codec_np.encode_varlen(seq, ack, flags, split_by_lengths(pay, lens)[0], layout)
        assert np.array_equal(host(b.frames), want) and np.array_equal(host(b.csum), cs)
        d = batch.unpack_batch_varlen(b.frames, b.frame_off, layout, csum=b.csum if layout == 5 else None,
                                      check=False)
        assert int(d.status.item()) == 0 and bool((d.ok == 1).all())
        assert np.array_equal(host(d.seq), seq)
        # caller-provided frame buffer larger than needed: the frames are its prefix
        big = torch.full((int(lens.sum()) + n * layout + 100,), 0xAA, dtype=torch.uint8, device=cuda)
        c = batch.pack_batch_varlen(tab, dev(pay, cuda), dev(lens, cuda), layout, out=big, check=False).check()
        assert c.frames is big and np.array_equal(host(big[:len(want)]), want)
        assert (host(big[len(want):]) == 0xAA).all()


def test_varlen_device_checks_reject_bad_batches(cuda):
    """Every argument check runs on the device; a rejected batch writes no frames."""
    import torch
    n = 4096
    seq, ack, flags, _ = synth.synth(5, 0, n, 0)
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    lens = np.full(n, 3, np.int32)
    pay = dev(np.zeros(3 * n, np.uint8), cuda)

    def rejected(match, **kw):
        kw.setdefault("payload", pay)
        kw.setdefault("lengths", dev(lens, cuda))
        for check in (True, False):
            out = torch.full((4 * 70000 * 7 + 64,), 0x5C, dtype=torch.uint8, device=cuda) \
                if "out" not in kw else kw["out"]
            args = dict(kw, out=out)
            with pytest.raises(ValueError, match=match):
                r = batch.pack_batch_varlen(tab, args.pop("payload"), args.pop("lengths"), 7, check=check,
                                            **args)
                r.check()  # check=False: raises here, not inside the call
            assert bool((out == 0x5C).all()), "a rejected batch must leave the frame buffer alone"

    bad = lens.copy(); bad[777] = 70000
    rejected("65535", lengths=dev(bad, cuda), payload=dev(np.zeros(int(bad.sum()), np.uint8), cuda))
    rejected("sum", lengths=dev(lens + 1, cuda))
    offs = (np.arange(n) * 3).astype(np.int64); offs[100] = 3 * n - 1
    rejected("inside payload", payload_off=dev(offs, cuda))
    offs2 = offs.copy(); offs2[5] = -4
    rejected("inside payload", payload_off=dev(offs2, cuda))
    small = torch.full((n * 10 - 1,), 0x5C, dtype=torch.uint8, device=cuda)
    rejected("too small", out=small)
    # without check the call returns at once; the status tells.  Contract on a
    # rejected batch (include/rudp.h): frame_off[n] holds the scan's total on every
    # path -- the small-frame kernel (hint 4 B) and the scan + tile path (300 B).
    r = batch.pack_batch_varlen(tab, pay, dev(lens + 1, cuda), 7, check=False)
    assert int(r.status.item()) & 2
    assert int(r.frame_off[-1].item()) == 4 * n + 7 * n
    big = np.full(n, 300, np.int32)
    r = batch.pack_batch_varlen(tab, dev(np.zeros(300 * n - 1, np.uint8), cuda), dev(big, cuda), 7, check=False)
    assert int(r.status.item()) & 2
    assert int(r.frame_off[-1].item()) == 307 * n
    # decode: offsets decreasing, past the buffer, negative
    fr = batch.pack_batch_varlen(tab, pay, dev(lens, cuda), 7)
    for mut in ((7, 3), (n, 10 ** 9), (0, -8)):
        off = fr.frame_off.clone()
        off[mut[0]] = mut[1]
        for check in (True, False):
            with pytest.raises(ValueError, match="non-decreasing"):
                batch.unpack_batch_varlen(fr.frames, off, 7, check=check).check()


def test_varlen_empty_batches_sync_free(cuda):
    import torch
    z = torch.zeros(0, dtype=torch.uint16, device=cuda)
    r = batch.pack_batch_varlen((z, z, z.to(torch.uint8)), torch.zeros(0, dtype=torch.uint8, device=cuda),
                                torch.zeros(0, dtype=torch.int32, device=cuda), 5, check=False).check()
    assert r.frames.numel() == 0 and host(r.frame_off).tolist() == [0]
    d = batch.unpack_batch_varlen(r.frames, r.frame_off, 5, check=False).check()
    assert d.ok.numel() == 0
    # header-only frames (all lengths 0): frames exist, payload buffer is empty
    n = 1000
    seq, ack, flags, _ = synth.synth(8, 0, n, 0)
    r = batch.pack_batch_varlen((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)),
                                torch.zeros(0, dtype=torch.uint8, device=cuda),
                                torch.zeros(n, dtype=torch.int32, device=cuda), 7, check=False).check()
    want, _, _ = codec_np.encode_varlen(seq, ack, flags, [b""] * n, 7)
    assert np.array_equal(host(r.frames), want)


@pytest.mark.parametrize("slots", [1, 2, 4])
def test_socket_ring_overlapped_decode_side_stream(cuda, slots):
    """The receive ring (§8f row 1): recvmmsg into slot k+1 while slot k's H2D copy
    and decode run on a side stream; every batch equals the oracle's decode."""
    import socket
    import threading

    import torch
    from rudp import netio
    n = 30000
    rng = np.random.default_rng(50 + slots)
    seq, ack, flags, _ = synth.synth(50 + slots, 0, n, 0)
    pays = [rng.integers(32, 127, int(k), dtype=np.uint8).tobytes() for k in rng.integers(1, 9, n)]
    fr, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    fr = fr.copy()
    fr[off[999] + 3] ^= 0x20  # one corrupted datagram
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    side = torch.cuda.Stream(cuda)
    recv = netio.BatchReceiver(rx, max_msgs=4096, slot_bytes=64, slots=slots, device=cuda, stream=side)
    t = threading.Thread(target=lambda: netio.send_batch(tx, fr, off, "127.0.0.1", rx.getsockname()[1]))
    t.start()
    pending, got = [], 0
    while got < n:
        k = recv.recv(timeout_ms=3000)
        assert k > 0
        # what the socket delivered into this slot (copied before the slot is reused)
        snap = (recv.frames[:recv.frame_off[k]].copy(), recv.frame_off[:k + 1].copy())
        dec, d_frames, d_off = recv.decode("rudp7")  # async: the next recv overlaps it
        pending.append((snap, dec, d_frames, d_off))
        got += k
    t.join()
    torch.cuda.synchronize()
    i0 = 0
    for (h_fr, h_off), dec, d_frames, d_off in pending:
        dec.check()
        k = len(h_off) - 1
        host_frames = [bytes(h_fr[h_off[i]:h_off[i + 1]]) for i in range(k)]
        want = [bytes(fr[off[i]:off[i + 1]]) for i in range(i0, i0 + k)]
        assert host_frames == want
        flat = np.frombuffer(b"".join(want), np.uint8)
        w_off = np.concatenate([[0], np.cumsum([len(x) for x in want])]).astype(np.int64)
        exp = codec_np.decode_varlen(flat, w_off, 7)
        for g, e in zip((dec.seq, dec.ack, dec.flags, dec.ok, dec.csum), exp):
            assert np.array_equal(host(g), e)
        assert np.array_equal(host(d_frames), flat) and np.array_equal(host(d_off), w_off)
        i0 += k
    assert i0 == n
    rx.close()
    tx.close()


@pytest.mark.parametrize("fpt", [1, 2, 4, 8])
def test_small_frame_tiles_vs_oracle(cuda, fpt):
    """Small-frame varlen encode (scan's last pass + framing in one tile kernel)
    and decode tiles, every tile size: tiles that fit, tiles with a burst past
    the LDS budget (per-packet path), ragged last tiles, both layouts."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(70 + fpt)
    for n, lo, hi, burst in ((1, 0, 3, False), (255, 1, 1, False), (256 * fpt + 3, 0, 9, False),
                             (5 * 256 * fpt - 1, 1, 4, True), (40000, 0, 15, True)):
        lens = rng.integers(lo, hi + 1, n).astype(np.int32)
        if burst:
            lens[n // 3] = 9000  # far past the tile's budget at these hints
        pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        seq, ack, flags, _ = synth.synth(fpt * 1000 + n, 0, n, 0)
        pays = split_by_lengths(pay, lens)[0]
        for layout in (5, 7):
            want, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
            results = []
            # the small-frame kernels (own tile bases: lengths from pass 1's 4-bit codes, code 15
            # reading len[] again, or from len[]; then after the pass-2 launch), then the vector kernels
            for small, fused, nib in ((16, 1, 1), (16, 1, 0), (16, 0, 1), (0, 1, 1)):
                old = (lib.rudpx_tune(46, small), lib.rudpx_tune(47, fpt), lib.rudpx_tune(50, fused),
                       lib.rudpx_tune(74, nib))
                try:
                    r = batch.pack_batch_varlen((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda),
                                                dev(lens, cuda), layout, want_csum=True, check=False).check()
                    d = batch.unpack_batch_varlen(r.frames, r.frame_off, layout,
                                                  csum=r.csum if layout == 5 else None, check=False).check()
                    bad_off = r.frame_off.clone()
                    if n > 2:
                        bad_off[n // 2] = bad_off[n // 2 + 1] + 1  # one decreasing pair
                        db = batch.unpack_batch_varlen(r.frames, bad_off, layout, check=False)
                        assert int(db.status.item()) == _native.ST_OFFSETS
                        okb = host(db.ok)
                        assert okb[n // 2 - 1] == 4 or okb[n // 2] == 4
                finally:
                    lib.rudpx_tune(46, old[0])
                    lib.rudpx_tune(47, old[1])
                    lib.rudpx_tune(50, old[2])
                    lib.rudpx_tune(74, old[3])
                ctx = (fpt, n, layout, small, fused, nib)
                assert np.array_equal(host(r.frames), want), ctx
                assert np.array_equal(host(r.frame_off), off) and np.array_equal(host(r.csum), cs), ctx
                exp = codec_np.decode_varlen(want, off, layout, cs if layout == 5 else None)
                for g, e in zip((d.seq, d.ack, d.flags, d.ok, d.csum), exp):
                    assert np.array_equal(host(g), e), ctx
                results.append(host(r.frames))
            assert all(np.array_equal(results[0], x) for x in results[1:])


@pytest.mark.parametrize("dist", ["ragged", "equal", "bursty", "tiny_runs", "zeros", "jumbo", "threshold"])
def test_varlen_tile_forms_vs_oracle(cuda, dist):
    """Varlen encode tile forms (key 51 packet / byte tiles / the device's choice;
    52 each sum pass) == the oracle, checksums included, for
    ragged / equal lengths, bursts past the budget's slack, long runs of tiny
    packets (more than a tile's slots), zero-length packets and packets longer
    than a whole tile's LDS budget."""
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(sum(map(ord, dist)))
    n = 20011
    if dist == "ragged":
        lens = rng.integers(0, 2945, n)
    elif dist == "equal":
        lens = np.full(n, 1472)
    elif dist == "bursty":
        lens = rng.integers(1000, 2000, n)
        lens[rng.choice(n, 40, replace=False)] = rng.integers(5000, 20000, 40)
    elif dist == "tiny_runs":
        lens = rng.integers(1200, 1700, n)
        for s0 in rng.choice(n - 400, 10, replace=False):
            lens[s0:s0 + 300] = rng.integers(0, 3, 300)
    elif dist == "zeros":
        lens = rng.integers(0, 2945, n)
        lens[rng.random(n) < 0.3] = 0
    elif dist == "threshold":  # frames around the 32-B prebuilt-header-chunk limit among MTU ones
        lens = rng.integers(1300, 1600, n)
        m = rng.random(n) < 0.35
        lens[m] = rng.choice(np.array([0, 1, 9, 15, 16, 17, 23, 24, 25, 26, 27, 28, 40]), int(m.sum()))
    else:  # jumbo: a few packets over a whole tile's budget (~27 KB at a 1.5-KB hint)
        lens = rng.integers(1000, 2000, n)
        lens[rng.choice(n, 12, replace=False)] = rng.integers(30000, 60000, 12)
    lens = lens.astype(np.int32)
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(0xB7 + n, 0, n, 0)
    pays = split_by_lengths(pay, lens)[0]
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    for layout in (5, 7):
        want, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
        # (tile form: 1 the scan's choice / 2 byte tiles / 3 packet tiles through
        # records / 0 packet tiles from frame_off, sum pass: 2 block sums / 0
        # chunks, XCD order)
        for knobs in ((1, 2, 1), (1, 0, 1), (1, 2, 0), (3, 2, 1), (2, 2, 1), (2, 2, 0), (2, 0, 1), (0, 2, 1),
                      (0, 0, 1), (0, 2, 0)):
            old = [lib.rudpx_tune(key, v) for key, v in zip((51, 52, 49), knobs)]
            try:
                r = batch.pack_batch_varlen(tab, dev(pay, cuda), dev(lens, cuda), layout, want_csum=True,
                                            check=False).check()
            finally:
                for key, v in zip((51, 52, 49), old):
                    lib.rudpx_tune(key, v)
            ctx = (dist, layout, knobs)
            assert np.array_equal(host(r.frames), want), ctx
            assert np.array_equal(host(r.frame_off), off), ctx
            assert np.array_equal(host(r.csum), cs), ctx


@pytest.mark.parametrize("world", [2, 8])
def test_varlen_rank_shards_rebase_to_unsharded(cuda, world):
    """SURVEY.md §8e for variable lengths: each rank encodes its packet slice on
    the GPU (its own scan, offsets from 0); rebased by rudp.shard.frame_base
    the shards concatenate to the unsharded GPU encode and the oracle."""
    from rudp import shard
    rng = np.random.default_rng(0x5A + world)
    n = 8192
    lens = rng.integers(0, 2945, n).astype(np.int32)
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(0x5A, 0, n, 0)
    bounds = np.concatenate([[0], np.cumsum(lens)])
    want, want_off, want_cs = codec_np.encode_varlen(seq, ack, flags, split_by_lengths(pay, lens)[0], 7)
    full = batch.pack_batch_varlen((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda),
                                   dev(lens, cuda), 7, want_csum=True)
    frames, offs, csums, totals = [], [], [], []
    for r in range(world):
        first, m = shard.rank_slice(r, world, n)
        sl = slice(first, first + m)
        res = batch.pack_batch_varlen((dev(seq[sl], cuda), dev(ack[sl], cuda), dev(flags[sl], cuda)),
                                      dev(pay[bounds[first]:bounds[first + m]], cuda), dev(lens[sl], cuda), 7,
                                      want_csum=True)
        frames.append(host(res.frames))
        offs.append(host(res.frame_off).astype(np.int64))
        csums.append(host(res.csum))
        totals.append(int(offs[-1][-1]))
    glob = [o + shard.frame_base(totals, r) for r, o in enumerate(offs)]
    got_off = np.concatenate([g[:-1] for g in glob] + [glob[-1][-1:]])
    assert np.array_equal(np.concatenate(frames), want) and np.array_equal(host(full.frames), want)
    assert np.array_equal(got_off, np.asarray(want_off)) and np.array_equal(host(full.frame_off), np.asarray(want_off))
    assert np.array_equal(np.concatenate(csums), want_cs)


@pytest.mark.parametrize("L", [1, 300])
def test_varlen_reuse_outputs_equal_fresh(cuda, L):
    """reuse= hands an earlier result's buffers to the next call (no allocation):
    the outputs equal a fresh call's and the oracle's; a mismatched shape is refused;
    the decode's status (no status word) still reports a rejected frame."""
    import torch
    n = 5000
    seq, ack, flags, pay = synth.synth(21, 0, n, L)
    tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
    lens = dev(np.full(n, L, np.int32), cuda)
    flat = dev(pay.reshape(-1), cuda)
    want_fr, want_off, want_cs = codec_np.encode_varlen(seq, ack, flags, [p.tobytes() for p in pay], 5)
    first = batch.pack_batch_varlen(tab, flat, lens, 5, want_csum=True)
    keep = first.frames.clone()
    seq2, ack2, flags2, pay2 = synth.synth(22, 0, n, L)
    tab2 = (dev(seq2, cuda), dev(ack2, cuda), dev(flags2, cuda))
    again = batch.pack_batch_varlen(tab2, dev(pay2.reshape(-1), cuda), lens, 5, want_csum=True, reuse=first,
                                    check=False).check()
    assert again._buf.data_ptr() == first._buf.data_ptr()
    want2, _, want_cs2 = codec_np.encode_varlen(seq2, ack2, flags2, [p.tobytes() for p in pay2], 5)
    assert np.array_equal(host(again.frames), want2) and np.array_equal(host(again.csum), want_cs2)
    assert np.array_equal(host(keep), want_fr) and np.array_equal(host(again.frame_off), want_off)
    with pytest.raises(ValueError, match="reuse"):
        batch.pack_batch_varlen(tab, flat, lens, 5, want_csum=False, reuse=again)
    d1 = batch.unpack_batch_varlen(again.frames, again.frame_off, 5, csum=again.csum)
    d2 = batch.unpack_batch_varlen(again.frames, again.frame_off, 5, csum=again.csum, reuse=d1, check=False)
    assert d2._buf.data_ptr() == d1._buf.data_ptr()
    want_d = codec_np.decode_varlen(want2, want_off, 5, want_cs2)
    for got, exp in zip((d2.seq, d2.ack, d2.flags, d2.ok, d2.csum), want_d):
        assert np.array_equal(host(got), exp)
    bad = again.frame_off.clone()
    bad[17] = bad[18] + 1
    d3 = batch.unpack_batch_varlen(again.frames, bad, 5, csum=again.csum, reuse=d2, check=False)
    # frame 17 = [off[18] + 1, off[18]) is decreasing: rejected; frame 16 only grew (checksum)
    assert int(d3.status.item()) == _native.ST_OFFSETS and int(d3.ok[17].item()) == _native.OK_BAD_OFFSETS
    assert int((d3.ok == _native.OK_BAD_OFFSETS).sum().item()) == 1
    with pytest.raises(ValueError, match="non-decreasing"):
        d3.check()
    assert torch.equal(d3.ok[:16], torch.ones(16, dtype=torch.uint8, device=cuda))


def test_varlen_decode_status_on_side_stream(cuda):
    """a decode enqueued on a side stream behind long work, checked from
    the caller's current stream: the status is reduced on the decode's stream, so
    check() sees the rejected frame (it read ok[] before the kernel wrote it when
    the reduction ran on the current stream)."""
    import torch
    n = 4096
    frames = torch.zeros(n * 8, dtype=torch.uint8, device=cuda)
    off = torch.arange(0, n * 8 + 1, 8, dtype=torch.int64, device=cuda)
    off[100] = 10 ** 9  # frames 99 and 100 reach past the buffer
    side = torch.cuda.Stream(device=cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    for _ in range(3):
        with torch.cuda.stream(side):
            torch.cuda._sleep(50_000_000)  # ~20 ms of GPU time before the decode on `side`
        d = batch.unpack_batch_varlen(frames, off, "rudp7", stream=side, check=False)
        with pytest.raises(ValueError, match="non-decreasing"):
            d.check()
    torch.cuda.synchronize()
