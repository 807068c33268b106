"""Decode + strict UTF-8 in one pass (rudp_decode_utf8 / rudp_decode_varlen_utf8, ABI 6).

The reference's receive parses every datagram and decodes its payload:
utils/reliableUDP.py:118-123 (Packet(data) -> get_header_field ... ->
get_payload), whose strict bytes.decode() is utils/packet.py:73.  The fused
calls must give exactly the unfused decode's fields plus rudp_validate_utf8's
answer, pinned by the reference's own get_payload() outcomes
(tests/golden/varlen.npz ``utf8_valid``) and, for generated bodies, by
Python's strict decoder (oracle/codec_np.utf8_valid), in every kernel form:
small-frame tiles, vector, LDS tiles, tiles over their budget, byte kernels
(misaligned buffers), fixed-length tiles (verify and copy-out, staged and
unstaged outputs) and the fixed-length fallbacks (frames past a 64 KiB tile,
payload lengths that are not a multiple of 16).
"""
import numpy as np
import pytest

from conftest import split_by_lengths
from oracle import codec_np
from rudp import _native, batch

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).to(cuda)


def host(t):
    return t.cpu().numpy()


def _near_utf8(rng, n, lo=0, hi=12):
    """Mostly-valid UTF-8 strings with a few random byte edits (hits every DFA edge)."""
    chars = [chr(c) for c in (0x41, 0x7F, 0x80, 0x7FF, 0x800, 0xD7FF, 0xE000, 0xFFFD, 0xFFFF,
                               0x10000, 0x1F600, 0x10FFFF, 0xE9, 0x4E2D)]
    out = []
    for _ in range(n):
        s = "".join(chars[i] for i in rng.integers(0, len(chars), rng.integers(lo, hi))).encode()
        b = bytearray(s)
        for _ in range(rng.integers(0, 3)):
            if b and rng.random() < 0.7:
                b[rng.integers(0, len(b))] = int(rng.integers(0, 256))
            elif rng.random() < 0.5 and b:
                del b[rng.integers(0, len(b))]
            else:
                b.insert(int(rng.integers(0, len(b) + 1)),
                         int(rng.choice([0x80, 0xBF, 0xC0, 0xE0, 0xED, 0xF0, 0xF4, 0xF5])))
        out.append(bytes(b))
    return out


def _pack(frames):
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames) + b"\x00", np.uint8)[:-1]
    return flat, off


def _varlen_decode(d_flat, nbytes, d_off, n, hint, H, utf8, csum=None):
    """Raw ABI call with an explicit length hint (it picks the kernel form)."""
    import torch
    dv = d_off.device
    out = {k: torch.full((n,), 0xAB, dtype=dt, device=dv) for k, dt in
           (("seq", torch.uint16), ("ack", torch.uint16), ("flags", torch.uint8), ("ok", torch.uint8),
            ("csum", torch.uint16), ("valid", torch.uint8))}
    _native.check(_native.lib().rudp_decode_varlen_utf8(
        d_flat.data_ptr(), nbytes, d_off.data_ptr(), hint, n, csum.data_ptr() if csum is not None else None,
        out["seq"].data_ptr(), out["ack"].data_ptr(), out["flags"].data_ptr(), out["ok"].data_ptr(),
        out["csum"].data_ptr(), out["valid"].data_ptr() if utf8 else None, None, H, 0,
        torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    if not utf8:
        del out["valid"]
    return {k: host(v) for k, v in out.items()}


def _check_all_forms(cuda, frames, H, hints, want_valid=None):
    """Every hint (and a misaligned copy: the byte kernel) gives the unfused
    decode's fields and the strict decoder's answer."""
    import torch
    flat, off = _pack(frames)
    if want_valid is None:
        want_valid = codec_np.utf8_valid(flat, off, H)
    n = len(frames)
    d_flat, d_off = dev(flat, cuda), dev(off, cuda)
    raw = torch.zeros(len(flat) + 32, dtype=torch.uint8, device=cuda)
    mis = raw[3:3 + len(flat)]
    mis.copy_(d_flat)
    for buf in (d_flat, mis):
        for hint in hints:
            plain = _varlen_decode(buf, len(flat), d_off, n, hint, H, False)
            fused = _varlen_decode(buf, len(flat), d_off, n, hint, H, True)
            ctx = (H, hint, buf is mis)
            assert np.array_equal(fused.pop("valid"), want_valid), ctx
            for k in plain:
                assert np.array_equal(fused[k], plain[k]), (k,) + ctx
    return want_valid


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_fused_matches_reference_get_payload(cuda, golden_varlen, H):
    """The reference's 333 get_payload() outcomes, through the small-frame
    tile (hint 0), the vector kernel (64), LDS tiles (200, 1600) and the byte
    kernel (misaligned)."""
    g = golden_varlen
    bodies, _ = split_by_lengths(g["utf8_bodies"], g["utf8_lengths"])
    hdr = b"\x00\x01\x00\x02\x40" + (b"\x12\x34" if H == 7 else b"")
    _check_all_forms(cuda, [hdr + b for b in bodies], H, (0, 64, 200, 1600), g["utf8_valid"])


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_fused_small_and_ragged_bodies(cuda, H):
    """Generated near-UTF-8 bodies: 1-40 B (small tiles, some over budget at
    hint 0), and 300-3000 B (tiles and their per-frame fallback)."""
    rng = np.random.default_rng(600 + H)
    hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
    small = [hdr + b for b in _near_utf8(rng, 20000, 0, 12)]
    v = _check_all_forms(cuda, small, H, (0, 16, 64))
    assert 0.2 < v.mean() < 0.9
    big = []
    for b in _near_utf8(rng, 2000):
        L = int(rng.integers(300, 3000))
        big.append(hdr + ((b or b"A") * (L // max(1, len(b)) + 1))[:L])
    v = _check_all_forms(cuda, big, H, (0, 200, 1600, 4000))
    assert 0.05 < v.mean() < 0.95


def test_varlen_fused_short_empty_and_rejected_frames(cuda):
    """Frames shorter than the header: get_payload() is None, valid 1.  A
    frame with bad offsets is rejected (ok 4) and valid 0: nothing of it is read."""
    import torch
    frames = [bytes(range(0xC0, 0xC0 + k)) for k in range(12)] + [b"\x00\x01\x00\x02\x40\xff"]
    flat, off = _pack(frames)
    for H in (5, 7):
        want = codec_np.utf8_valid(flat, off, H)
        assert want[:H + 1].all()  # header-only and shorter frames: None, never raises
        for hint in (0, 64, 200):
            got = _varlen_decode(dev(flat, cuda), len(flat), dev(off, cuda), len(frames), hint, H, True)
            assert np.array_equal(got["valid"], want), (H, hint)
    bad = off.copy()
    bad[3] = bad[4] + 1                # frame 3 decreasing
    bad[-1] = len(flat) + 9            # the last frame past the buffer
    for hint in (0, 64, 200):
        got = _varlen_decode(dev(flat, cuda), len(flat), dev(bad, cuda), len(frames), hint, 5, True)
        assert got["ok"][3] == _native.OK_BAD_OFFSETS and got["ok"][-1] == _native.OK_BAD_OFFSETS
        assert got["valid"][3] == 0 and got["valid"][-1] == 0, hint
    d = batch.unpack_batch_varlen(dev(flat, cuda), dev(bad, cuda), 5, check=False, utf8=True)
    assert int(d.status.item()) == _native.ST_OFFSETS and d.status.dtype == torch.int32
    assert host(d.valid)[3] == 0


def test_unpack_batch_varlen_utf8_and_reuse(cuda, golden_varlen):
    """The Python entry: valid next to the usual fields; reuse= keeps the choice."""
    g = golden_varlen
    bodies, _ = split_by_lengths(g["utf8_bodies"], g["utf8_lengths"])
    flat, off = _pack([b"\x00\x01\x00\x02\x40" + b for b in bodies])
    d_flat, d_off = dev(flat, cuda), dev(off, cuda)
    d = batch.unpack_batch_varlen(d_flat, d_off, 5, utf8=True)
    assert np.array_equal(host(d.valid), g["utf8_valid"])
    plain = batch.unpack_batch_varlen(d_flat, d_off, 5)
    assert plain.valid is None
    for k in ("seq", "ack", "flags", "ok", "csum"):
        assert np.array_equal(host(getattr(d, k)), host(getattr(plain, k))), k
    d2 = batch.unpack_batch_varlen(d_flat, d_off, 5, utf8=True, reuse=d)
    assert np.array_equal(host(d2.valid), g["utf8_valid"])
    with pytest.raises(ValueError, match="utf8"):
        batch.unpack_batch_varlen(d_flat, d_off, 5, reuse=d)


def _fixed_frames(rng, n, L, H, ascii_share=0.0):
    bodies = []
    for b in _near_utf8(rng, n):
        if rng.random() < ascii_share:
            b = bytes(rng.integers(0x20, 0x7F, 8, dtype=np.uint8))
        reps = b * (L // max(1, len(b)) + 1) if b else b"A" * L
        bodies.append((reps + b"A" * L)[:L])
    hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
    return np.frombuffer(b"".join(hdr + x for x in bodies), np.uint8).reshape(n, L + H)


@pytest.mark.parametrize("L", [0, 1, 16, 17, 64, 256, 1472, 2048, 4096])
@pytest.mark.parametrize("H", [5, 7])
def test_fixed_fused_vs_strict_decoder(cuda, L, H):
    """Fixed-length frames: the LDS-tile decode (verify and copy-out, staged
    and unstaged outputs) judges UTF-8 in its pass; other shapes (L % 16 != 0,
    tiles past 64 KiB) run the validation kernel after it.  Same fields as
    rudp_decode, valid == Python's strict decoder."""
    import torch
    rng = np.random.default_rng(9000 + 10 * L + H)
    n = 4099
    fr = _fixed_frames(rng, n, L, H, ascii_share=0.3)
    off = np.arange(n + 1, dtype=np.int64) * (L + H)
    want = codec_np.utf8_valid(fr.reshape(-1), off, H)
    if L >= 16:
        assert 0.05 < want.mean() < 0.95
    d = dev(fr, cuda)
    cs = None
    if H == 5:  # sideband checksums: from an encode of the same bodies
        enc, cs = batch.pack_batch((dev(fr[:, 0].astype(np.uint16) << 8 | fr[:, 1], cuda),
                                    dev(fr[:, 2].astype(np.uint16) << 8 | fr[:, 3], cuda),
                                    dev(fr[:, 4], cuda)), dev(fr[:, H:], cuda), 5)
        assert torch.equal(enc, d)
    for copy in (False, True):
        a = batch.unpack_batch(d, H, csum=cs, copy_payload=copy)
        b = batch.unpack_batch(d, H, csum=cs, copy_payload=copy, utf8=True)
        assert np.array_equal(host(b.valid), want), copy
        for k in ("seq", "ack", "flags", "ok", "csum", "payload"):
            assert torch.equal(getattr(a, k), getattr(b, k)), (k, copy)
        assert a.valid is None
    # unstaged outputs: a valid array off 4-byte alignment
    raw = torch.full((n + 8,), 9, dtype=torch.uint8, device=cuda)
    outs = [torch.empty((n,), dtype=dt, device=cuda) for dt in
            (torch.uint16, torch.uint16, torch.uint8, torch.uint8, torch.uint16)]
    _native.check(_native.lib().rudp_decode_utf8(
        d.data_ptr() if d.numel() else None, None, L + H, n, cs.data_ptr() if cs is not None else None,
        *(o.data_ptr() for o in outs), None, raw.data_ptr() + 1, H, 0, torch.cuda.current_stream().cuda_stream))
    assert np.array_equal(host(raw[1:n + 1]), want)
    assert int(raw[0].item()) == 9 and int(raw[n + 1].item()) == 9


def test_fixed_fused_ascii_and_reference_frames(cuda, golden_small):
    """Reference-framed batches (ASCII payloads: all valid) and the full-range
    byte batches of tests/golden/frames_small.npz."""
    for L in (1, 16, 64, 1472):
        fr = golden_small[f"L{L}_full_frames7"]
        off = np.arange(fr.shape[0] + 1, dtype=np.int64) * fr.shape[1]
        want = codec_np.utf8_valid(fr.reshape(-1), off, 7)
        got = batch.unpack_batch(dev(fr, cuda), 7, utf8=True)
        assert np.array_equal(host(got.valid), want), L
        ascii_fr = golden_small[f"L{L}_frames7"]
        got = batch.unpack_batch(dev(ascii_fr, cuda), 7, utf8=True)
        assert (host(got.valid) == 1).all() and (host(got.ok) == 1).all(), L


@pytest.mark.slow
def test_fused_full_size_mtu(cuda):
    """1M x 1472 B synthetic ASCII frames (the bench's decode leg): all valid,
    all checksums good; one injected bad byte per 4096 frames is found."""
    import torch
    n, L = 1 << 20, 1472
    tab, pay = batch.synth_batch(n, L, 0x5EED0003, device=cuda)
    fr, _ = batch.pack_batch(tab, pay, 7)
    d = batch.unpack_batch(fr, 7, utf8=True)
    assert bool((d.valid == 1).all()) and bool((d.ok == 1).all())
    idx = torch.arange(0, n, 4096, device=cuda)
    col = 7 + (idx % L)
    fr[idx, col] = 0xFF
    d = batch.unpack_batch(fr, 7, utf8=True)
    bad = (d.valid == 0).nonzero().flatten()
    assert torch.equal(bad, idx)


def _expect_checked(flat, off, H):
    """Per-frame rule of the checked decode: a frame whose own offsets are
    decreasing or past the buffer is rejected (ok 4, zero fields, valid 0);
    every other frame decodes as the oracle decodes it alone."""
    n = len(off) - 1
    out = {k: np.zeros(n, dt) for k, dt in (("seq", np.uint16), ("ack", np.uint16), ("flags", np.uint8),
                                            ("ok", np.uint8), ("csum", np.uint16), ("valid", np.uint8))}
    for i in range(n):
        fo, fe = int(off[i]), int(off[i + 1])
        if fo > fe or fe > len(flat) or fo < 0:
            out["ok"][i] = _native.OK_BAD_OFFSETS
            continue
        one = np.array([0, fe - fo], np.int64)
        seg = flat[fo:fe]
        for k, v in zip(("seq", "ack", "flags", "ok", "csum"), codec_np.decode_varlen(seg, one, H)):
            out[k][i] = v[0]
        out["valid"][i] = codec_np.utf8_valid(seg, one, H)[0]
    return out


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_inner_offsets_outside_the_tile(cuda, H):
    """Offsets that go backwards inside a tile: the frame before the drop is
    valid (its own pair is in order and inside the buffer) although it reaches
    past the tile's last offset; the frame at the drop is rejected.  Every
    kernel form (small tiles, vector, LDS tiles) must decode the valid one from
    HBM, not reject it."""
    rng = np.random.default_rng(4040 + H)
    hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
    frames = [hdr + b for b in _near_utf8(rng, 6000, 0, 6)]
    flat, off = _pack(frames)
    off = off.copy()
    for k in (3, 700, 2049, 4100):
        off[k + 1] = off[k + 1 + 400]   # frame k spans 400 frames' bytes; frame k + 1 goes backwards
    want = _expect_checked(flat, off, H)
    assert (want["ok"] == _native.OK_BAD_OFFSETS).sum() >= 4
    d_flat, d_off = dev(flat, cuda), dev(off, cuda)
    for hint in (0, 16, 64, 200, 1600):
        got = _varlen_decode(d_flat, len(flat), d_off, len(frames), hint, H, True)
        for k in want:
            assert np.array_equal(got[k], want[k]), (k, hint)


def test_dedup_small_and_two_pass_forms_agree(cuda):
    """The one-launch small-frame dedup and the two-pass form (rudpx_tune 62 = 0)
    give the reference proxy's flags (window semantics of proxy.py:90, :92-94)
    on short datagrams with many repeats, empty ones and rejected offsets, at
    windows 1, 500 and 1024 (the one-launch form's limit) and past it (4096)."""
    import contextlib
    import ctypes
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(62)
    pool = [b"", bytes(5)] + [bytes(rng.integers(0, 256, int(rng.integers(1, 14)), dtype=np.uint8))
                              for _ in range(400)]
    seq = [pool[int(k)] for k in rng.integers(0, len(pool), 30000)]
    flat, off = _pack(seq)
    bad = off.copy()
    bad[1000] = bad[1001] + 1
    bad[-1] = len(flat) + 3

    @contextlib.contextmanager
    def small(v):
        old = lib.rudpx_tune(62, v)
        try:
            yield
        finally:
            lib.rudpx_tune(62, old)
    for window in (1, 500, 1024, 4096):
        canon = [f if f else bytes(5) for f in seq]
        last, want = {}, []
        for i, k in enumerate(canon):
            want.append(int(k in last and last[k] >= i - window))
            last[k] = i
        for form in (1, 0):
            with small(form):
                got = batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(off, cuda), window=window)
                assert host(got).tolist() == want, (window, form)
                g2 = host(batch.detect_retransmissions(dev(flat, cuda), frame_off=dev(bad, cuda), window=window,
                                                       check=False))
                assert g2[1000] == _native.DUP_BAD_OFFSETS and g2[-1] == _native.DUP_BAD_OFFSETS, (window, form)
                assert int((g2 == _native.DUP_BAD_OFFSETS).sum()) == 2


@pytest.mark.parametrize("H", [5, 7])
def test_fused_multibyte_text_every_corruption_offset(cuda, H):
    """Valid multi-byte text (2-, 3- and 4-byte characters across every 16-B
    chunk boundary) takes the table check on every chunk: all valid; then one
    byte per frame replaced at every payload offset, with bytes that make each
    error class (stray continuation, truncated lead, overlong, surrogate, past
    U+10FFFF): the answer equals Python's strict decoder, fixed-length tiles
    and packed tiles alike."""
    import torch
    text = ("é中😀aßЖ€𝄞" * 200).encode()
    L = 1472
    body = text[:L]
    while True:  # cut on a character boundary, pad with ASCII
        try:
            body.decode()
            break
        except UnicodeDecodeError:
            body = body[:-1]
    body = body + b"x" * (L - len(body))
    subs = [0x80, 0xBF, 0xC0, 0xC1, 0xE0, 0xED, 0xF0, 0xF4, 0xF5, 0xFF, 0x41]
    rows = [body]
    for k in range(L):
        b = bytearray(body)
        b[k] = subs[k % len(subs)]
        rows.append(bytes(b))
    hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
    fr = np.frombuffer(b"".join(hdr + r for r in rows), np.uint8).reshape(len(rows), L + H)
    off = np.arange(len(rows) + 1, dtype=np.int64) * (L + H)
    want = codec_np.utf8_valid(fr.reshape(-1), off, H)
    assert want[0] == 1 and 0 < want.mean() < 1
    got = batch.unpack_batch(dev(fr, cuda), H, utf8=True)
    assert np.array_equal(host(got.valid), want)
    for hint in (0, 200, 1600):
        g = _varlen_decode(dev(fr.reshape(-1), cuda), fr.size, dev(off, cuda), len(rows), hint, H, True)
        assert np.array_equal(g["valid"], want), hint
    assert bool((batch.validate_utf8(dev(fr, cuda), H) == torch.from_numpy(want).to(cuda)).all())


@pytest.mark.parametrize("blocks", [1, 0])
def test_varlen_tile_block_sums_and_chunk_sums_agree(cuda, blocks):
    """The varlen decode tile's two sum forms (128-B block sums from phase 1,
    rudpx_tune 63 = 1, the default; chunk by chunk, 0) on ragged frames of
    0-3000 B with near-UTF-8 bodies, the fused check on and off: equal to the
    oracle's fields and Python's strict decoder."""
    import ctypes
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old = lib.rudpx_tune(63, blocks)
    try:
        rng = np.random.default_rng(63 + blocks)
        for H in (5, 7):
            hdr = b"\x12\x34\x00\x00\x80" + (b"\xbe\xef" if H == 7 else b"")
            frames = []
            for b in _near_utf8(rng, 3000):
                L = int(rng.integers(0, 3000))
                frames.append(hdr + ((b or b"A") * (L // max(1, len(b)) + 1))[:L])
            flat, off = _pack(frames)
            want = codec_np.decode_varlen(flat, off, H)
            want_v = codec_np.utf8_valid(flat, off, H)
            for hint in (200, 1600, 3000):
                got = _varlen_decode(dev(flat, cuda), len(flat), dev(off, cuda), len(frames), hint, H, True)
                for k, w in zip(("seq", "ack", "flags", "ok", "csum"), want):
                    assert np.array_equal(got[k], w), (k, H, hint)
                assert np.array_equal(got["valid"], want_v), (H, hint)
    finally:
        lib.rudpx_tune(63, old)


@pytest.mark.parametrize("single", [1, 0])
def test_small_encode_one_tile_batches(cuda, single):
    """A checked small-frame encode of at most 1024 packets (a recvmmsg batch)
    runs as one launch with no scan pass (rudpx_tune 64 = 1, the default):
    frames, offsets and checksums equal the oracle's for 1..1024 packets of
    1-4 byte payloads, and every argument check still reports (lengths past
    65535, a payload size that disagrees, a frame buffer too small)."""
    import ctypes
    import torch
    from oracle import synth
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old = lib.rudpx_tune(64, single)
    try:
        rng = np.random.default_rng(64 + single)
        for n in (1, 7, 255, 1000, 1024):
            lens = rng.integers(1, 5, n).astype(np.int32)
            pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
            seq, ack, flags, _ = synth.synth(n, 0, n, 0)
            tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
            pays = [bytes(pay[o:o + k]) for o, k in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)]
            for H in (5, 7):
                want, off, cs = codec_np.encode_varlen(seq, ack, flags, pays, H)
                res = batch.pack_batch_varlen(tab, dev(pay, cuda), dev(lens, cuda), H, want_csum=True)
                assert np.array_equal(host(res.frames), want), (n, H)
                assert np.array_equal(host(res.frame_off), off) and np.array_equal(host(res.csum), cs), (n, H)
        n = 600
        lens = np.ones(n, np.int32)
        z16, z8 = dev(np.zeros(n, np.uint16), cuda), dev(np.zeros(n, np.uint8), cuda)
        with pytest.raises(ValueError, match="sum"):
            batch.pack_batch_varlen((z16, z16, z8), dev(np.zeros(n + 1, np.uint8), cuda), dev(lens, cuda))
        big = lens.copy()
        big[17] = 70000
        with pytest.raises(ValueError, match="65535"):
            batch.pack_batch_varlen((z16, z16, z8), dev(np.zeros(n, np.uint8), cuda), dev(big, cuda))
        with pytest.raises(ValueError, match="too small"):
            batch.pack_batch_varlen((z16, z16, z8), dev(np.zeros(n, np.uint8), cuda), dev(lens, cuda),
                                    out=torch.empty(n * 6 - 1, dtype=torch.uint8, device=cuda))
    finally:
        lib.rudpx_tune(64, old)


@pytest.mark.parametrize("L", [32, 48, 64, 96, 160, 1472])
@pytest.mark.parametrize("H", [5, 7])
def test_fixed_fused_sequences_across_frame_edges(cuda, L, H):
    """The fixed-length tile judges a wave's frames as one stream: payloads of
    valid multi-byte text cut at random points (a sequence left open at the
    payload's end, continuations at its start), lone lead / continuation bytes
    at the first and last payload bytes, and a ragged last tile (waves with
    fewer or no frames), against Python's strict decoder."""
    rng = np.random.default_rng(7000 + 10 * L + H)
    n = 3 * 256 + 37
    chars = "é中😀aßЖ€𝄞"
    bodies = []
    for i in range(n):
        s = int(rng.integers(0, len(chars)))
        t = (chars[s:] + chars * (L // 4 + 2)).encode()
        cut = L
        while True:  # the longest prefix of at most L bytes that ends on a character boundary
            try:
                t[:cut].decode()
                break
            except UnicodeDecodeError:
                cut -= 1
        b = bytearray(t[:cut] + b"x" * (L - cut))
        kind = i % 5
        if kind == 1:
            b[-1] = int(rng.choice([0xC3, 0xE4, 0xF0, 0xF4]))   # a lead left open at the end
        elif kind == 2:
            b[0] = int(rng.choice([0x80, 0xA0, 0xBF]))          # a continuation first
        elif kind == 3:
            b[int(rng.integers(0, L))] = int(rng.integers(0x80, 0x100))
        bodies.append(bytes(b))
    hdr = b"\xe4\xb8\x00\xf0\x80" + (b"\xc3\xa9" if H == 7 else b"")  # header bytes that look like UTF-8
    fr = np.frombuffer(b"".join(hdr + x for x in bodies), np.uint8).reshape(n, L + H)
    off = np.arange(n + 1, dtype=np.int64) * (L + H)
    want = codec_np.utf8_valid(fr.reshape(-1), off, H)
    assert 0.1 < want.mean() < 0.9
    for copy in (False, True):
        got = batch.unpack_batch(dev(fr, cuda), H, copy_payload=copy, utf8=True)
        assert np.array_equal(host(got.valid), want), copy


@pytest.mark.parametrize("L", [1024, 1472, 2048])
@pytest.mark.parametrize("H", [5, 7])
def test_fused_tile_high_bits_after_an_ascii_start(cuda, L, H):
    """The 16-lane decode tile sums a payload's first 512 B (two window rounds)
    and tests them for high bits: with one, the sums and the UTF-8 check share
    one pass over the windows; with none, the plain sums loop finishes the
    payload and a high bit it meets sends the wave to the separate window check.
    Frames with an ASCII start of every length around that edge, then valid
    multi-byte text, a corrupted byte, a truncated sequence or more ASCII, in
    every mix within a wave: checksums verify, fields equal the encode's inputs
    and valid equals Python's strict decoder."""
    import torch
    rng = np.random.default_rng(L * 10 + H)
    text = ("é中😀aßЖ€𝄞" * 400).encode()
    bodies = []
    for prefix in (0, 1, 15, 16, 100, 495, 496, 500, 511, 512, 513, 527, 528, 700, L - 17, L - 4, L - 1, L):
        for kind in range(5):
            tail = text[:L - prefix]
            b = bytearray(b"a" * prefix + tail)
            if kind == 1 and len(tail):  # a corrupted byte in the tail
                b[prefix + int(rng.integers(0, len(tail)))] = int(rng.choice([0x80, 0xC0, 0xED, 0xF5, 0xFF]))
            elif kind == 2 and prefix < L:  # a lead byte as the payload's last
                b[-1] = 0xE4
            elif kind == 3:  # all ASCII
                b = bytearray(b"a" * L)
            elif kind == 4 and prefix < L:  # one 2-byte character at the very end
                b[-2:] = "é".encode()
            bodies.append(bytes(b[:L]))
    n = len(bodies)
    order = rng.permutation(n)  # every mix of kinds within a wave's 4 frames
    pay = np.frombuffer(b"".join(bodies[i] for i in order), np.uint8).reshape(n, L)
    seq = rng.integers(0, 1 << 16, n).astype(np.uint16)
    ack = rng.integers(0, 1 << 16, n).astype(np.uint16)
    flags = rng.integers(0, 256, n).astype(np.uint8)
    fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda), H, want_csum=True)
    off = np.arange(n + 1, dtype=np.int64) * (L + H)
    want = codec_np.utf8_valid(host(fr).reshape(-1), off, H)
    assert 0.1 < want.mean() < 0.9
    for copy in (False, True):
        d = batch.unpack_batch(fr, H, csum=cs if H == 5 else None, copy_payload=copy, utf8=True)
        assert np.array_equal(host(d.valid), want), copy
        assert (host(d.ok) == 1).all(), copy
        assert np.array_equal(host(d.seq), seq) and np.array_equal(host(d.ack), ack)
        assert np.array_equal(host(d.flags), flags)
        if copy:
            assert torch.equal(d.payload, dev(pay, cuda))
    assert np.array_equal(host(batch.validate_utf8(fr, H)), want)


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_tile_windows_text_of_any_length(cuda, H):
    """Packed frames at hints of 769-1536 B take the varlen decode tile at 16
    lanes a frame, which checks each payload over payload-aligned windows (the
    last one masked to the payload) with the bytes before a window handed
    across the DPP row.  Text payloads of every length (0-3000 B: whole
    windows and every remainder), with a corrupted byte, a truncated last
    character or a lead byte at the very end; the answer equals Python's
    strict decoder at hints 1000 and 1472 and the fields agree with the
    checksum-only decode."""
    rng = np.random.default_rng(1600 + H)
    text = ("é中😀aßЖ€𝄞" * 600).encode()
    rows = []
    for k in range(3000):
        L = int(rng.integers(0, 3001)) if k % 3 else int(rng.integers(1400, 1560))
        body = bytearray(text[:L].decode("utf-8", "ignore").encode())
        body += b"q" * (L - len(body))
        kind = k % 5
        if kind == 1 and L:
            body[int(rng.integers(0, L))] = int(rng.choice([0x80, 0xBF, 0xC1, 0xE0, 0xED, 0xF4, 0xF5, 0xFF]))
        elif kind == 2 and L >= 2:
            body[-1] = 0xF0
        elif kind == 3 and L >= 3:
            body[-3:] = "€".encode()[:2] + b"q"  # a 3-byte character cut to 2, then ASCII
        rows.append(bytes(body))
    hdr = b"\x12\x34\x56\x78\x40" + (b"\x00\x00" if H == 7 else b"")
    frames = [hdr + r for r in rows]
    flat = np.frombuffer(b"".join(frames), np.uint8)
    off = np.zeros(len(frames) + 1, np.int64)
    off[1:] = np.cumsum([len(f) for f in frames])
    want = codec_np.utf8_valid(flat, off, H)
    assert 0.2 < want.mean() < 0.9
    d_flat, d_off = dev(flat, cuda), dev(off, cuda)
    for hint in (1000, 1472):
        g = _varlen_decode(d_flat, flat.size, d_off, len(frames), hint, H, True)
        assert np.array_equal(g["valid"], want), hint
        plain = _varlen_decode(d_flat, flat.size, d_off, len(frames), hint, H, False)
        for k in plain:
            assert np.array_equal(g[k], plain[k]), (hint, k)
    assert np.array_equal(host(batch.validate_utf8(d_flat, H, frame_off=d_off)), want)
