"""Checked varlen decode by byte spans (decode_varlen_span_kernel, rudpx_tune
65 = 1; span bytes rudpx_tune 66).

The reference parses each datagram on its own (utils/reliableUDP.py:118-123,
utils/packet.py:31-38, :73); a batch decode must give, frame for frame, what
the oracle restatement gives (oracle/codec_np.decode_varlen + utf8_valid), and
what the frame-tile form gives, whatever the lengths: ragged MTU-scale frames,
frames longer than the span budget (per-frame path), spans of many tiny frames
(more than the LDS holds), frames that do not start at byte 0, buffers larger
than the frames, and offsets out of order (the index pass flags them and the
launch checks frame by frame).
"""
import contextlib
import ctypes

import numpy as np
import pytest

from oracle import codec_np
from rudp import _native

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    import torch
    return torch.from_numpy(np.array(a, copy=True)).to(cuda)


@contextlib.contextmanager
def knobs(**kv):
    keys = {"span": 65, "span_bytes": 66}
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old = {k: lib.rudpx_tune(keys[k], v) for k, v in kv.items()}
    try:
        yield
    finally:
        for k, v in old.items():
            lib.rudpx_tune(keys[k], v)


def _decode(cuda, flat_bytes, off, n, hint, H, utf8, lim=None):
    import torch
    d_flat = dev(flat_bytes, cuda)
    d_off = dev(off, cuda)
    out = {k: torch.full((n,), 0xAB, dtype=dt, device=cuda) for k, dt in
           (("seq", torch.uint16), ("ack", torch.uint16), ("flags", torch.uint8), ("ok", torch.uint8),
            ("csum", torch.uint16), ("valid", torch.uint8))}
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    _native.check(_native.lib().rudp_decode_varlen_utf8(
        d_flat.data_ptr(), len(flat_bytes) if lim is None else lim, d_off.data_ptr(), hint, n, None,
        out["seq"].data_ptr(), out["ack"].data_ptr(), out["flags"].data_ptr(), out["ok"].data_ptr(),
        out["csum"].data_ptr(), out["valid"].data_ptr() if utf8 else None, status.data_ptr(), H, 0,
        torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    if not utf8:
        del got["valid"]
    return got, int(status.item())


def _want(flat, off, H, lim):
    """The oracle per frame: rejected pairs (decreasing, or past the buffer) read nothing."""
    n = len(off) - 1
    seq = np.zeros(n, np.uint16); ack = np.zeros(n, np.uint16); flags = np.zeros(n, np.uint8)
    ok = np.zeros(n, np.uint8); csum = np.zeros(n, np.uint16); valid = np.zeros(n, np.uint8)
    good = (off[:-1] <= off[1:]) & (off[1:] <= lim)
    idx = np.nonzero(good)[0]
    if len(idx):
        sub_frames = [bytes(flat[off[i]:off[i + 1]]) for i in idx]
        sflat = np.frombuffer(b"".join(sub_frames) + b"\x00", np.uint8)[:-1]
        soff = np.concatenate([[0], np.cumsum([len(f) for f in sub_frames])]).astype(np.int64)
        s, a, f, o, c = codec_np.decode_varlen(sflat, soff, H)
        seq[idx], ack[idx], flags[idx], ok[idx], csum[idx] = s, a, f, o, c
        valid[idx] = codec_np.utf8_valid(sflat, soff, H)
    ok[~good] = _native.OK_BAD_OFFSETS
    return {"seq": seq, "ack": ack, "flags": flags, "ok": ok, "csum": csum, "valid": valid}, bool((~good).any())


def _bodies(rng, lens, text_frac=0.3):
    """ASCII bodies, some with valid multi-byte text, some with a stray high byte."""
    out = []
    text = ("é中😀aßЖ€" * 800).encode()
    for L in lens:
        r = rng.random()
        if r < text_frac:
            b = text[:L]
            while True:
                try:
                    b.decode()
                    break
                except UnicodeDecodeError:
                    b = b[:-1]
            b = b + b"y" * (L - len(b))
        else:
            b = bytearray(rng.integers(0x20, 0x7F, L, dtype=np.uint8).tobytes())
            if L and r > 0.85:
                b[int(rng.integers(0, L))] = int(rng.integers(0x80, 0x100))
            b = bytes(b)
        out.append(b)
    return out


def _frames(rng, lens, H):
    hdrs = rng.integers(0, 256, (len(lens), H), dtype=np.uint8)
    return [hdrs[i].tobytes() + b for i, b in enumerate(_bodies(rng, lens))]


def _check(cuda, frames, off, H, hints, lim=None, lead=0, slack=0):
    flat = np.frombuffer(bytes(lead) + b"".join(frames) + bytes(slack) + b"\x00", np.uint8)[:-1]
    lim = len(flat) if lim is None else lim
    want, any_bad = _want(flat, off, H, lim)
    for hint in hints:
        for span in (1, 0):
            with knobs(span=span):
                got, st = _decode(cuda, flat, off, len(off) - 1, hint, H, True, lim)
            for k in want:
                assert np.array_equal(got[k], want[k]), (k, hint, span, np.nonzero(got[k] != want[k])[0][:5])
            assert (st != 0) == any_bad, (st, hint, span)
            with knobs(span=span):
                plain, _ = _decode(cuda, flat, off, len(off) - 1, hint, H, False, lim)
            for k in plain:
                assert np.array_equal(plain[k], want[k]), (k, hint, span, "plain")


def _offsets(frames, lead=0):
    return (lead + np.concatenate([[0], np.cumsum([len(f) for f in frames])])).astype(np.int64)


@pytest.mark.parametrize("H", [5, 7])
@pytest.mark.parametrize("span_bytes", [4096, 24576])
def test_span_decode_ragged(cuda, H, span_bytes):
    """Lengths uniform in [0, 2944] (the BASELINE ragged shape, 20000 frames),
    small and default spans, hints 256 / 1472 / 3000."""
    rng = np.random.default_rng(6500 + H + span_bytes)
    frames = _frames(rng, rng.integers(0, 2945, 20000), H)
    with knobs(span_bytes=span_bytes):
        _check(cuda, frames, _offsets(frames), H, (256, 1472, 3000))


@pytest.mark.parametrize("H", [5, 7])
def test_span_decode_edges(cuda, H):
    """Frames longer than the span budget (per-frame path inside the launch),
    runs of header-only and empty frames (more frames per span than the LDS
    holds), frames starting past byte 0 and a buffer larger than the frames."""
    rng = np.random.default_rng(6600 + H)
    lens = list(rng.integers(0, 3000, 3000))
    lens[100:110] = [20000, 9000, 0, 0, 30000, 1, 2, 3, 4, 5]
    lens[500:1500] = [0] * 1000                     # 1000 header-only frames: > 128 per 4 KiB span
    lens[2000:2300] = list(rng.integers(0, 9, 300))
    frames = _frames(rng, lens, H)
    frames[600] = frames[600][:3]                   # shorter than the header
    frames[601] = b""
    with knobs(span_bytes=4096):
        _check(cuda, frames, _offsets(frames, lead=5), H, (256, 1472), lead=5, slack=777)
        _check(cuda, frames, _offsets(frames), H, (1472,))


@pytest.mark.parametrize("H", [5, 7])
def test_span_decode_offsets_out_of_order(cuda, H):
    """A decreasing pair and a frame past the buffer: the index pass flags
    the batch, every frame is checked on its own (rejections read nothing,
    valid frames decode)."""
    rng = np.random.default_rng(6700 + H)
    frames = _frames(rng, rng.integers(0, 2945, 4000), H)
    off = _offsets(frames)
    off[1000] = off[1001] + 3
    off[2000 + 1] = off[2000 + 1 + 300]
    with knobs(span_bytes=8192):
        _check(cuda, frames, off, H, (1472,))
    off2 = _offsets(frames)
    off2[-1] += 50                                   # the last frame reaches past the buffer
    with knobs(span_bytes=8192):
        _check(cuda, frames, off2, H, (1472,))


@pytest.mark.parametrize("H", [5, 7])
def test_huge_frames_fold_like_the_reference(cuda, H):
    """Frames far past 64 KiB (offsets are untrusted input, the reference's
    Packet parses any length): all-0xFF and random payloads of 0.2-3 MB, whose
    word sums pass 2^32 many times over, next to small frames; every kernel
    form (byte kernel misaligned, vector, frame tiles, spans) folds to the
    oracle's checksum."""
    import torch
    rng = np.random.default_rng(6800 + H)
    frames = [rng.integers(0, 256, H, dtype=np.uint8).tobytes() + b for b in
              (b"\xff" * 3_000_001, b"", bytes(rng.integers(0, 256, 200_000, dtype=np.uint8)), b"\xff" * 65536,
               b"abc", bytes(rng.integers(0, 256, 1_000_003, dtype=np.uint8)))]
    frames += _frames(rng, rng.integers(0, 2945, 40), H)
    off = _offsets(frames)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    want, _ = _want(flat, off, H, len(flat))
    for span in (1, 0):
        with knobs(span=span, span_bytes=8192):
            for hint in (0, 64, 200, 1472):
                got, st = _decode(cuda, flat, off, len(frames), hint, H, True)
                for k in want:
                    assert np.array_equal(got[k], want[k]), (k, hint, span)
    raw = torch.zeros(len(flat) + 32, dtype=torch.uint8, device=cuda)  # misaligned: the byte kernel
    mis = raw[3:3 + len(flat)]
    mis.copy_(torch.from_numpy(flat.copy()).to(cuda))
    out = {k: torch.zeros(len(frames), dtype=dt, device=cuda) for k, dt in
           (("seq", torch.uint16), ("ack", torch.uint16), ("flags", torch.uint8), ("ok", torch.uint8),
            ("csum", torch.uint16))}
    d_off = dev(off, cuda)
    _native.check(_native.lib().rudp_decode_varlen_checked(
        mis.data_ptr(), len(flat), d_off.data_ptr(), 1472, len(frames), None, out["seq"].data_ptr(),
        out["ack"].data_ptr(), out["flags"].data_ptr(), out["ok"].data_ptr(), out["csum"].data_ptr(), None, H, 0,
        torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    for k in out:
        assert np.array_equal(out[k].cpu().numpy(), want[k]), (k, "byte kernel")


@pytest.mark.parametrize("bal", [1, 0])
def test_encode_chunk_map_by_units(cuda, bal):
    """The varlen encode tile's chunk map built by output units spread over the
    lanes (rudpx_tune 67 = 1) or by G lanes per frame (0): ragged payloads of
    0-2944 B with runs of empty and short ones (the coded map's header-chunk
    classes and the frame walk), equal to the oracle's frames byte for byte."""
    import torch
    from oracle import synth
    from rudp import batch
    rng = np.random.default_rng(6900 + bal)
    n = 30000
    lens = rng.integers(0, 2945, n).astype(np.int32)
    lens[1000:1400] = rng.integers(0, 40, 400)
    lens[5000:5100] = 0
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(bal + 5, 0, n, 0)
    pays = [bytes(pay[o:o + k]) for o, k in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)]
    want, want_off, _ = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old = lib.rudpx_tune(67, bal)
    try:
        tab = tuple(torch.from_numpy(a).to(cuda) for a in (seq, ack, flags))
        res = batch.pack_batch_varlen(tab, torch.from_numpy(pay).to(cuda), torch.from_numpy(lens).to(cuda), "rudp7")
        assert np.array_equal(res.frames.cpu().numpy(), want)
        assert np.array_equal(res.frame_off.cpu().numpy(), want_off)
    finally:
        lib.rudpx_tune(67, old)


@pytest.mark.parametrize("r4", [1, 0])
@pytest.mark.parametrize("H", [5, 7])
def test_decode_tile_chunk_reads(cuda, r4, H):
    """The varlen decode tile's payload chunks read four at a time per lane
    (rudpx_tune 69 = 1) or one at a time (0): ragged, short, empty and out-of-order
    frames at the hints that pick 16, 8, 4 and 2 lanes per frame, equal to
    the oracle (fields, checksums, UTF-8 verdicts, rejections)."""
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old = lib.rudpx_tune(69, r4)
    try:
        rng = np.random.default_rng(6900 + 10 * r4 + H)
        lens = list(rng.integers(0, 2945, 6000))
        lens[100:400] = list(rng.integers(0, 30, 300))
        frames = _frames(rng, lens, H)
        off = _offsets(frames)
        off[3001] = off[3002] + 2          # a decreasing pair inside a tile
        flat = np.frombuffer(b"".join(frames), np.uint8)
        want, _ = _want(flat, off, H, len(flat))
        for hint in (200, 700, 1472, 3000):
            got, _ = _decode(cuda, flat, off, len(frames), hint, H, True)
            for k in want:
                assert np.array_equal(got[k], want[k]), (k, hint, r4)
    finally:
        lib.rudpx_tune(69, old)
