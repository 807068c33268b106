"""Fixed-length batches the fixed-length tiles do not take, on the tile kernels.

pack_batch / unpack_batch on ``[N, L]`` payloads / ``[N, L + H]`` frames take
the fixed-length encode and decode tiles only when L is a multiple of 16 and
every buffer is 16-B aligned.  The reference's own traffic is one character
per datagram (utils/reliableUDP.py:11, :60; framed by utils/packet.py:60-65,
:80-81, parsed by :16, :29-40, :68-73), so L = 1-4 is THE shape: those
batches (and any other L, and unaligned views) go through the varlen tile
kernels with implicit offsets (capi.hip encode_stride / rudp_decode_utf8,
VarlenArgs::stride) -- the small-frame tile under 16 B, the MTU tile above,
the per-packet vector kernel past 6 KiB -- with get_payload()'s strict UTF-8
in the same pass and a payload copy-out kernel.  Everything here is compared
byte for byte with the reference-generated goldens (tests/golden/
frames_small.npz) where they hold the length, and with oracle/codec_np.py.
"""
import ctypes

import numpy as np
import pytest

from conftest import small_lengths
from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu

LENGTHS = [1, 2, 3, 15, 17, 63, 100, 1471]
COUNTS = [1, 17, 1023, 1024, 1025, 5000]


def dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def host(t):
    return t.cpu().numpy()


def _view(a, shift, cuda):
    """A device copy of `a` starting `shift` elements into a larger allocation."""
    import torch
    a = np.ascontiguousarray(a)
    flat = a.reshape(-1)
    raw = torch.zeros(flat.size + shift + 16, dtype={np.uint8: torch.uint8, np.uint16: torch.uint16}[a.dtype.type],
                      device=cuda)
    v = raw[shift:shift + flat.size]
    v.copy_(torch.from_numpy(flat).to(cuda))
    return v.view(*a.shape) if a.ndim > 1 else v


def _decode_raw(frames_t, F, n, H, cuda, csum=None, pay_out=None, utf8=True):
    """rudp_decode_utf8 through the C ABI, output buffers filled with a marker first."""
    import torch
    out = {k: torch.full((n,), 0xAB, dtype=dt, device=cuda) for k, dt in
           (("seq", torch.uint16), ("ack", torch.uint16), ("flags", torch.uint8), ("ok", torch.uint8),
            ("csum", torch.uint16), ("valid", torch.uint8))}
    _native.check(_native.lib().rudp_decode_utf8(
        frames_t.data_ptr() if F else None, None, F, n, csum.data_ptr() if csum is not None else None,
        out["seq"].data_ptr(), out["ack"].data_ptr(), out["flags"].data_ptr(), out["ok"].data_ptr(),
        out["csum"].data_ptr(), pay_out.data_ptr() if pay_out is not None else None,
        out["valid"].data_ptr() if utf8 else None, H, 0, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return {k: host(v) for k, v in out.items()}


def _check_decode(got, frames, H, csum_in=None, utf8=True):
    seq, ack, flags, ok, cs, _ = codec_np.decode(frames, H, csum_in)
    n, F = frames.shape
    assert np.array_equal(got["seq"], seq) and np.array_equal(got["ack"], ack)
    assert np.array_equal(got["flags"], flags) and np.array_equal(got["ok"], ok)
    if F >= H:
        assert np.array_equal(got["csum"], cs)
    if utf8:
        off = np.arange(n + 1, dtype=np.int64) * F
        assert np.array_equal(got["valid"], codec_np.utf8_valid(frames.reshape(-1), off, H))


# ---------------------------------------------------------------- goldens
@pytest.mark.parametrize("layout", [5, 7])
def test_stride_goldens(cuda, golden_small, layout):
    """Every golden length that is not a multiple of 16 (0, 1, 2, 3, 15, 17, 31,
    100): frames equal the reference's to_byte(), the reference-framed batches
    decode to the fields the reference read back, with Python's strict-decoder
    answer for each (full-range payloads) and the payloads copied out."""
    for L in small_lengths(golden_small):
        if L % 16 == 0 and L:
            continue
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        fr, cs = batch.pack_batch((dev(g["seq"], cuda), dev(g["ack"], cuda), dev(g["flags"], cuda)),
                                  dev(g["payload"], cuda), layout, want_csum=True)
        assert np.array_equal(host(fr), g[f"frames{layout}"]), L
        assert np.array_equal(host(cs), g["csum"]), L
        full = g[f"full_frames{layout}"]
        ref = g[f"full_fields{layout}"]
        d = batch.unpack_batch(dev(full, cuda), layout, copy_payload=True, utf8=True)
        assert np.array_equal(host(d.seq), ref[:, 0]) and np.array_equal(host(d.ack), ref[:, 1]), L
        assert np.array_equal(host(d.flags), ref[:, 2]), L
        assert np.array_equal(host(d.payload), full[:, layout:]), L
        off = np.arange(full.shape[0] + 1, dtype=np.int64) * full.shape[1]
        assert np.array_equal(host(d.valid), codec_np.utf8_valid(full.reshape(-1), off, layout)), L
        assert (host(d.ok) == (1 if layout == 7 else 3)).all(), L


# ----------------------------------------------------------- vs the oracle
@pytest.mark.parametrize("L", LENGTHS)
def test_stride_vs_oracle(cuda, L):
    for n in COUNTS:
        seq, ack, flags, pay = synth.synth(0x5100 + L, 7 * n, n, L, ascii=n % 2 == 1)
        for layout in (5, 7):
            fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda), layout,
                                      want_csum=True)
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            assert np.array_equal(host(fr), want_fr), (L, n, layout)
            assert np.array_equal(host(cs), want_cs), (L, n, layout)
            d = batch.unpack_batch(fr, layout, copy_payload=True, utf8=True,
                                   csum=cs if layout == 5 else None)
            assert (host(d.ok) == 1).all(), (L, n, layout)
            assert np.array_equal(host(d.seq), seq) and np.array_equal(host(d.ack), ack)
            assert np.array_equal(host(d.flags), flags) and np.array_equal(host(d.payload), pay)
            off = np.arange(n + 1, dtype=np.int64) * (L + layout)
            assert np.array_equal(host(d.valid), codec_np.utf8_valid(want_fr.reshape(-1), off, layout))


@pytest.mark.parametrize("L", [1, 3, 100, 1471])
def test_stride_many_tiles(cuda, L):
    """Batches of many tiles (XCD-ordered, ragged last tile) with one corrupted frame
    per 997."""
    n = 300001 if L < 16 else 20011
    seq, ack, flags, pay = synth.synth(0x5200 + L, 0, n, L, ascii=False)
    for layout in (5, 7):
        fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda), layout,
                                  want_csum=True)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(host(fr), want_fr) and np.array_equal(host(cs), want_cs), (L, layout)
        bad = want_fr.copy()
        rows = np.arange(0, n, 997)
        bad[rows, (rows * 7) % (L + layout)] ^= 0x21
        got = _decode_raw(dev(bad, cuda), L + layout, n, layout, cuda, csum=dev(want_cs, cuda) if layout == 5 else None)
        _check_decode(got, bad, layout, want_cs if layout == 5 else None)
        assert (got["ok"][rows] == 0).all()


# ------------------------------------------------------- unaligned views
@pytest.mark.parametrize("L", [1, 3, 17, 100, 1024, 1472])
def test_stride_unaligned_views(cuda, L):
    """Payload, frames, header-table and copy-out buffers that are views at any
    byte offset (L = 1024 / 1472: multiples of 16 that miss the fixed tile only
    through their alignment).  Bytes outside the views are never written."""
    import torch
    n = 1031
    seq, ack, flags, pay = synth.synth(0x5300 + L, 11, n, L, ascii=False)
    for layout in (5, 7):
        F = L + layout
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        for ps, fs, ts in ((1, 0, 0), (0, 5, 1), (3, 13, 3), (8, 1, 0), (15, 7, 2)):
            pay_v = _view(pay, ps, cuda)
            tab = (_view(seq, ts, cuda), _view(ack, ts, cuda), _view(flags, ts, cuda))
            raw = torch.full((n * F + fs + 32,), 0x5A, dtype=torch.uint8, device=cuda)
            out = raw[fs:fs + n * F].view(n, F)
            fr, cs = batch.pack_batch(tab, pay_v, layout, out=out, want_csum=True)
            assert np.array_equal(host(fr), want_fr), (L, layout, ps, fs, ts)
            assert np.array_equal(host(cs), want_cs), (L, layout, ps, fs, ts)
            r = host(raw)
            assert (r[:fs] == 0x5A).all() and (r[fs + n * F:] == 0x5A).all(), (L, layout, ps, fs)
            # decode the misaligned frames, payloads copied to a misaligned view
            for os_ in (0, 9):
                praw = torch.full((n * L + os_ + 32,), 0x33, dtype=torch.uint8, device=cuda)
                pv = praw[os_:os_ + n * L]
                got = _decode_raw(out, F, n, layout, cuda, csum=cs if layout == 5 else None, pay_out=pv)
                _check_decode(got, want_fr, layout, want_cs if layout == 5 else None)
                assert (got["ok"] == 1).all()
                assert np.array_equal(host(pv).reshape(n, L), pay), (L, layout, fs, os_)
                pr = host(praw)
                assert (pr[:os_] == 0x33).all() and (pr[os_ + n * L:] == 0x33).all()


# ---------------------------------------------------------------- UTF-8
@pytest.mark.parametrize("L", [2, 3, 7, 100, 1471])
def test_stride_utf8_text(cuda, L):
    """Fixed-length payloads of multi-byte text (1-4 byte characters, some cut at the
    payload's end, some corrupted): the fused check equals Python's strict decoder."""
    rng = np.random.default_rng(L)
    n = 4099
    chars = "aé中😀߿ࠀ￿\U0010ffff"
    rows = []
    for i in range(n):
        s = "".join(chars[k] for k in rng.integers(0, len(chars), L)).encode()[:L]
        b = bytearray(s.ljust(L, b"z"))
        if i % 5 == 0:
            b[int(rng.integers(0, L))] = int(rng.integers(0x80, 0x100))
        rows.append(bytes(b))
    pay = np.frombuffer(b"".join(rows), np.uint8).reshape(n, L)
    seq, ack, flags, _ = synth.synth(0x5400 + L, 0, n, 0)
    for layout in (5, 7):
        fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda), layout,
                                  want_csum=True)
        want_fr, _ = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(host(fr), want_fr)
        d = batch.unpack_batch(fr, layout, utf8=True)
        off = np.arange(n + 1, dtype=np.int64) * (L + layout)
        want_valid = codec_np.utf8_valid(want_fr.reshape(-1), off, layout)
        assert 0 < want_valid.sum() < n
        assert np.array_equal(host(d.valid), want_valid), (L, layout)


# ------------------------------------------------------------- host path
@pytest.mark.parametrize("L", [1, 100])
def test_stride_host_staged(cuda, L):
    """numpy in, numpy out: rudp_encode_host / rudp_decode_host stage through the
    slot ring into the same stride kernels (copy-out and UTF-8 included)."""
    n = 70001
    seq, ack, flags, pay = synth.synth(0x5500 + L, 0, n, L, ascii=True)
    for layout in (5, 7):
        fr, cs = batch.pack_batch((seq, ack, flags), pay, layout, want_csum=True)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(fr, want_fr) and np.array_equal(cs, want_cs)
        d = batch.unpack_batch(fr, layout, csum=cs if layout == 5 else None, copy_payload=True, utf8=True)
        assert (d.ok == 1).all() and (d.valid == 1).all()
        assert np.array_equal(d.payload, pay) and np.array_equal(d.seq, seq)


def test_stride_header_only_and_short(cuda):
    """L = 0 (the final ACK / FIN|ACK frames, utils/reliableUDP.py:88-92, :156-161)
    and frames shorter than the header (ok = 2, truncated fields) at batch sizes
    that span several small-frame tiles."""
    n = 3000
    seq, ack, flags, _ = synth.synth(0x5600, 0, n, 0)
    for layout in (5, 7):
        fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)),
                                  dev(np.zeros((n, 0), np.uint8), cuda), layout, want_csum=True)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, np.zeros((n, 0), np.uint8), layout)
        assert np.array_equal(host(fr), want_fr) and np.array_equal(host(cs), want_cs)
        got = _decode_raw(fr, layout, n, layout, cuda, csum=cs if layout == 5 else None)
        _check_decode(got, want_fr, layout, want_cs if layout == 5 else None)
        assert (got["valid"] == 1).all()  # no payload: get_payload() returns None, never raises
        for F in range(1, layout):
            short = np.ascontiguousarray(want_fr[:, :F])
            got = _decode_raw(dev(short, cuda), F, n, layout, cuda)
            _check_decode(got, short, layout, utf8=False)
            assert (got["ok"] == 2).all()
