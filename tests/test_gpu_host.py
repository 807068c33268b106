"""Host-memory entry points of ABI 7: the reference's real boundary is a UDP
socket buffer in host memory (utils/reliableUDP.py:61, :67, :118), so a batch
starts and ends there and is staged through the GPU in chunks.

- rudp_decode_host(h_valid): fixed-length frames, parse + verify + get_payload()'s
  strict UTF-8 (utils/packet.py:68-73) in the decode pass;
- rudp_decode_varlen_host: packed frames + offsets (a recvmmsg batch), every
  frame's offsets checked as rudp_decode_varlen_utf8 checks them;
- rudp_encode_varlen_host: packed payloads -> packed frames (a sendmmsg batch).

Pinned by the reference's own outputs (tests/golden/varlen.npz: frames the
reference framed, its 333 get_payload() outcomes; frames_small.npz) and, for
generated shapes, by the device-resident entry points on the same bytes and
the oracle restatement (oracle/codec_np).
"""
import ctypes

import numpy as np
import torch
import pytest

from conftest import small_lengths, split_by_lengths
from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu


class _Knobs:
    """Diagnostics-build knobs for one test (small staging slots: many chunks)."""

    def __init__(self, **kv):
        self.kv = kv
        self.old = {}

    def __enter__(self):
        lib = _native.tools_lib()
        keys = {"slots": 8, "stage_mb": 9, "min_chunks": 71}
        for k, v in self.kv.items():
            self.old[keys[k]] = lib.rudpx_tune(keys[k], v)
        return lib

    def __exit__(self, *exc):
        lib = _native.tools_lib(activate=False)
        for k, v in self.old.items():
            lib.rudpx_tune(k, v)
        _native.use_product()


def _device_varlen(cuda, flat, off, H, csum=None):
    """rudp_decode_varlen_utf8 of the same bytes, device-resident: the reference result."""
    import torch
    d = batch.unpack_batch_varlen(torch.from_numpy(flat.copy()).to(cuda), torch.from_numpy(off.copy()).to(cuda), H,
                                  csum=None if csum is None else torch.from_numpy(csum.copy()).to(cuda),
                                  check=False, utf8=True)
    return {k: getattr(d, k).cpu().numpy() for k in ("seq", "ack", "flags", "ok", "csum", "valid")}


def _host_fields(d):
    return {k: np.asarray(getattr(d, k)) for k in ("seq", "ack", "flags", "ok", "csum", "valid")}


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_host_decode_reference_get_payload(cuda, golden_varlen, H):
    """The reference's 333 get_payload() outcomes through the host entry, and
    the oracle's fields for the same frames."""
    g = golden_varlen
    bodies, _ = split_by_lengths(g["utf8_bodies"], g["utf8_lengths"])
    hdr = b"\x00\x01\x00\x02\x40" + (b"\x12\x34" if H == 7 else b"")
    frames = [hdr + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8).copy()
    d = batch.unpack_batch_varlen(flat, off, H, utf8=True)
    assert np.array_equal(d.valid, g["utf8_valid"])
    want = codec_np.decode_varlen(flat, off, H)
    for k, w in zip(("seq", "ack", "flags", "ok", "csum"), want):
        assert np.array_equal(getattr(d, k), w), k
    assert int(d.status[0]) == 0
    start, end = d.payload
    assert all(bytes(flat[s:e]) == b for s, e, b in zip(start, end, bodies))


@pytest.mark.parametrize("H", [5, 7])
def test_varlen_host_decode_reference_frames(cuda, golden_varlen, H):
    """Frames the reference itself framed (varlen.npz frames5 / frames7): every
    one verifies and gives back the header the reference was given."""
    g = golden_varlen
    flat = g[f"frames{H}"]
    off = np.concatenate([[0], np.cumsum(g["lengths"].astype(np.int64) + H)]).astype(np.int64)
    d = batch.unpack_batch_varlen(flat, off, H, csum=g["csum"] if H == 5 else None, utf8=True)
    assert (d.ok == 1).all()
    assert np.array_equal(d.seq, g["seq"]) and np.array_equal(d.ack, g["ack"])
    assert np.array_equal(d.flags, g["flags"])
    assert np.array_equal(d.csum, g["csum"])
    assert np.array_equal(d.valid, codec_np.utf8_valid(flat, off, H))


def test_fixed_host_decode_utf8_reference_frames(cuda, golden_small):
    """unpack_batch(numpy, utf8=True) on the reference-framed batches of every
    payload length in frames_small.npz, both layouts."""
    for L in small_lengths(golden_small):
        for H in (5, 7):
            fr = golden_small[f"L{L}_frames{H}"]
            cs = golden_small[f"L{L}_csum"]
            d = batch.unpack_batch(fr, H, csum=cs if H == 5 else None, utf8=True)
            off = np.arange(fr.shape[0] + 1, dtype=np.int64) * fr.shape[1]
            assert np.array_equal(d.valid, codec_np.utf8_valid(fr.reshape(-1), off, H)), (L, H)
            assert (d.ok == 1).all(), (L, H)
            assert np.array_equal(d.seq, golden_small[f"L{L}_seq"]), (L, H)
            assert np.array_equal(d.ack, golden_small[f"L{L}_ack"]), (L, H)
            assert np.array_equal(d.flags, golden_small[f"L{L}_flags"]), (L, H)


@pytest.mark.parametrize("L", [64, 1472])
def test_fixed_host_decode_utf8_many_chunks(cuda, L):
    """Fixed-length host decode with the UTF-8 answer over many chunks (1-MiB
    slots): valid text, random bytes and corrupted frames mixed."""
    n = 3001 if L == 1472 else 40001
    rng = np.random.default_rng(L)
    seq, ack, flags, pay = synth.synth(0x77 + L, 0, n, L, ascii=True)
    pay = pay.copy()
    bad = rng.random(n) < 0.2
    pay[bad, rng.integers(0, L, int(bad.sum()))] = 0xC3  # a lone lead byte or a valid pair
    with _Knobs(stage_mb=1, slots=2):
        for H in (5, 7):
            fr, cs = codec_np.encode(seq, ack, flags, pay, H)
            fr = fr.copy()
            fr[7, H] ^= 0x40
            d = batch.unpack_batch(fr, H, csum=cs if H == 5 else None, utf8=True, copy_payload=True)
            off = np.arange(n + 1, dtype=np.int64) * (L + H)
            assert np.array_equal(d.valid, codec_np.utf8_valid(fr.reshape(-1), off, H)), H
            want = codec_np.decode(fr, H, cs if H == 5 else None)
            for k, w in zip(("seq", "ack", "flags", "ok", "csum"), want):
                assert np.array_equal(getattr(d, k), w), (k, H)
            assert d.ok[7] == 0
            assert np.array_equal(d.payload, fr[:, H:])


def _oracle_varlen(seq, ack, flags, lens, pay, H):
    """codec_np.encode per payload length (vectorized over the packets of one
    length), scattered back to back: (frames, frame_off, csum)."""
    lens = lens.astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens + H)])
    po = np.concatenate([[0], np.cumsum(lens)])
    flat = np.empty(int(off[-1]), np.uint8)
    cs = np.empty(len(lens), np.uint16)
    for L in np.unique(lens):
        idx = np.nonzero(lens == L)[0]
        p = pay[po[idx][:, None] + np.arange(L)[None, :]] if L else np.zeros((len(idx), 0), np.uint8)
        fr, c = codec_np.encode(seq[idx], ack[idx], flags[idx], p, H)
        flat[off[idx][:, None] + np.arange(L + H)[None, :]] = fr
        cs[idx] = c
    return flat, off, cs


def _ragged_frames(rng, n, H, hi):
    """Lengths uniform in [0, hi]; payloads cut from valid multi-byte text, so
    some end mid-character (invalid) and the rest are valid."""
    lens = rng.integers(0, hi + 1, n)
    seq, ack, flags = (rng.integers(0, 1 << 16, n).astype(np.uint16), rng.integers(0, 1 << 16, n).astype(np.uint16),
                       rng.integers(0, 256, n).astype(np.uint8))
    text = np.frombuffer(("é中a" * (hi // 2 + 8)).encode(), np.uint8)
    starts = rng.integers(0, 6, n)  # a start mid-character: invalid from the first byte
    pay = np.concatenate([text[s:s + k] for s, k in zip(starts, lens)]) if n else np.zeros(0, np.uint8)
    return _oracle_varlen(seq, ack, flags, lens, pay, H)


@pytest.mark.parametrize("hi,stage_mb", [(24, 1), (2944, 1), (2944, 128)])
def test_varlen_host_decode_equals_device(cuda, hi, stage_mb):
    """Packed host frames decoded chunk by chunk (1-MiB slots: a chunk per
    ~700 MTU frames) give exactly the device-resident decode of the same
    bytes, for the small-frame tiles (lengths to 24 B) and the MTU tiles."""
    rng = np.random.default_rng(hi + stage_mb)
    n = 30011 if hi > 100 else 150001
    with _Knobs(stage_mb=stage_mb, slots=3):
        for H in (5, 7):
            flat, off, cs = _ragged_frames(rng, n, H, hi)
            flat = flat.copy()
            flat[off[5] + H:off[6]] ^= 0x01  # a bad checksum (or an empty payload, untouched)
            d = batch.unpack_batch_varlen(flat, off, H, csum=cs if H == 5 else None, utf8=True)
            got, want = _host_fields(d), _device_varlen(cuda, flat, off, H, cs if H == 5 else None)
            for k in want:
                assert np.array_equal(got[k], want[k]), (k, H, hi)
            assert np.array_equal(d.valid, codec_np.utf8_valid(flat, off, H))


def test_varlen_host_decode_bad_offsets(cuda):
    """Offsets out of order, past the buffer, negative and pointing back into
    earlier frames: every frame gets the device-resident checked rule's answer
    (rejected frames ok = 4, valid = 0, nothing read), across chunk seams."""
    rng = np.random.default_rng(5)
    n, H = 20000, 7
    flat, off, _ = _ragged_frames(rng, n, H, 40)
    off = off.copy()
    nb = flat.size
    off[100] = off[99] - 1                 # frame 99 decreasing (frame 100 then spans more)
    off[5000] = nb + 17                    # past the buffer: frames 4999 and 5000 rejected
    off[7000] = -3                         # negative: a huge offset, rejected
    off[12000:12003] = off[10:13]          # valid pairs pointing back into earlier bytes
    with _Knobs(stage_mb=1, min_chunks=8):
        d = batch.unpack_batch_varlen(flat, off, H, utf8=True, check=False)
        with pytest.raises(ValueError, match="non-decreasing"):
            d.check()
        got, want = _host_fields(d), _device_varlen(cuda, flat, off, H)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    assert got["ok"][99] == 4 and got["ok"][4999] == 4 and got["ok"][5000] == 4 and got["ok"][6999] == 4
    assert got["ok"][12000] == 1 and got["ok"][12001] == 1


def test_varlen_host_decode_frame_over_slot(cuda):
    """One valid frame larger than a staging slot is refused, not truncated."""
    big = np.zeros(3 << 20, np.uint8)
    off = np.array([0, 7, big.size], np.int64)
    with _Knobs(stage_mb=1):
        with pytest.raises(ValueError, match="staging slot"):
            batch.unpack_batch_varlen(big, off, 7)


def test_varlen_host_decode_reuse(cuda, golden_varlen):
    """reuse= an earlier host result: its arrays take the outputs, same answers."""
    g = golden_varlen
    flat = g["frames7"]
    off = np.concatenate([[0], np.cumsum(g["lengths"].astype(np.int64) + 7)]).astype(np.int64)
    d1 = batch.unpack_batch_varlen(flat, off, 7, utf8=True)
    keep = {k: np.array(getattr(d1, k), copy=True) for k in ("seq", "ack", "flags", "ok", "csum", "valid")}
    d1.ok[:] = 9
    d2 = batch.unpack_batch_varlen(flat, off, 7, utf8=True, reuse=d1)
    assert d2.ok is d1.ok
    for k, v in keep.items():
        assert np.array_equal(getattr(d2, k), v), k
    with pytest.raises(ValueError, match="reuse"):
        batch.unpack_batch_varlen(flat, off, 7, reuse=d1)  # utf8 choice differs


def test_host_entry_outputs_are_pinned(cuda, golden_varlen):
    """The host entries' per-packet outputs are page-locked (the D2H runs at the
    link's rate): unpack_batch_varlen / pack_batch_varlen / unpack_batch on numpy."""
    g = golden_varlen
    flat = g["frames7"]
    off = np.concatenate([[0], np.cumsum(g["lengths"].astype(np.int64) + 7)]).astype(np.int64)
    d = batch.unpack_batch_varlen(flat, off, 7, utf8=True)
    for name in ("seq", "ack", "flags", "ok", "csum", "valid"):
        assert torch.from_numpy(getattr(d, name)).is_pinned(), name
    n = len(g["lengths"])
    enc = batch.pack_batch_varlen((d.seq, d.ack, d.flags), np.zeros(int(g["lengths"].sum()), np.uint8),
                                  g["lengths"].astype(np.int32), 7, want_csum=True)
    assert torch.from_numpy(enc.frame_off).is_pinned() and torch.from_numpy(enc.csum).is_pinned()
    assert enc.frame_off.shape == (n + 1,)


def test_varlen_host_decode_empty(cuda):
    d = batch.unpack_batch_varlen(np.zeros(0, np.uint8), np.zeros(1, np.int64), 7, utf8=True)
    assert d.ok.shape == (0,) and d.valid.shape == (0,)


@pytest.mark.parametrize("hi,stage_mb", [(9, 1), (2944, 1), (1472, 128)])
def test_varlen_host_encode_equals_oracle(cuda, golden_varlen, hi, stage_mb):
    """Packed host payloads framed chunk by chunk: frames, offsets and checksums
    equal the oracle's, and the reference's own varlen.npz frames."""
    g = golden_varlen
    for H in (5, 7):
        r = batch.pack_batch_varlen((g["seq"], g["ack"], g["flags"]), g["payload"], g["lengths"], H,
                                    want_csum=True)
        assert np.array_equal(r.frames, g[f"frames{H}"]) and np.array_equal(r.csum, g["csum"]), H
    rng = np.random.default_rng(hi)
    n = 40009 if hi > 100 else 300007
    lens = rng.integers(0, hi + 1, n).astype(np.int32)
    seq, ack = rng.integers(0, 1 << 16, n).astype(np.uint16), rng.integers(0, 1 << 16, n).astype(np.uint16)
    flags = rng.integers(0, 256, n).astype(np.uint8)
    pay = rng.integers(0, 256, int(lens.sum())).astype(np.uint8)
    with _Knobs(stage_mb=stage_mb, slots=2):
        for H in (5, 7):
            r = batch.pack_batch_varlen((seq, ack, flags), pay, lens, H, want_csum=True)
            want_fr, want_off, want_cs = _oracle_varlen(seq, ack, flags, lens, pay, H)
            assert np.array_equal(r.frame_off, want_off), H
            assert np.array_equal(r.frames, want_fr), H
            assert np.array_equal(r.csum, want_cs), H


def test_varlen_host_encode_rejects(cuda):
    """Lengths over 65535, a sum that is not the payload size and a frame buffer
    too small raise before any work; nothing is written."""
    n = 4
    tab = (np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8))
    with pytest.raises(ValueError, match="65535"):
        batch.pack_batch_varlen(tab, np.zeros(70000, np.uint8), np.array([1, 2, 3, 69994], np.int32), 7)
    with pytest.raises(ValueError, match="sum"):
        batch.pack_batch_varlen(tab, np.zeros(9, np.uint8), np.array([1, 2, 3, 4], np.int32), 7)
    out = np.full(10, 0xAB, np.uint8)
    with pytest.raises(ValueError, match="too small"):
        batch.pack_batch_varlen(tab, np.zeros(10, np.uint8), np.array([1, 2, 3, 4], np.int32), 7, out=out)
    assert (out == 0xAB).all()
    # the C entry checks the same before any work (a caller that skips the Python checks)
    lens = np.array([1, 2, 3, 70000], np.uint32)
    b = _native.RudpBatch(n=n, payload_len=1, reserved=0, seq=tab[0].ctypes.data, ack=tab[1].ctypes.data,
                          flags=tab[2].ctypes.data, payload=np.zeros(70006, np.uint8).ctypes.data,
                          len=lens.ctypes.data, payload_off=None)
    fr, fo = np.zeros(80000, np.uint8), np.zeros(n + 1, np.uint64)
    assert _native.lib().rudp_encode_varlen_host(ctypes.byref(b), 70006, fr.ctypes.data, fr.size, fo.ctypes.data,
                                                 None, 7, 0) == _native.EINVAL
    assert b"65535" in _native.lib().rudp_last_error()
    lens[3] = 100  # a sum that is not the payload's size: refused before any read of it
    assert _native.lib().rudp_encode_varlen_host(ctypes.byref(b), 70006, fr.ctypes.data, fr.size, fo.ctypes.data,
                                                 None, 7, 0) == _native.EINVAL
    assert b"sum" in _native.lib().rudp_last_error()
    assert not fr.any()


def test_varlen_host_decode_wide_descending_pair(cuda):
    """a descending pair whose offsets lie far apart inside a buffer
    larger than a staging slot (here 2.5 MiB -> 7 with 1-MiB slots) is rejected
    as the device-resident checked decode rejects it (ok = 4), not refused with
    RUDP_ENOTSUP; only a VALID frame over a slot is refused."""
    rng = np.random.default_rng(8)
    H = 7
    nb = 3 << 20
    flat = rng.integers(0x20, 0x7F, nb).astype(np.uint8)
    hi = 5 * (1 << 19)  # 2.5 MiB
    off = np.array([0, 7, 14, nb + 5, hi, hi + 7, hi + 14, 7, 14, 21], np.int64)
    with _Knobs(stage_mb=1, slots=2):
        d = batch.unpack_batch_varlen(flat, off, H, utf8=True, check=False)
        got, want = _host_fields(d), _device_varlen(cuda, flat, off, H)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    assert got["ok"][2] == 4 and got["ok"][3] == 4 and got["ok"][6] == 4
    assert got["ok"][4] != 4 and got["ok"][7] != 4


@pytest.mark.parametrize("direct", [1, 0])
def test_varlen_host_one_char_outputs_direct_or_copied(cuda, direct):
    """1-char datagrams through the host entries with the per-frame outputs
    stored by the kernels straight into the pinned arrays (knob 73 = 1, the
    product's form) or copied back from the slot (0), and through the raw C
    ABI into PAGEABLE numpy arrays (always copied): every form equals the
    device-resident decode / the oracle's frames, across many chunks."""
    rng = np.random.default_rng(73 + direct)
    n, H = 200003, 5
    lens = np.ones(n, np.int32)
    seq, ack = rng.integers(0, 1 << 16, n).astype(np.uint16), rng.integers(0, 1 << 16, n).astype(np.uint16)
    flags = rng.choice(np.array([0, 0x80, 0x20, 0xA0, 0x40, 0x60], np.uint8), n)
    pay = rng.integers(0x20, 0x80, n).astype(np.uint8)
    pay[::1001] = 0xC3  # a lone lead byte: invalid UTF-8
    want_fr, want_off, want_cs = _oracle_varlen(seq, ack, flags, lens, pay, H)
    with _Knobs(stage_mb=1, slots=3) as lib:
        lib.rudpx_tune(73, direct)
        try:
            r = batch.pack_batch_varlen((seq, ack, flags), pay, lens, H, want_csum=True)
            assert np.array_equal(r.frames, want_fr) and np.array_equal(r.frame_off, want_off)
            assert np.array_equal(r.csum, want_cs)
            d = batch.unpack_batch_varlen(want_fr, want_off, H, csum=want_cs, utf8=True)
            got = _host_fields(d)
            # pageable outputs through the raw entry (the copy path whatever the knob)
            pg = {k: np.full(n, 0xAB, dt) for k, dt in (("seq", np.uint16), ("ack", np.uint16), ("flags", np.uint8),
                                                        ("ok", np.uint8), ("csum", np.uint16), ("valid", np.uint8))}
            st = np.zeros(1, np.uint32)
            rc = lib.rudp_decode_varlen_host(want_fr.ctypes.data, want_fr.size, want_off.ctypes.data, 0, n,
                                             want_cs.ctypes.data, *[pg[k].ctypes.data for k in
                                                                    ("seq", "ack", "flags", "ok", "csum", "valid")],
                                             st.ctypes.data, H, 0)
            assert rc == 0
            fo = np.zeros(n + 1, np.uint64)
            cs = np.zeros(n, np.uint16)
            fr = np.zeros(want_fr.size, np.uint8)
            b = _native.RudpBatch(n=n, payload_len=1, reserved=0, seq=seq.ctypes.data, ack=ack.ctypes.data,
                                  flags=flags.ctypes.data, payload=pay.ctypes.data, len=lens.ctypes.data,
                                  payload_off=None)
            assert lib.rudp_encode_varlen_host(ctypes.byref(b), pay.size, fr.ctypes.data, fr.size, fo.ctypes.data,
                                               cs.ctypes.data, H, 0) == 0
        finally:
            lib.rudpx_tune(73, 1)
    want = _device_varlen(cuda, want_fr, want_off, H, want_cs)
    for k in want:
        assert np.array_equal(got[k], want[k]), (k, direct)
        assert np.array_equal(pg[k], want[k]), (k, direct)
    assert (got["ok"] == 1).all() and got["valid"].sum() == n - len(range(0, n, 1001))
    assert np.array_equal(fr, want_fr) and np.array_equal(fo.astype(np.int64), want_off)
    assert np.array_equal(cs, want_cs)


def _pinned(a):
    t = torch.empty(a.shape, dtype={np.uint8: torch.uint8, np.uint16: torch.uint16, np.int32: torch.int32,
                                    np.int64: torch.int64}[a.dtype.type], pin_memory=True)
    out = t.numpy()
    out[...] = a
    return out


@pytest.mark.parametrize("zero_copy", [1, 0])
def test_varlen_host_zero_copy_pinned_batches(cuda, zero_copy):
    """A recvmmsg / sendmmsg batch of 1-char datagrams whose every array is
    pinned host memory: one launch that reads and writes the host arrays over
    PCIe (knob 75 = 1, the product's form) or the slot pipeline (0).  Frames,
    offsets and checksums equal the oracle's; the decode's fields equal the
    device-resident decode of the same bytes, rejected offsets included."""
    rng = np.random.default_rng(75 + zero_copy)
    n, H = 300007, 5
    lens = rng.integers(0, 5, n).astype(np.int32)  # 0-4 B payloads (UTF-8 characters), mean ~2
    seq, ack = rng.integers(0, 1 << 16, n).astype(np.uint16), rng.integers(0, 1 << 16, n).astype(np.uint16)
    flags = rng.integers(0, 256, n).astype(np.uint8)
    pay = rng.integers(0, 256, int(lens.sum())).astype(np.uint8)
    want_fr, want_off, want_cs = _oracle_varlen(seq, ack, flags, lens, pay, H)
    p_seq, p_ack, p_flags, p_pay, p_lens = (_pinned(a) for a in (seq, ack, flags, pay, lens))
    p_fr = _pinned(np.zeros(want_fr.size + 64, np.uint8))[:want_fr.size]
    off = want_off.copy()
    # One decreasing pair: frame 999 is rejected; frame 1000 then starts a byte
    # early, is read and fails its checksum (RUDP_OK_BAD_CSUM).
    off[1000] = off[999] - 1
    off[5000] = want_fr.size + 9  # past the buffer: frames 4999 and 5000 rejected
    p_off = _pinned(off)
    with _Knobs() as lib:
        old = lib.rudpx_tune(75, zero_copy)
        try:
            r = batch.pack_batch_varlen((p_seq, p_ack, p_flags), p_pay, p_lens, H, want_csum=True, out=p_fr)
            assert np.array_equal(r.frames, want_fr) and np.array_equal(r.frame_off, want_off)
            assert np.array_equal(r.csum, want_cs)
            d = batch.unpack_batch_varlen(r.frames, p_off, H, csum=_pinned(want_cs), utf8=True, check=False)
            got = _host_fields(d)
            assert int(np.asarray(d.status)[0]) == 8  # RUDP_ST_OFFSETS: rejected frames in the batch
            clean = batch.unpack_batch_varlen(r.frames, _pinned(want_off), H, csum=_pinned(want_cs), utf8=True,
                                              check=False)
            assert int(np.asarray(clean.status)[0]) == 0 and (clean.ok == 1).all()
        finally:
            lib.rudpx_tune(75, old)
    want = _device_varlen(cuda, want_fr, off, H, want_cs)
    for k in want:
        assert np.array_equal(got[k], want[k]), (k, zero_copy)
    assert got["ok"][999] == 4 and got["ok"][1000] == 0 and got["ok"][4999] == 4 and got["ok"][5000] == 4
    assert (np.delete(got["ok"], [999, 1000, 4999, 5000]) == 1).all()


def test_varlen_host_zero_copy_rejects(cuda):
    """The zero-copy encode makes no host pass over the lengths: the device's
    checked encode judges the batch and its status comes back as the host
    checks' ValueErrors (a length over 65535, a sum that is not the payload's
    size, a frame buffer too small), with no frame byte written."""
    n, H = 100003, 5
    z16, z8 = _pinned(np.zeros(n, np.uint16)), _pinned(np.zeros(n, np.uint8))
    tab = (z16, z16, z8)
    cases = []
    big = np.ones(n, np.int32)
    big[n // 2] = 70000
    cases.append(("65535", big, int(big.sum()), int(big.sum()) + n * H))
    ones = np.ones(n, np.int32)
    cases.append(("sum", ones, n + 5, n + 5 + n * H))
    cases.append(("sum", ones, n - 5, n - 5 + n * H))
    cases.append(("too small", ones, n, n + n * H - 16))
    with _Knobs() as lib:
        old = lib.rudpx_tune(75, 1)
        try:
            for msg, lens, pb, cap in cases:
                out = _pinned(np.full(cap + 64, 0xAB, np.uint8))[:cap]
                with pytest.raises(ValueError, match=msg):
                    batch.pack_batch_varlen(tab, _pinned(np.zeros(pb + 16, np.uint8))[:pb], _pinned(lens), H,
                                            want_csum=True, out=out)
                assert (out == 0xAB).all(), msg
            # and a good batch through the same arrays after the refusals
            pay = _pinned(np.arange(n, dtype=np.uint8))
            out = _pinned(np.zeros(n + n * H + 64, np.uint8))[:n + n * H]
            r = batch.pack_batch_varlen(tab, pay, _pinned(ones), H, want_csum=True, out=out)
        finally:
            lib.rudpx_tune(75, old)
    want_fr, want_off, want_cs = _oracle_varlen(np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8),
                                                ones, np.arange(n, dtype=np.uint8), H)
    assert np.array_equal(r.frames, want_fr) and np.array_equal(r.frame_off, want_off)
    assert np.array_equal(r.csum, want_cs)
