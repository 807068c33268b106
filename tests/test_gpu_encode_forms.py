"""Encode tile kernel forms (LDS-DMA or register phase 1, prebuilt header
chunks, early header-table loads, LDS-scratch chunk builds) against the oracle.

Bit-exact: frames and checksum sideband equal oracle/codec_np.encode (the
restatement pinned to the reference utils/packet.py by tests/golden).
"""
import ctypes

import numpy as np
import pytest

from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu


def _lib():
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int
    return lib


def _encode(cuda, seq, ack, flags, pay, layout):
    import torch
    tab = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(cuda) for x in (seq, ack, flags))
    fr, cs = batch.pack_batch(tab, torch.from_numpy(pay).to(cuda), layout, want_csum=True)
    return fr.cpu().numpy(), cs.cpu().numpy()


def _with(lib, settings, fn):
    old = [(k, lib.rudpx_tune(k, v)) for k, v in settings]
    try:
        return fn()
    finally:
        for k, v in reversed(old):
            lib.rudpx_tune(k, v)


@pytest.mark.parametrize("L", [16, 64, 256, 1472])
def test_dma_phase1_vs_oracle(cuda, L):
    lib = _lib()
    for n in (1, 17, 1031):
        seq, ack, flags, pay = synth.synth(0x5C + L, n, n, L, ascii=False)
        for layout in (5, 7):
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            fr, cs = _with(lib, [(25, 1)], lambda: _encode(cuda, seq, ack, flags, pay, layout))
            assert np.array_equal(fr, want_fr), (L, n, layout)
            assert np.array_equal(cs, want_cs), (L, n, layout)


@pytest.mark.parametrize("L", [16, 32, 48, 64, 256, 1024, 1472, 4096])
def test_prebuilt_header_chunks_vs_oracle(cuda, L):
    """Encode phase 2 with header chunks prebuilt by the packet leaders
    (rudpx_tune 29), every tile size with T % 16 == 0, both store dealings,
    header-table loads before or after phase 1 (rudpx_tune 30)."""
    lib = _lib()
    for n in (1, 2, 15, 16, 17, 257, 1031):
        seq, ack, flags, pay = synth.synth(0x5D + L, n, n, L, ascii=False)
        for layout in (5, 7):
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            for tile in (0, 16, 32, 256):
                if tile and tile * L > 65536:
                    continue
                for align, early, scr in ((0, 0, 0), (1, 0, 0), (0, 1, 0), (-1, -1, 0), (0, 0, 1), (-1, -1, 1)):
                    fr, cs = _with(lib, [(29, 1), (2, tile), (23, align), (30, early), (37, scr)],
                                   lambda: _encode(cuda, seq, ack, flags, pay, layout))
                    assert np.array_equal(fr, want_fr), (L, n, layout, tile, align, early, scr)
                    assert np.array_equal(cs, want_cs), (L, n, layout, tile, align, early, scr)


# (key, values) of launch-policy knobs not covered elsewhere: encode nt load /
# store (0, 1), phase-1 loads in flight (3), XCD-contiguous tile order (5);
# decode lanes per packet (4); varlen lanes (15)
# and varlen tile geometry (17, 18).
_ENCODE_KNOBS = [(0, (0,)), (1, (0,)), (3, (2, 4)), (5, (1,))]


@pytest.mark.parametrize("L", [64, 256, 1472])
def test_encode_policy_knobs_vs_oracle(cuda, L):
    lib = _lib()
    n = 2053
    seq, ack, flags, pay = synth.synth(0x5E + L, 3, n, L, ascii=False)
    for layout in (5, 7):
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        for key, values in _ENCODE_KNOBS:
            for v in values:
                for dma in (1, 0):
                    fr, cs = _with(lib, [(key, v), (25, dma)],
                                   lambda: _encode(cuda, seq, ack, flags, pay, layout))
                    assert np.array_equal(fr, want_fr), (L, layout, key, v, dma)
                    assert np.array_equal(cs, want_cs), (L, layout, key, v, dma)


@pytest.mark.parametrize("L", [64, 1472])
def test_decode_and_varlen_policy_knobs_vs_oracle(cuda, L):
    import torch
    lib = _lib()
    n = 3001
    seq, ack, flags, pay = synth.synth(0x5F + L, 0, n, L, ascii=False)
    fr, _ = codec_np.encode(seq, ack, flags, pay, 7)
    fr[5, 9] ^= 0x10
    want = codec_np.decode(fr, 7)
    d_fr = torch.from_numpy(fr).to(cuda)
    for lg in (1, 2, 3, 4):
        if (1 << lg) > L // 16:
            continue
        for verify_tile in (1, 0):
            d = _with(lib, [(4, lg), (12, verify_tile)], lambda: batch.unpack_batch(d_fr, 7))
            for g, w in zip((d.seq, d.ack, d.flags, d.ok, d.csum), want[:5]):
                assert np.array_equal(g.cpu().numpy(), w), (L, lg, verify_tile)
    # varlen encode: lanes per packet and tile geometry
    lens = np.full(n, L, np.int32)
    lens[::7] = L // 2 + 3
    flat = np.concatenate([pay[i, :lens[i]] for i in range(n)])
    pays = [flat[int(a):int(b)].tobytes() for a, b in zip(np.concatenate([[0], np.cumsum(lens)[:-1]]),
                                                         np.cumsum(lens))]
    want_fr, want_off, _ = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    tab = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(cuda) for x in (seq, ack, flags))
    d_flat, d_lens = torch.from_numpy(flat).to(cuda), torch.from_numpy(lens).to(cuda)
    for settings in ([(15, 1)], [(15, 3)], [(17, 64)], [(18, 8192)], [(18, 32768)], [(17, 4), (18, 4096)]):
        res = _with(lib, settings, lambda: batch.pack_batch_varlen(tab, d_flat, d_lens, 7))
        assert np.array_equal(res.frames.cpu().numpy(), want_fr), (L, settings)
        assert np.array_equal(res.frame_off.cpu().numpy(), want_off), (L, settings)
