"""Randomized differential test of the fixed-length encode/decode kernels
against the oracle: random payload lengths (fast-path multiples of 16 and
arbitrary ones), batch sizes, layouts, buffer offsets and kernel knobs
(tile size, 64-B dealing, early table loads, header-chunk forms, LDS-DMA
or register phase 1, staged decode outputs).  Bit-exact, seeded."""
import ctypes

import numpy as np
import pytest

from oracle import codec_np, synth
from rudp import _native, batch

pytestmark = pytest.mark.gpu

# (key, choices) drawn per case; the first choice is the default
_KNOBS = {2: (0, 16, 32, 64, 128, 256), 23: (-1, 0, 1), 30: (-1, 0, 1, 2), 29: (1, 0), 37: (-1, 0, 1),
          25: (1, 0), 34: (1, 0), 12: (1, 0), 11: (1, 0), 5: (1, 0), 49: (0, 1), 48: (0, 256, 4096)}


def _lib():
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.rudpx_tune.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("seed", range(6))
def test_random_shapes_and_knobs_vs_oracle(cuda, seed):
    import torch
    lib = _lib()
    rng = np.random.default_rng(9000 + seed)
    for case in range(12):
        L = int(16 * rng.integers(1, 257)) if rng.random() < 0.8 else int(rng.integers(0, 700))
        n = int(rng.integers(1, 3000))
        layout = int(rng.choice([5, 7]))
        shift = int(rng.choice([0, 0, 16, 1]))  # payload/frames offset inside their buffers
        knobs = {k: int(rng.choice(v)) for k, v in _KNOBS.items()}
        if knobs[2] and knobs[2] * L > 65536:
            knobs[2] = 0
        seq, ack, flags, pay = synth.synth(int(rng.integers(1 << 30)), case, n, L, ascii=False)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        old = [(k, lib.rudpx_tune(k, v)) for k, v in knobs.items()]
        try:
            tab = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(cuda) for x in (seq, ack, flags))
            raw = torch.zeros(n * L + 64, dtype=torch.uint8, device=cuda)
            p = raw[shift:shift + n * L].view(n, L) if L else torch.empty((n, 0), dtype=torch.uint8, device=cuda)
            p.copy_(torch.from_numpy(pay).to(cuda))
            F = L + layout
            rawf = torch.zeros(n * F + 64, dtype=torch.uint8, device=cuda)
            fr = rawf[shift:shift + n * F].view(n, F)
            frames, cs = batch.pack_batch(tab, p, layout, out=fr, want_csum=True)
            ctx = (seed, case, L, n, layout, shift, knobs)
            assert np.array_equal(frames.cpu().numpy(), want_fr), ctx
            assert np.array_equal(cs.cpu().numpy(), want_cs), ctx
            # decode the frames back (corrupt one), verify-only and with copy-out
            bad = int(rng.integers(n))
            fr[bad, int(rng.integers(F))] ^= 0x5A
            host_fr = fr.cpu().numpy()
            csum_in = torch.from_numpy(want_cs).to(cuda) if layout == 5 else None
            want_d = codec_np.decode(host_fr, layout, want_cs if layout == 5 else None)
            for copy in (False, True):
                d = batch.unpack_batch(fr, layout, csum=csum_in, copy_payload=copy)
                for name, g, w in zip(("seq", "ack", "flags", "ok", "csum"),
                                      (d.seq, d.ack, d.flags, d.ok, d.csum), want_d[:5]):
                    assert np.array_equal(g.cpu().numpy(), w), (ctx, copy, name)
                if copy:
                    assert np.array_equal(d.payload.cpu().numpy(), host_fr[:, layout:]), (ctx, copy)
        finally:
            for k, v in reversed(old):
                lib.rudpx_tune(k, v)


_VKNOBS = {51: (1, 0, 2), 52: (2, 0), 49: (0, 1), 46: (16, 0, 64), 47: (0, 1, 2, 4, 8), 50: (1, 0), 14: (1, 0), 16: (1, 0), 36: (1, 2, 0), 43: (1, 0), 44: (-1, 0, 6, 7, 8), 45: (34816, 0, 16384), 30: (-1, 0, 1, 2), 39: (110, 125, 100), 33: (1, 2, 0),
           38: (110, 125), 41: (1, 0), 42: (130, 110)}


@pytest.mark.parametrize("seed", range(4))
def test_random_varlen_vs_oracle(cuda, seed):
    """Packed variable-length batches: random length distributions, hints and
    varlen knobs; encode frames/offsets/checksums, decode fields and UTF-8
    flags against the oracle."""
    import torch
    lib = _lib()
    rng = np.random.default_rng(7000 + seed)
    for case in range(8):
        n = int(rng.integers(1, 4000))
        kind = case % 4
        if kind == 0:
            lens = rng.integers(0, 40, n)
        elif kind == 1:
            lens = rng.integers(300, 3000, n)
        elif kind == 2:
            lens = np.full(n, int(rng.choice([64, 1024, 1472])))
        else:
            lens = np.where(rng.random(n) < 0.8, 1, rng.integers(500, 4000, n))
        lens = lens.astype(np.int32)
        layout = int(rng.choice([5, 7]))
        knobs = {k: int(rng.choice(v)) for k, v in _VKNOBS.items()}
        seq, ack, flags, _ = synth.synth(int(rng.integers(1 << 30)), 0, n, 0)
        packed = rng.integers(0, 128, int(lens.sum()), dtype=np.uint8)  # ASCII: UTF-8 valid
        if rng.random() < 0.5 and len(packed):
            packed[rng.integers(0, len(packed), 1 + len(packed) // 500)] = 0xC3  # some invalid
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        pays = [packed[offs[i]:offs[i + 1]].tobytes() for i in range(n)]
        want_fr, want_off, want_cs = codec_np.encode_varlen(seq, ack, flags, pays, layout)
        old = [(k, lib.rudpx_tune(k, v)) for k, v in knobs.items()]
        try:
            tab = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(cuda) for x in (seq, ack, flags))
            res = batch.pack_batch_varlen(tab, torch.from_numpy(packed).to(cuda),
                                          torch.from_numpy(lens).to(cuda), layout, want_csum=True)
            ctx = (seed, case, kind, n, layout, knobs)
            assert np.array_equal(res.frames.cpu().numpy(), want_fr), ctx
            assert np.array_equal(res.frame_off.cpu().numpy(), want_off), ctx
            assert np.array_equal(res.csum.cpu().numpy(), want_cs), ctx
            d = batch.unpack_batch_varlen(res.frames, res.frame_off, layout,
                                          csum=res.csum if layout == 5 else None)
            want_d = codec_np.decode_varlen(want_fr, want_off, layout, want_cs if layout == 5 else None)
            for name, g, w in zip(("seq", "ack", "flags", "ok", "csum"),
                                  (d.seq, d.ack, d.flags, d.ok, d.csum), want_d[:5]):
                assert np.array_equal(g.cpu().numpy(), w), (ctx, name)
            v = batch.validate_utf8(res.frames, layout, frame_off=res.frame_off)
            assert np.array_equal(v.cpu().numpy(), codec_np.utf8_valid(want_fr, want_off, layout)), ctx
        finally:
            for k, val in reversed(old):
                lib.rudpx_tune(k, val)
