"""HIP kernels (through the C ABI) against the oracle and the reference goldens.

Bit-exact everywhere: this is byte/integer work.  Small shapes are diffed
element-wise against the committed golden vectors (produced by the reference
utils/packet.py) and against oracle/codec_np.py; the BASELINE configs at full
size are checked through SHA-256 digests of the reference-framed batches.
"""
import hashlib

import numpy as np
import pytest

from conftest import small_lengths
from oracle import codec_np, synth
from rudp import batch

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def host(t):
    return t.cpu().numpy()


def gpu_encode(cuda, seq, ack, flags, pay, layout, want_csum=True):
    fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda),
                              layout, want_csum=want_csum)
    return host(fr), (host(cs) if cs is not None else None)


# ------------------------------------------------------------------ synth
@pytest.mark.parametrize("n,L,ascii", [(1000, 1472, True), (777, 65, False), (5000, 64, True),
                                       (100, 0, True), (300, 7, False), (33, 1024, False)])
def test_synth_matches_numpy(cuda, n, L, ascii):
    tab, pay = batch.synth_batch(n, L, seed=0xABCDEF + L, first_index=12345, ascii=ascii,
                                 device=cuda)
    want = synth.synth(0xABCDEF + L, 12345, n, L, ascii=ascii)
    for got, exp in zip((tab.seq, tab.ack, tab.flags, pay), want):
        assert np.array_equal(host(got), exp)


# --------------------------------------------------------------- goldens
@pytest.mark.parametrize("layout", [5, 7])
def test_encode_matches_reference_goldens(cuda, golden_small, layout):
    for L in small_lengths(golden_small):
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        fr, cs = gpu_encode(cuda, g["seq"], g["ack"], g["flags"], g["payload"], layout)
        assert np.array_equal(fr, g[f"frames{layout}"]), f"L={L}"
        assert np.array_equal(cs, g["csum"]), f"L={L}"


@pytest.mark.parametrize("layout", [5, 7])
def test_decode_matches_reference_goldens(cuda, golden_small, layout):
    for L in small_lengths(golden_small):
        fr = golden_small[f"L{L}_full_frames{layout}"]
        ref = golden_small[f"L{L}_full_fields{layout}"]
        d = batch.unpack_batch(dev(fr, cuda), layout, copy_payload=True)
        assert np.array_equal(host(d.seq), ref[:, 0]), f"L={L}"
        assert np.array_equal(host(d.ack), ref[:, 1])
        assert np.array_equal(host(d.flags), ref[:, 2])
        assert np.array_equal(host(d.payload), fr[:, layout:])
        if layout == 7:
            assert np.array_equal(host(d.csum), ref[:, 3]) and (host(d.ok) == 1).all()
        else:
            assert (host(d.ok) == 3).all()
            _, want = codec_np.encode(ref[:, 0], ref[:, 1], ref[:, 2], fr[:, 5:], 5)
            assert np.array_equal(host(d.csum), want)
            d2 = batch.unpack_batch(dev(fr, cuda), 5, csum=dev(want, cuda))
            assert (host(d2.ok) == 1).all()


# ------------------------------------------------------- shapes & edge cases
LENGTHS = [16, 32, 48, 64, 80, 128, 256, 1008, 1024, 1472, 2048, 4096, 4112, 1, 5, 63, 1471]
COUNTS = [1, 15, 16, 17, 255, 257, 4099]


@pytest.mark.parametrize("L", LENGTHS)
def test_roundtrip_vs_oracle(cuda, L):
    for n in COUNTS:
        seq, ack, flags, pay = synth.synth(0x1000 + L, 3 * n, n, L, ascii=False)
        for layout in (5, 7):
            fr, cs = gpu_encode(cuda, seq, ack, flags, pay, layout)
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            assert np.array_equal(fr, want_fr), (L, n, layout)
            assert np.array_equal(cs, want_cs), (L, n, layout)
            d = batch.unpack_batch(dev(fr, cuda), layout, copy_payload=True,
                                   csum=dev(cs, cuda) if layout == 5 else None)
            assert (host(d.ok) == 1).all(), (L, n, layout)
            assert np.array_equal(host(d.seq), seq) and np.array_equal(host(d.ack), ack)
            assert np.array_equal(host(d.flags), flags)
            assert np.array_equal(host(d.payload), pay)


def test_misaligned_buffers_take_stride_tiles(cuda):
    """1024-B payloads in views at odd byte offsets miss the fixed-length tiles
    only through their alignment: the varlen tiles with implicit offsets frame
    and decode them (tests/test_gpu_stride.py covers every shape)."""
    import torch
    n, L = 1000, 1024
    seq, ack, flags, pay = synth.synth(77, 0, n, L, ascii=False)
    raw = torch.zeros(n * L + 16, dtype=torch.uint8, device=cuda)
    view = raw[3:3 + n * L].view(n, L)
    view.copy_(dev(pay, cuda))
    out_raw = torch.zeros(n * (L + 7) + 16, dtype=torch.uint8, device=cuda)
    out = out_raw[5:5 + n * (L + 7)].view(n, L + 7)
    fr, _ = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), view, 7, out=out)
    want, _ = codec_np.encode(seq, ack, flags, pay, 7)
    assert np.array_equal(host(fr), want)
    d = batch.unpack_batch(out, 7, copy_payload=True)
    assert (host(d.ok) == 1).all() and np.array_equal(host(d.payload), pay)


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_header_table_views_any_alignment(cuda, shift):
    """The encode tile takes a full tile's header table by LDS-DMA only when
    the seq/ack/flags arrays are 16-B aligned (1472-B payloads); tables that are
    views at odd element offsets, and the batch's partial last tile, take the
    leaders' own loads.  Frames and checksums equal the oracle's either way."""
    import torch
    n, L = 16 * 300 + 5, 1472
    seq, ack, flags, pay = synth.synth(91 + shift, 0, n, L, ascii=False)
    cols = []
    for a, dt in ((seq, torch.uint16), (ack, torch.uint16), (flags, torch.uint8)):
        raw = torch.zeros(n + 8, dtype=dt, device=cuda)
        v = raw[shift:shift + n]
        v.copy_(dev(a, cuda))
        cols.append(v)
    for layout in (5, 7):
        fr, cs = batch.pack_batch(tuple(cols), dev(pay, cuda), layout, want_csum=True)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(host(fr), want_fr), (shift, layout)
        assert np.array_equal(host(cs), want_cs), (shift, layout)


@pytest.mark.parametrize("layout", [5, 7])
def test_single_byte_corruption_detected(cuda, layout):
    n, L = 4096, 1472
    seq, ack, flags, pay = synth.synth(99, 0, n, L, ascii=False)
    fr, cs = gpu_encode(cuda, seq, ack, flags, pay, layout)
    rng = np.random.default_rng(5)
    pos = rng.integers(0, L + layout, size=n)
    delta = rng.integers(1, 256, size=n).astype(np.uint8)
    bad = fr.copy()
    bad[np.arange(n), pos] += delta
    d = batch.unpack_batch(dev(bad, cuda), layout, csum=dev(cs, cuda) if layout == 5 else None)
    assert (host(d.ok) == 0).all()
    ok_np = codec_np.decode(bad, layout, cs if layout == 5 else None)[3]
    assert np.array_equal(host(d.ok), ok_np)


@pytest.mark.parametrize("layout", [5, 7])
def test_short_frames(cuda, layout):
    for F in range(0, layout):
        fr = np.arange(37 * F, dtype=np.uint8).reshape(37, F) if F else np.zeros((37, 0), np.uint8)
        d = batch.unpack_batch(dev(fr, cuda), layout)
        seq, ack, flags, ok, cs, _ = codec_np.decode(fr, layout)
        assert (host(d.ok) == 2).all()
        assert np.array_equal(host(d.seq), seq) and np.array_equal(host(d.ack), ack)
        assert np.array_equal(host(d.flags), flags)


def test_header_only_frames(cuda):
    # payload_len 0: the final ACK / FIN|ACK frames of utils/reliableUDP.py:88-92, :156-161
    seq = np.array([0x0E21, 0, 0], np.uint16)
    ack = np.array([1, 0x0E21, 0x0E1C], np.uint16)
    flags = np.array([0x40, 0x60, 0x40], np.uint8)
    fr, cs = gpu_encode(cuda, seq, ack, flags, np.zeros((3, 0), np.uint8), 5)
    assert [bytes(r).hex() for r in fr] == ["0e21000140", "00000e2160", "00000e1c40"]
    d = batch.unpack_batch(dev(fr, cuda), 5, csum=dev(cs, cuda))
    assert (host(d.ok) == 1).all()


def test_empty_batch(cuda):
    fr, cs = gpu_encode(cuda, np.zeros(0, np.uint16), np.zeros(0, np.uint16), np.zeros(0, np.uint8),
                        np.zeros((0, 64), np.uint8), 5)
    assert fr.shape == (0, 69) and cs.shape == (0,)
    d = batch.unpack_batch(dev(np.zeros((0, 71), np.uint8), cuda), 7)
    assert host(d.ok).shape == (0,)


def test_side_stream(cuda):
    import torch
    seq, ack, flags, pay = synth.synth(3, 0, 2048, 1472, ascii=False)
    s = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s):
        fr, _ = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)), dev(pay, cuda), 7)
    s.synchronize()
    assert np.array_equal(host(fr), codec_np.encode(seq, ack, flags, pay, 7)[0])


def test_host_staged_path(cuda):
    seq, ack, flags, pay = synth.synth(11, 0, 70000, 1024, ascii=False)
    for layout in (5, 7):
        fr, cs = batch.pack_batch((seq, ack, flags), pay, layout)  # numpy in -> numpy out
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(fr, want_fr) and np.array_equal(cs if cs is not None else want_cs, want_cs)
        d = batch.unpack_batch(fr, layout, csum=cs if layout == 5 else None, copy_payload=True)
        assert (d.ok == 1).all() and np.array_equal(d.payload, pay)
        assert np.array_equal(d.seq, seq) and np.array_equal(d.flags, flags)


# ------------------------------------------------- full-size BASELINE configs
def _digest_run(cuda, cfg, layout, chunk_index):
    import torch
    n = min(cfg["chunk"], cfg["n"] - chunk_index * cfg["chunk"])
    tab, pay = batch.synth_batch(n, cfg["L"], cfg["seed"], first_index=chunk_index * cfg["chunk"],
                                 device=cuda)
    fr, cs = batch.pack_batch(tab, pay, layout, want_csum=True)
    torch.cuda.synchronize()
    h_fr = hashlib.sha256(host(fr).tobytes()).hexdigest()
    h_cs = hashlib.sha256(host(cs).astype("<u2").tobytes()).hexdigest()
    return h_fr, h_cs, (tab, pay, fr, cs)


@pytest.mark.slow
@pytest.mark.parametrize("name,layout,chunk", [("C2", 5, 0), ("C2", 7, 0), ("C3", 5, 0), ("C3", 7, 0),
                                               ("C4", 5, 0), ("C4", 7, 0),
                                               ("C5", 7, 0), ("C5", 7, 9), ("C5", 5, 15)])
def test_full_size_digests(cuda, digests, name, layout, chunk):
    cfg = digests[name]
    h_fr, h_cs, _ = _digest_run(cuda, cfg, layout, chunk)
    want = cfg["layouts"][str(layout)]
    assert h_fr == want["frames"][chunk]
    assert h_cs == want["csum"][chunk]


@pytest.mark.slow
def test_c4_roundtrip_full_size(cuda, digests):
    """Config 4: 1M x 1472 B encode -> decode, bit-exact vs the reference digest."""
    import torch
    cfg = digests["C4"]
    h_fr, _, (tab, pay, fr, cs) = _digest_run(cuda, cfg, 7, 0)
    assert h_fr == cfg["layouts"]["7"]["frames"][0]
    d = batch.unpack_batch(fr, 7, copy_payload=True)
    assert bool((d.ok == 1).all())
    assert torch.equal(d.payload, pay)
    assert torch.equal(d.seq.view(torch.int16), tab.seq.view(torch.int16))
    assert torch.equal(d.ack.view(torch.int16), tab.ack.view(torch.int16))
    assert torch.equal(d.flags, tab.flags)
    assert torch.equal(d.csum.view(torch.int16), cs.view(torch.int16))


@pytest.mark.parametrize("L", [16, 64, 256, 1472, 4096, 8192])
def test_decode_paths_agree(cuda, L):
    """Every decode kernel (LDS tile, aligned chunks, register windows) gives the same answer."""
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    n = 3001
    seq, ack, flags, pay = synth.synth(0x77 + L, 0, n, L, ascii=False)
    fr, cs = gpu_encode(cuda, seq, ack, flags, pay, 7)
    fr[17, 9] ^= 0x40  # one corrupted frame
    want = codec_np.decode(fr, 7)
    results = []
    for verify_tile, copy_tile, align, stage in ((1, 1, -1, 0), (1, 1, 1, 0), (0, 0, -1, 0),
                                                 (1, 1, -1, 1), (1, 1, 1, 1)):
        lib.rudpx_tune(12, verify_tile)
        lib.rudpx_tune(11, copy_tile)
        lib.rudpx_tune(23, align)  # tile loads/stores from a 64-B boundary
        lib.rudpx_tune(34, stage)  # tile outputs staged in LDS, written as dwords
        try:
            for copy in (False, True):
                d = batch.unpack_batch(dev(fr, cuda), 7, copy_payload=copy)
                got = [host(x) for x in (d.seq, d.ack, d.flags, d.ok, d.csum)]
                for g, w in zip(got, want[:5]):
                    assert np.array_equal(g, w), (L, verify_tile, copy, align, stage)
                if copy:
                    assert np.array_equal(host(d.payload), fr[:, 7:])
                results.append(got)
        finally:
            lib.rudpx_tune(12, 1)
            lib.rudpx_tune(11, 1)
            lib.rudpx_tune(23, -1)
            lib.rudpx_tune(34, 0)
    assert host(d.ok)[17] == 0


@pytest.mark.parametrize("L", [16, 64, 1024, 1472, 4096])
def test_encode_tile_sizes_agree(cuda, L):
    """Every encode tile size gives the oracle's frames (T < 16: tiles share boundary chunks)."""
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    for n in (1, 3, 4, 5, 9, 33, 1027):
        seq, ack, flags, pay = synth.synth(0x99 + L, n, n, L, ascii=False)
        for layout in (5, 7):
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            combos = [(256, t, pc) for t in (4, 8, 16, 32, 256) for pc in (-1, 0, 5)]
            combos += [(64, t, 0) for t in (4, 8, 16, 32)] + [(128, t, 16) for t in (8, 64)]
            for block, tile, per_cu in combos:
                lib.rudpx_tune(10, block)
                lib.rudpx_tune(2, tile)
                lib.rudpx_tune(6, per_cu)
                try:
                    fr, cs = gpu_encode(cuda, seq, ack, flags, pay, layout)
                finally:
                    lib.rudpx_tune(10, 256)
                    lib.rudpx_tune(2, 0)
                    lib.rudpx_tune(6, -1)
                assert np.array_equal(fr, want_fr), (L, n, layout, block, tile, per_cu)
                assert np.array_equal(cs, want_cs), (L, n, layout, block, tile, per_cu)


@pytest.mark.parametrize("L", [16, 48, 64, 1024, 1472, 4096])
def test_encode_align64_vs_oracle(cuda, L):
    """Encode tile kernels dealing wave stores from the first 64-B boundary
    (rudpx_tune 23 = 1) or the first 16-B one (0) give the oracle's frames,
    fixed-length and varlen, every tile size."""
    import ctypes
    import torch
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    for n in (1, 5, 16, 17, 257, 1031):
        seq, ack, flags, pay = synth.synth(0x55 + L, n, n, L, ascii=False)
        for layout in (5, 7):
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            tab = (dev(seq, cuda), dev(ack, cuda), dev(flags, cuda))
            lens = torch.full((n,), L, dtype=torch.int32, device=cuda)
            for align in (1, 0):
                for tile in (0, 4, 8, 32):
                    old = (lib.rudpx_tune(23, align), lib.rudpx_tune(2, tile))
                    try:
                        fr, cs = gpu_encode(cuda, seq, ack, flags, pay, layout)
                        v = batch.pack_batch_varlen(tab, dev(pay.reshape(-1), cuda), lens, layout,
                                                    want_csum=True)
                    finally:
                        lib.rudpx_tune(23, old[0])
                        lib.rudpx_tune(2, old[1])
                    assert np.array_equal(fr, want_fr), (L, n, layout, align, tile)
                    assert np.array_equal(cs, want_cs), (L, n, layout, align, tile)
                    assert np.array_equal(host(v.frames), want_fr.reshape(-1)), (L, n, layout, align)
                    assert np.array_equal(host(v.csum), want_cs), (L, n, layout, align)


def test_concurrent_callers(cuda):
    """The proxy calls the codec from ThreadPoolExecutor workers (proxy.py:127, :154):
    host-staged and device-resident calls from 8 threads at once stay exact, and an
    error in one thread leaves the others' calls and messages alone."""
    from concurrent.futures import ThreadPoolExecutor
    import torch
    from rudp import _native

    import threading
    start = threading.Barrier(8)  # eight distinct threads, all inside the library together

    def job(k):
        start.wait(timeout=60)
        L = (64, 1472, 100, 1024)[k % 4]
        seq, ack, flags, pay = synth.synth(0x7000 + k, k * 1000, 3000, L, ascii=False)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, 7)
        for rep in range(3):
            if k % 2:   # host-staged pipeline (shared, mutex-guarded staging)
                fr, cs = batch.pack_batch((seq, ack, flags), pay, 7, want_csum=True)
                d = batch.unpack_batch(fr, 7)
                got_fr, got_cs, ok = fr, cs, d.ok
            else:       # device path on this thread's own stream
                s = torch.cuda.Stream(cuda)
                with torch.cuda.stream(s):
                    fr, cs = batch.pack_batch((dev(seq, cuda), dev(ack, cuda), dev(flags, cuda)),
                                              dev(pay, cuda), 7, want_csum=True)
                    d = batch.unpack_batch(fr, 7)
                s.synchronize()
                got_fr, got_cs, ok = host(fr), host(cs), host(d.ok)
            assert np.array_equal(got_fr, want_fr), (k, rep)
            assert np.array_equal(got_cs, want_cs), (k, rep)
            assert (ok == 1).all(), (k, rep)
            if k == 3 and rep == 1:  # a failing C call on this thread only
                assert _native.lib().rudp_device_count(None) == -22
        return _native.lib().rudp_last_error().decode()

    with ThreadPoolExecutor(8) as ex:
        msgs = list(ex.map(job, range(8)))
    # rudp_last_error is per thread: only the thread that failed carries a message
    assert "NULL" in msgs[3] and not any(m for i, m in enumerate(msgs) if i != 3), msgs


@pytest.mark.parametrize("slots,stage_mb", [(2, 1), (3, 1), (8, 2)])
def test_host_pipeline_many_chunks(cuda, slots, stage_mb):
    """rudp_encode_host / rudp_decode_host with small staging slots: the batch cycles
    through the slot ring in many chunks (ragged last chunk), H2D/kernel/D2H overlapped."""
    import ctypes
    from rudp import _native
    lib = _native.tools_lib()
    lib.rudpx_tune.argtypes = [ctypes.c_int, ctypes.c_int]
    old_slots, old_mb = lib.rudpx_tune(8, slots), lib.rudpx_tune(9, stage_mb)
    try:
        n, L = 20011, 1472   # ~29 MiB of frames: 15-30 chunks
        seq, ack, flags, pay = synth.synth(0x4321 + slots, 7, n, L, ascii=False)
        for layout in (5, 7):
            fr, cs = batch.pack_batch((seq, ack, flags), pay, layout, want_csum=True)
            want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
            assert np.array_equal(fr, want_fr) and np.array_equal(cs, want_cs), layout
            fr[n - 1, 9] ^= 0x10  # the last frame of the ragged last chunk
            d = batch.unpack_batch(fr, layout, csum=cs if layout == 5 else None, copy_payload=True)
            ok = d.ok.copy()
            assert ok[n - 1] == 0 and (ok[:-1] == 1).all()
            assert np.array_equal(d.seq, seq) and np.array_equal(d.ack, ack)
            assert np.array_equal(d.payload[:-1], pay[:-1])
    finally:
        lib.rudpx_tune(8, old_slots)
        lib.rudpx_tune(9, old_mb)


@pytest.mark.parametrize("L", [65535, 65520, 4096 + 16])
def test_maximum_payloads(cuda, L):
    """The largest payload utils/packet.py frames here (kMaxPayload = 65535): byte and
    vector paths, both layouts, round trip and a corrupted byte."""
    n = 37
    seq, ack, flags, pay = synth.synth(0x600D + L, 0, n, L, ascii=False)
    for layout in (5, 7):
        fr, cs = gpu_encode(cuda, seq, ack, flags, pay, layout)
        want_fr, want_cs = codec_np.encode(seq, ack, flags, pay, layout)
        assert np.array_equal(fr, want_fr) and np.array_equal(cs, want_cs), (L, layout)
        fr[5, L // 2] ^= 0x01
        for copy in (False, True):
            d = batch.unpack_batch(dev(fr, cuda), layout, copy_payload=copy,
                                   csum=dev(cs, cuda) if layout == 5 else None)
            ok = host(d.ok)
            assert ok[5] == 0 and ok.sum() == n - 1, (L, layout, copy)
            if copy:
                assert np.array_equal(host(d.payload), fr[:, layout:])


def test_payload_over_maximum_rejected(cuda):
    import torch
    pay = torch.zeros((2, 65536), dtype=torch.uint8, device=cuda)
    tab = batch.synth_batch(2, 0, 1, device=cuda)[0]
    with pytest.raises(ValueError, match="exceeds"):
        batch.pack_batch(tab, pay, 7)
