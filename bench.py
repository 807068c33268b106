"""Benchmark: device-resident checksum + framing of Reliable-UDP packet batches.

Contract (see DESIGN.md "Measurement"): `python bench.py --gpus N --steps K
--warmup W`; for N > 1 launched by torch.distributed.run, one rank per GPU.
A step is one rudp_encode launch over one batch of synthetic packets already
resident in HBM (default: 1M x 1472 B per GPU, layout rudp7, the workload of
BASELINE.json's 70%-of-roofline target).  Packet batches shard by slicing the
packet array: each rank generates and frames its own slice,
no collective touches the data path (scaling "weak": fixed work per GPU).
Rank 0 prints one JSON line.

Measured beside the headline (rank 0, N = 1 only): the other BASELINE
shapes as "legs" (1M x 1024, 1M x 64, decode-verify, C4 encode->decode round
trip, host-memory end to end), a device-to-device copy ceiling, and the
reference algorithm's CPU path (the oracle's bit-string port of
utils/packet.py) on a bounded sample on the host cores.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "reliable-udp_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak, MI355X_MICROARCH.md
GIB = float(1 << 30)
SEEDS = {1024: 0x5EED0002, 64: 0x5EED0003, 1472: 0x5EED0004}


def algorithmic_bytes_encode(L: int) -> int:
    """Per packet: read L payload + 5 header-table bytes, write L + 2 + 5."""
    return 2 * L + 12


def algorithmic_bytes_decode(L: int, H: int = 7) -> int:
    """Per packet, zero-copy decode-verify: read L + H, write seq/ack/flags/ok = 6."""
    return L + H + 6


# ------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    seed, first, n, L = args
    from oracle import bitstring_packet as bp
    from oracle import codec_np, synth
    seq, ack, flags, pay = synth.synth(seed, first, n, L)
    _, csum = codec_np.encode(seq, ack, flags, pay, 5)
    rows = [(int(seq[i]), int(ack[i]), int(flags[i]), pay[i].tobytes(), int(csum[i])) for i in range(n)]
    t0 = time.perf_counter()
    for s, a, f, p, c in rows:
        bp.encode_like_reference(s, a, f, p, csum=c)
    return n * L, time.perf_counter() - t0


def cpu_baseline(L: int, per_worker: int, workers: int):
    """Reference algorithm (bit-string port, rudp7 encode) on the host cores."""
    import multiprocessing as mp
    seed = SEEDS.get(L, 0x5EED0004)
    ctx = mp.get_context("fork")  # before any HIP call in this process
    tasks = [(seed, w * per_worker, per_worker, L) for w in range(workers)]
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, tasks)
    single = _cpu_worker((seed, 0, max(per_worker // 4, 256), L))
    total = sum(b for b, _ in res)
    wall = max(t for _, t in res)
    return {
        "value": total / wall / GIB,
        "unit": "GiB/s",
        "cores": workers,
        "kind": "port",
        "sample": f"{workers} workers x {per_worker} packets x {L} B: the reference's framing "
                  f"(Packet(), set_header_field x4, set_payload, to_byte: utils/packet.py's bit-string "
                  f"algorithm, oracle/bitstring_packet.py) of the rudp7 layout, payload GiB/s.  The "
                  f"reference has no checksum: the checksum field's value is computed with numpy "
                  f"before the clock and only the framing is timed",
        "single_core_value": single[0] / single[1] / GIB,
        "single_core_us_per_packet": single[1] / max(per_worker // 4, 256) * 1e6,
        "cpu_model": _cpu_model(),
        "os_cpu_count": os.cpu_count(),
        "cpu_share": usable_cpus(),
        "workers_note": "one worker per usable CPU (affinity mask / cgroup quota): os.cpu_count() "
                        "counts the whole host, of which this job may use only its share",
    }


def usable_cpus() -> dict:
    """CPUs this process may actually run on: the affinity mask, capped by a
    cgroup CPU quota when there is one (os.cpu_count() reports the whole host)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota) if quota else aff}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------- GPU helpers
class Workload:
    """Input/output buffer sets for one batch shape, rotated so the working
    set exceeds the 256 MiB Infinity Cache (SURVEY.md §7 hard part 4)."""

    def __init__(self, torch, batch, n, L, layout, first, seed, device, min_bytes=1 << 30):
        H = batch.layout_header_len(layout)
        set_bytes = n * (2 * L + H + 5)
        self.sets = []
        nsets = max(1, min(8, math.ceil(min_bytes / max(set_bytes, 1))))
        for k in range(nsets):
            tab, pay = batch.synth_batch(n, L, seed, first_index=first, device=device)
            out = torch.empty((n, L + H), dtype=torch.uint8, device=device)
            self.sets.append((tab, pay, out))
        self.n, self.L, self.H, self.layout = n, L, H, layout

    def encode(self, batch, i):
        tab, pay, out = self.sets[i % len(self.sets)]
        batch.pack_batch(tab, pay, self.layout, out=out, want_csum=False)

    def decode(self, batch, i):
        _, _, out = self.sets[i % len(self.sets)]
        return batch.unpack_batch(out, self.layout)


def time_events(torch, fn, steps, warmup):
    """Per-launch HIP-event times (ms) of `steps` calls on the current stream,
    after `warmup` untimed calls: a start/stop event pair around every call."""
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for i, (a, b) in enumerate(ev):
        a.record()
        fn(warmup + i)
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def rank_slice(rank: int, world: int, total: int):
    """Packets rank r frames when `total` packets are split over `world` ranks:
    [r*total/world, (r+1)*total/world) (no exchange step;
    rudp.shard.rank_slice)."""
    from rudp.shard import rank_slice as _rank_slice
    return _rank_slice(rank, world, total)


def verify_digests(w, cfg_name, first, n):
    """Hash this rank's frames of BASELINE config `cfg_name` per 2^20-packet chunk
    and compare them with the digests utils/packet.py produced
    (tests/golden/digests.json; make_golden.py).  Every buffer set of the
    workload holds the same batch; all of them are checked.  Returns (chunks
    checked, chunks matching), or None when the fixture has no entry for this
    shape and layout."""
    path = REPO / "tests" / "golden" / "digests.json"
    if not path.exists():
        return None
    cfg = json.loads(path.read_text()).get(cfg_name)
    if cfg is None:
        return None
    want = cfg["layouts"].get(str(w.H))
    if want is None or first % cfg["chunk"] or n % cfg["chunk"] or w.L != cfg["L"]:
        return None
    k0 = first // cfg["chunk"]
    if k0 + n // cfg["chunk"] > len(want["frames"]):
        return None
    from rudp import digest
    checked = matching = 0
    for tab, pay, out in w.sets:
        got = digest.chunk_sha256(out, None, cfg["chunk"])
        checked += len(got)
        matching += sum(h == want["frames"][k0 + k] for k, (h, _) in enumerate(got))
    return checked, matching


def verify_c5(w, first, n):
    """verify_digests for BASELINE config 5 (16M x 1472 B)."""
    return verify_digests(w, "C5", first, n)


def digest_field(chk):
    return None if chk is None else f"{chk[1]}/{chk[0]}"


def time_loop(torch, fn, steps, warmup, warm_ms=30.0):
    """HIP-event time of `steps` back-to-back calls on the current stream (ms),
    after `warmup` calls and at least `warm_ms` of back-to-back calls: after an
    idle stretch (a host-side digest, a PCIe-bound leg) the first launches run
    several percent slow (1M x 1024 B: 0.373 vs 0.351 ms right after the
    headline's digest check; tools/c2_probe.py)."""
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i = warmup
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        for _ in range(4):
            fn(i)
            i += 1
        torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    stop = torch.cuda.Event(enable_timing=True)
    start.record()
    for i in range(steps):
        fn(warmup + i)
    stop.record()
    stop.synchronize()
    return start.elapsed_time(stop)


C5_PACKETS = 1 << 24
C5_SEED = 0x5EED0005   # tests/golden/make_golden.py CONFIGS["C5"]


def over_ranks(torch, dist, world, share_device, device, wall_s, kernel_ms):
    """The job's clock: MAX over ranks of the wall time (device tensors over RCCL,
    CPU tensors over gloo), and every rank's HIP-event kernel time gathered, so
    the roofline can be the slowest GPU's.  Returns (wall_max_s, [kernel_ms per rank])."""
    if world == 1 and not dist.is_initialized():
        return wall_s, [kernel_ms]
    where = "cpu" if share_device else device
    t = torch.tensor([wall_s], dtype=torch.float64, device=where)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    k = torch.tensor([kernel_ms], dtype=torch.float64, device=where)
    ks = [torch.empty_like(k) for _ in range(dist.get_world_size())]
    dist.all_gather(ks, k)
    return float(t.item()), [float(x.item()) for x in ks]


def c5_strong_leg(torch, dist, batch, device, world, rank, layout, share_device, steps=10, total=None):
    """BASELINE config 5: 16M x 1472 B packets sharded over the ranks by slicing
    (rank r frames packets [r*16M/N, (r+1)*16M/N)); whole-job payload GiB/s."""
    total = total or C5_PACKETS
    first, n = rank_slice(rank, world, total)
    w = Workload(torch, batch, n, 1472, layout, first, C5_SEED, device, min_bytes=0)
    for i in range(2):
        w.encode(batch, i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        w.encode(batch, i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    wall, _ = over_ranks(torch, dist, world, share_device, device, time.perf_counter() - t0, 0.0)
    # every rank's frames against the reference's chunk digests (outside the clock)
    chk = verify_c5(w, first, n)
    ok = torch.tensor([0 if chk is None else int(chk[0] == chk[1]), 0 if chk is None else chk[1]],
                      dtype=torch.int64, device="cpu" if share_device else device)
    dist.all_reduce(ok, op=dist.ReduceOp.SUM)
    del w
    torch.cuda.empty_cache()
    return {"GiB_s": total * 1472 * steps / wall / GIB, "ms": wall / steps * 1e3,
            "ranks_bit_exact_vs_reference": int(ok[0].item()),
            "chunks_matching_reference_digests": int(ok[1].item()),
            "packets_total": total, "packets_per_gpu": n, "n_gpus": world, "steps": steps,
            "per_gpu_roofline_frac": n * algorithmic_bytes_encode(1472) / (wall / steps) / 1e9 / HBM_PEAK_GBS,
            "scaling": "strong"}


def copy_same_bytes(torch, device, alg_bytes, nsets, steps, encode_ms):
    """Streaming copy (rudpx_copy_vpt: one dwordx4 per thread, nt loads and stores,
    diagnostics build) moving alg_bytes per launch (half read, half written) over
    nsets rotating buffer pairs: the HBM ceiling at the size of one encode launch."""
    from rudp import _native
    lib = _native.tools_lib(activate=False)
    half = alg_bytes // 2 // 16 * 16
    bufs = [(torch.empty(half, dtype=torch.uint8, device=device), torch.empty(half, dtype=torch.uint8, device=device))
            for _ in range(nsets)]
    stream = torch.cuda.current_stream().cuda_stream
    ms = time_loop(torch, lambda i: lib.rudpx_copy_vpt(bufs[i % nsets][0].data_ptr(), bufs[i % nsets][1].data_ptr(),
                                                       half // 16, 1, 1, stream), steps, 3) / steps
    del bufs
    gbs = 2 * half / (ms / 1e3) / 1e9
    return {"copy_same_bytes_ms": ms, "copy_same_bytes_GBs": gbs,
            "copy_same_bytes_frac_of_peak": gbs / HBM_PEAK_GBS, "frac_of_copy_same_bytes": ms / encode_ms}


def legs(torch, batch, device, steps):
    out = {}
    for L, cfg_name in ((1024, "C2"), (64, "C3")):
        w = Workload(torch, batch, 1 << 20, L, "rudp7", 0, SEEDS[L], device)
        ms = time_loop(torch, lambda i: w.encode(batch, i), steps, 3) / steps
        # every buffer set's frames against the reference digests, outside the clock
        chk = verify_digests(w, cfg_name, 0, 1 << 20)
        out[f"encode_1Mx{L}"] = {
            "GiB_s": (1 << 20) * L / (ms / 1e3) / GIB, "ms": ms,
            "roofline_frac": (1 << 20) * algorithmic_bytes_encode(L) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
            "buffer_sets": len(w.sets),
            "matches_reference": None if chk is None else chk[0] == chk[1] > 0,
            "chunks_matching_reference_digests": digest_field(chk)}
        if L == 64:
            # the streaming copy of the same bytes in the same number of rotating sets: at
            # 147 MB per launch the ramp and tail of any HBM-bound launch are a visible part
            # of it, so this (not 8 TB/s) is what the 64-B encode can reach
            out["encode_1Mx64"].update(copy_same_bytes(torch, device, (1 << 20) * algorithmic_bytes_encode(L),
                                                       len(w.sets), steps, ms))
        del w
    w = Workload(torch, batch, 1 << 20, 1472, "rudp7", 0, SEEDS[1472], device)
    for i in range(len(w.sets)):
        w.encode(batch, i)
    ms = time_loop(torch, lambda i: w.decode(batch, i), steps, 3) / steps
    out["decode_verify_1Mx1472"] = {
        "GiB_s": (1 << 20) * 1472 / (ms / 1e3) / GIB, "ms": ms,
        "roofline_frac": (1 << 20) * algorithmic_bytes_decode(1472) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS}
    # the reference's whole receive per datagram: parse + verify + get_payload()'s strict
    # UTF-8 decode (utils/reliableUDP.py:118-123, utils/packet.py:73), in one pass
    # (rudp_decode_utf8), beside the two-pass form (decode, then the validation kernel)
    nsets = len(w.sets)
    ms_u = time_loop(torch, lambda i: batch.unpack_batch(w.sets[i % nsets][2], "rudp7", utf8=True),
                     steps, 3) / steps

    def two_pass(i):
        batch.unpack_batch(w.sets[i % nsets][2], "rudp7")
        batch.validate_utf8(w.sets[i % nsets][2], "rudp7")
    ms_2 = time_loop(torch, two_pass, steps, 3) / steps
    du = batch.unpack_batch(w.sets[0][2], "rudp7", utf8=True)
    out["decode_utf8_1Mx1472"] = {
        "GiB_s": (1 << 20) * 1472 / (ms_u / 1e3) / GIB, "ms": ms_u,
        "roofline_frac": (1 << 20) * (algorithmic_bytes_decode(1472) + 1) / (ms_u / 1e3) / 1e9 / HBM_PEAK_GBS,
        "two_pass_ms": ms_2,
        "all_valid_and_verified": bool((du.valid == 1).all()) and bool((du.ok == 1).all()),
        "note": "rudp_decode_utf8: parse + verify + strict UTF-8 per frame in the decode tile kernel; "
                "algorithmic bytes L + 7 read, 7 written; two_pass_ms = rudp_decode then rudp_validate_utf8"}
    del du
    # the same on valid multi-byte text (every chunk takes the table check): a 1472-B
    # payload of 1-4 byte characters, framed for every packet
    text = ("é中😀aßЖ€𝄞" * 200).encode()[:1472]
    while True:
        try:
            text.decode()
            break
        except UnicodeDecodeError:
            text = text[:-1]
    text += b"x" * (1472 - len(text))
    row = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(device)
    tab_t = w.sets[0][0]
    fr_t = batch.pack_batch(tab_t, row.expand(1 << 20, 1472).contiguous(), "rudp7")[0]
    ms_t = time_loop(torch, lambda i: batch.unpack_batch(fr_t, "rudp7", utf8=True), steps, 3) / steps
    dt = batch.unpack_batch(fr_t, "rudp7", utf8=True)
    out["decode_utf8_1Mx1472_multibyte_text"] = {
        "ms": ms_t, "roofline_frac": (1 << 20) * (algorithmic_bytes_decode(1472) + 1) / (ms_t / 1e3) / 1e9
        / HBM_PEAK_GBS, "all_valid_and_verified": bool((dt.valid == 1).all()) and bool((dt.ok == 1).all()),
        "note": "payload: valid UTF-8 of 1-4 byte characters (no all-ASCII chunk), one frame buffer"}
    del fr_t, dt, row

    def rt(i):
        w.encode(batch, i)
        w.decode(batch, i)
    ms = time_loop(torch, rt, steps, 3) / steps
    # C4: the frames of every buffer set against the reference digest, and the
    # last decode's fields and checksum status against the inputs (outside the clock)
    chk = verify_digests(w, "C4", 0, 1 << 20)
    d = w.decode(batch, 0)
    tab0 = w.sets[0][0]
    rt_ok = (bool((d.ok == 1).all()) and torch.equal(d.seq.view(torch.int16), tab0.seq.view(torch.int16))
             and torch.equal(d.ack.view(torch.int16), tab0.ack.view(torch.int16))
             and torch.equal(d.flags, tab0.flags))
    out["roundtrip_1Mx1472"] = {
        "GiB_s": (1 << 20) * 1472 / (ms / 1e3) / GIB, "ms": ms,
        "roofline_frac": (1 << 20) * (algorithmic_bytes_encode(1472) + algorithmic_bytes_decode(1472))
        / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
        "matches_reference": None if chk is None else chk[0] == chk[1] > 0 and rt_ok,
        "chunks_matching_reference_digests": digest_field(chk),
        "decode_fields_equal_inputs": rt_ok}
    del d
    # end to end from pinned host memory: H2D -> encode -> D2H, two-stream pipeline
    # (rudp_encode_host); PCIe-bound, recorded in DESIGN.md, never the headline
    n, L = 1 << 20, 1472
    del w
    torch.cuda.empty_cache()
    tab, pay = batch.synth_batch(n, L, SEEDS[L], device=device)
    pin = lambda shape, dt: torch.empty(shape, dtype=dt, pin_memory=True)  # noqa: E731
    hp, hs, ha, hf = pin((n, L), torch.uint8), pin((n,), torch.uint16), pin((n,), torch.uint16), pin((n,), torch.uint8)
    hp.copy_(pay)
    hs.copy_(tab.seq)
    ha.copy_(tab.ack)
    hf.copy_(tab.flags)
    hout = pin((n, L + 7), torch.uint8)
    torch.cuda.synchronize()
    del tab, pay
    args = ((hs.numpy(), ha.numpy(), hf.numpy()), hp.numpy())
    batch.pack_batch(*args, "rudp7", out=hout.numpy())
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        batch.pack_batch(*args, "rudp7", out=hout.numpy())
    dt = (time.perf_counter() - t0) / reps
    out["e2e_host_encode_1Mx1472"] = {
        "GiB_s": n * L / dt / GIB, "ms": dt * 1e3,
        "pcie_GBs_each_way": n * (L + 6) / dt / 1e9,
        "note": "pinned host in/out, rudp_encode_host (H2D, kernel, D2H on two streams)"}
    del hp, hs, ha, hf
    out.update(e2e_host_decode_legs(torch, batch, hout.numpy(), n, L))
    del hout
    # BASELINE config 5's shape on one GPU: 16M x 1472 B (23.6 GB in, 23.7 GB out)
    torch.cuda.empty_cache()
    w16 = Workload(torch, batch, C5_PACKETS, 1472, "rudp7", 0, C5_SEED, device, min_bytes=0)
    ts = sorted(time_events(torch, lambda i: w16.encode(batch, i), max(10, steps // 2), 3))
    ms = ts[len(ts) // 2]
    chk = verify_c5(w16, 0, C5_PACKETS)
    out["encode_16Mx1472_C5_1gpu"] = {
        "GiB_s": C5_PACKETS * 1472 / (ms / 1e3) / GIB, "ms": ms,
        "roofline_frac": C5_PACKETS * algorithmic_bytes_encode(1472) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
        "timing": f"median of {len(ts)} per-launch HIP-event pairs after 3 warmups",
        "ms_min_max": [ts[0], ts[-1]],
        "chunks_matching_reference_digests": digest_field(chk)}
    del w16
    torch.cuda.empty_cache()
    w = Workload(torch, batch, 1 << 20, 1472, "rudp7", 0, SEEDS[1472], device)
    for i in range(len(w.sets)):
        w.encode(batch, i)
    # strict UTF-8 validation of the 1M x 1472 frames (get_payload strictness)
    fr = w.sets[0][2]
    ms = time_loop(torch, lambda i: batch.validate_utf8(fr, "rudp7"), steps, 3) / steps
    out["utf8_validate_1Mx1472"] = {"GiB_s": (1 << 20) * 1472 / (ms / 1e3) / GIB, "ms": ms}
    # reference-shaped traffic: 1M one-character datagrams (utils/reliableUDP.py:11),
    # variable-length encode (scan + frame) and decode-verify, in packets/s, through the
    # Python entry points in their sync-free form (argument checks on the device, the
    # status read once after the loop) and, beside it, with the per-call eager check
    n1 = 1 << 20
    tab1, pay1 = batch.synth_batch(n1, 1, SEEDS[1472], device=device)
    lens1 = torch.ones(n1, dtype=torch.int32, device=device)
    flat1 = pay1.view(-1)
    enc = batch.pack_batch_varlen(tab1, flat1, lens1, "rudp5", want_csum=True)

    def varlen_pair(tab, flat, lens, layout, frames, off, csum, rounds=7):
        """Sync-free and eager-check encode / decode through the Python entry, and the
        raw C-ABI call chain beside them (preallocated outputs, no Python wrapper),
        interleaved round by round so all forms see the same box state; medians
        of the per-round means (ms per call)."""
        import ctypes
        from rudp import _native
        lib = _native.lib()
        H = batch.layout_header_len(layout)
        n = lens.shape[0]
        last = {}
        f_out = torch.empty_like(frames)
        o_out = torch.empty_like(off)
        c_out = torch.empty((n,), dtype=torch.uint16, device=device) if csum is not None else None
        st = torch.empty((1,), dtype=torch.int32, device=device)
        d_out = [torch.empty((n,), dtype=dt, device=device)
                 for dt in (torch.uint16, torch.uint16, torch.uint8, torch.uint8, torch.uint16)]
        rb = _native.RudpBatch(n=n, payload_len=flat.numel() // n, reserved=0, seq=tab.seq.data_ptr(),
                               ack=tab.ack.data_ptr(), flags=tab.flags.data_ptr(), payload=flat.data_ptr(),
                               len=lens.data_ptr(), payload_off=None)
        sp = torch.cuda.current_stream().cuda_stream

        def e(i, check=False):
            last["e"] = batch.pack_batch_varlen(tab, flat, lens, layout, want_csum=csum is not None,
                                                check=check)

        def d(i, check=False):
            last["d"] = batch.unpack_batch_varlen(frames, off, layout, csum=csum, check=check)

        # the same with the outputs of an earlier call reused (no allocation per call)
        e(0)
        d(0)

        def e_reuse(i):
            last["e"] = batch.pack_batch_varlen(tab, flat, lens, layout, want_csum=csum is not None,
                                                check=False, reuse=last["e"])

        def d_reuse(i):
            last["d"] = batch.unpack_batch_varlen(frames, off, layout, csum=csum, check=False, reuse=last["d"])

        def d_utf8(i):  # parse + verify + get_payload()'s strict UTF-8, one kernel
            last["u"] = batch.unpack_batch_varlen(frames, off, layout, csum=csum, check=False, utf8=True)

        def e_abi(i):
            lib.rudp_encode_varlen_checked(ctypes.byref(rb), flat.numel(), f_out.data_ptr(), f_out.numel(),
                                           o_out.data_ptr(), c_out.data_ptr() if c_out is not None else None,
                                           st.data_ptr(), H, device.index or 0, sp)

        def d_abi(i):  # no status word: the one-kernel form the Python entry uses
            lib.rudp_decode_varlen_checked(frames.data_ptr(), frames.numel(), off.data_ptr(),
                                           frames.numel() // n, n,
                                           csum.data_ptr() if csum is not None else None,
                                           *[t.data_ptr() for t in d_out], None, H,
                                           device.index or 0, sp)
        fns = {"encode": e, "decode": d, "encode_reuse": e_reuse, "decode_reuse": d_reuse, "decode_utf8": d_utf8,
               "encode_eager_check": lambda i: e(i, True),
               "decode_eager_check": lambda i: d(i, True), "encode_abi": e_abi, "decode_abi": d_abi}
        per = {k: [] for k in fns}
        for r in range(rounds):
            for k, fn in fns.items():
                per[k].append(time_loop(torch, fn, steps, 2 if r == 0 else 1) / steps)
        last["e"].check()
        last["d"].check()
        if int(st.item()) or bool((d_out[3] == _native.OK_BAD_OFFSETS).any()):
            raise RuntimeError("the raw C-ABI varlen calls rejected the bench batch")
        return {k: sorted(v)[len(v) // 2] for k, v in per.items()}

    t1 = varlen_pair(tab1, flat1, lens1, "rudp5", enc.frames, enc.frame_off, enc.csum)
    out["varlen_1M_x_1char"] = {"encode_Mpkt_s": n1 / t1["encode"] / 1e3, "encode_ms": t1["encode"],
                                "decode_verify_Mpkt_s": n1 / t1["decode"] / 1e3, "decode_ms": t1["decode"],
                                "ms_by_form": t1,
                                "note": "Python entry, sync-free (device-side argument checks, status "
                                        "read after the loop); *_reuse: outputs of an earlier call reused "
                                        "(reuse=); *_eager_check: one sync per call; *_abi: "
                                        "the C-ABI calls alone; medians of 7 interleaved rounds"}
    # the varlen path at MTU size: 1M x 1472 B payloads packed back to back
    # (frames at odd offsets), encode (scan + tile kernel) and decode-verify
    tabm, paym = batch.synth_batch(n1, 1472, SEEDS[1472], device=device)
    lensm = torch.full((n1,), 1472, dtype=torch.int32, device=device)
    flatm = paym.view(-1)
    encm = batch.pack_batch_varlen(tabm, flatm, lensm, "rudp7")
    tm = varlen_pair(tabm, flatm, lensm, "rudp7", encm.frames, encm.frame_off, None)
    ms_em, ms_dm = tm["encode"], tm["decode"]
    # algorithmic bytes: encode reads payload + len + table (1472 + 4 + 5), writes frame + offset
    # (1479 + 8); decode reads frame + offset, writes seq/ack/flags/ok/csum (8)
    out["varlen_1Mx1472"] = {
        "encode_GiB_s": n1 * 1472 / (ms_em / 1e3) / GIB, "encode_ms": ms_em,
        "encode_roofline_frac": n1 * (1472 + 9 + 1479 + 8) / (ms_em / 1e3) / 1e9 / HBM_PEAK_GBS,
        "decode_GiB_s": n1 * 1472 / (ms_dm / 1e3) / GIB, "decode_ms": ms_dm,
        "decode_roofline_frac": n1 * (1479 + 8 + 8) / (ms_dm / 1e3) / 1e9 / HBM_PEAK_GBS,
        "ms_by_form": tm,
        "note": "Python entry, sync-free (offset scan and device-side checks included); medians of "
                "7 interleaved rounds beside the eager-check and raw C-ABI forms"}
    # packed frames of valid multi-byte text (the fixed-length text leg's payload):
    # decode + get_payload()'s strict UTF-8 in the varlen tile, every payload checked
    text = ("é中😀aßЖ€𝄞" * 200).encode()[:1472]
    while True:
        try:
            text.decode()
            break
        except UnicodeDecodeError:
            text = text[:-1]
    text += b"x" * (1472 - len(text))
    flatt = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(device).repeat(n1)
    enct = batch.pack_batch_varlen(tabm, flatt, lensm, "rudp7")
    dt0 = batch.unpack_batch_varlen(enct.frames, enct.frame_off, "rudp7", utf8=True)
    ms_vt = time_loop(torch, lambda i: batch.unpack_batch_varlen(enct.frames, enct.frame_off, "rudp7", check=False,
                                                                  utf8=True, reuse=dt0), steps, 3) / steps
    dt0.check()
    out["varlen_decode_utf8_text_1Mx1472"] = {
        "ms": ms_vt, "roofline_frac": n1 * (1479 + 8 + 9) / (ms_vt / 1e3) / 1e9 / HBM_PEAK_GBS,
        "all_valid_and_verified": bool((dt0.valid == 1).all()) and bool((dt0.ok == 1).all()),
        "note": "packed rudp7 frames of valid multi-byte text through unpack_batch_varlen(utf8=True), sync-free"}
    del flatt, enct, dt0
    # ragged MTU-range lengths: uniform in [0, 2944] (mean 1472), packed; the tile
    # kernel takes byte tiles for this batch (the scan counts its overflowing
    # packet tiles), against the equal-length 1472-B leg above
    g = torch.Generator(device=device).manual_seed(SEEDS[1472])
    lensr = torch.randint(0, 2945, (n1,), dtype=torch.int32, device=device, generator=g)
    totr = int(lensr.sum().item())
    tabr, _ = batch.synth_batch(n1, 0, SEEDS[1472], device=device)
    flatr = torch.randint(0, 256, (totr,), dtype=torch.uint8, device=device, generator=g)
    encr = batch.pack_batch_varlen(tabr, flatr, lensr, "rudp7")
    tr = varlen_pair(tabr, flatr, lensr, "rudp7", encr.frames, encr.frame_off, None)
    ms_er, ms_dr = tr["encode"], tr["decode"]
    # the same ratio from interleaved rounds of the two encodes (sync-free, each
    # reusing its earlier outputs), so drift of the box between the two legs cancels
    re_ = batch.pack_batch_varlen(tabm, flatm, lensm, "rudp7", check=False)
    rr_ = batch.pack_batch_varlen(tabr, flatr, lensr, "rudp7", check=False)
    ratios = []
    for _ in range(7):
        te = time_loop(torch, lambda i: batch.pack_batch_varlen(tabm, flatm, lensm, "rudp7", check=False,
                                                                reuse=re_), steps, 1) / steps
        tg = time_loop(torch, lambda i: batch.pack_batch_varlen(tabr, flatr, lensr, "rudp7", check=False,
                                                                reuse=rr_), steps, 1) / steps
        ratios.append(tg / te * (n1 * 1472) / totr)
    re_.check()
    rr_.check()
    del re_, rr_, tabm, paym, lensm, flatm, encm
    out["varlen_1M_ragged_0_2944"] = {
        "payload_bytes": totr,
        "encode_GiB_s": totr / (ms_er / 1e3) / GIB, "encode_ms": ms_er,
        "encode_roofline_frac": (2 * totr + n1 * (9 + 7 + 8)) / (ms_er / 1e3) / 1e9 / HBM_PEAK_GBS,
        "encode_vs_equal_lengths": ms_er / ms_em * (n1 * 1472) / totr,
        "encode_vs_equal_lengths_interleaved": sorted(ratios)[len(ratios) // 2],
        "decode_GiB_s": totr / (ms_dr / 1e3) / GIB, "decode_ms": ms_dr,
        "decode_roofline_frac": (totr + n1 * (7 + 8 + 8)) / (ms_dr / 1e3) / 1e9 / HBM_PEAK_GBS,
        "ms_by_form": tr,
        "note": "lengths uniform in [0, 2944]; encode_vs_equal_lengths = time per payload byte over "
                "the equal 1472-B leg's; *_interleaved: the median of 7 rounds alternating the two "
                "encodes"}
    del tabr, flatr, lensr, encr
    # the proxy's retransmission check (proxy.py:90, 500-deep history) over the same 1M datagrams
    # sync-free (offsets checked on the device, rejected frames flagged 2) and with the
    # eager check (one device reduction + sync per call)
    ms_x = time_loop(torch, lambda i: batch.detect_retransmissions(enc.frames, frame_off=enc.frame_off,
                                                                   window=500, check=False), steps, 3) / steps
    ms_xe = time_loop(torch, lambda i: batch.detect_retransmissions(enc.frames, frame_off=enc.frame_off,
                                                                    window=500), steps, 3) / steps
    out["proxy_dedup_1M_window500"] = {"Mpkt_s": n1 / ms_x / 1e3, "ms": ms_x, "ms_eager_check": ms_xe,
                                       "note": "rudp_dedup_window_checked through the Python entry, sync-free"}
    del tab1, pay1, lens1, flat1, enc
    # the proxy-role caller's batch sizes (recvmmsg batches of <= 1024, proxy.py:126-154) and a
    # large socket batch: per-call cost of the sync-free entries back to back, and the latency of
    # one call waited for (launch + kernels + one synchronize)
    # fixed-length payloads off the 16-B grid (the reference's 1-char datagrams; 1000 B),
    # against the varlen path on the same bytes
    out.update(fixed_stride_legs(torch, batch, device, steps))
    out["small_batch_calls"] = small_batch_calls(torch, batch, device)
    # socket boundary: 1M one-character frames sendmmsg'd over loopback, recvmmsg'd into a
    # pinned ring and decoded on the GPU per received batch (rudp.netio)
    out["socket_e2e_1M_x_1char"] = socket_leg(torch, batch, device)
    # the proxy's role with many datagrams in flight: the batched relay (recvmmsg with
    # sources, GPU retransmission flags, sendmmsg) beside the per-datagram one
    out["relay_1char"] = relay_leg(torch, batch, device)
    # device-to-device streaming-copy ceiling, same byte count as one encode's payload:
    # the fastest copy in tools/sweep.py (one dwordx4 per thread, nt loads and stores,
    # rudpx_copy_vpt) and, for reference, the grid-stride copy (rudpx_copy, 65536 blocks)
    # (the copy kernels live in the diagnostics build, librudp_tools.so; the codec legs
    # above all ran librudp.so)
    from rudp import _native
    lib = _native.tools_lib(activate=False)
    a = w.sets[0][1]
    b = torch.empty_like(a)
    stream = torch.cuda.current_stream().cuda_stream
    ms = time_loop(torch, lambda i: lib.rudpx_copy_vpt(a.data_ptr(), b.data_ptr(), a.numel() // 16,
                                                       1, 1, stream), steps, 3) / steps
    ms_gs = time_loop(torch, lambda i: lib.rudpx_copy(a.data_ptr(), b.data_ptr(), a.numel() // 16,
                                                      65536, stream), steps, 3) / steps
    out["d2d_copy_ceiling_GBs"] = 2 * a.numel() / (ms / 1e3) / 1e9
    out["d2d_copy_gridstride_GBs"] = 2 * a.numel() / (ms_gs / 1e3) / 1e9
    del w, a, b
    torch.cuda.empty_cache()
    return out


def fixed_stride_legs(torch, batch, device, steps, rounds=5):
    """Fixed-length batches that miss the fixed-length tiles (payloads not a multiple
    of 16 B), against the varlen path on the same bytes: 1M one-character rudp5
    datagrams -- the reference's own traffic, utils/reliableUDP.py:11, :60, framed by
    utils/packet.py:60-65 + :80-81 -- encoded (pack_batch on [N, 1] payloads) and
    decoded with get_payload()'s strict UTF-8 (unpack_batch(utf8=True),
    utils/packet.py:73), and 1M x 1000 B rudp7 encoded.  Both forms through the raw
    C ABI with preallocated outputs (rudp_encode / rudp_decode_utf8 against
    rudp_encode_varlen_checked / rudp_decode_varlen_utf8: at ~10 us per call the
    Python entries' allocations would be the clock), and through the Python entries;
    rounds of the forms interleaved, medians.  The fixed frames are compared with
    the varlen frames (pinned by the reference goldens) outside the clock."""
    import ctypes
    from rudp import _native
    lib = _native.lib()
    sp = torch.cuda.current_stream().cuda_stream
    di = device.index or 0
    out = {}
    n = 1 << 20
    for L, layout in ((1, "rudp5"), (1000, "rudp7")):
        H = batch.layout_header_len(layout)
        F = L + H
        tab, pay = batch.synth_batch(n, L, SEEDS[1472], device=device)
        lens = torch.full((n,), L, dtype=torch.int32, device=device)
        flat = pay.view(-1)
        want_cs = H == 5
        fr, cs = batch.pack_batch(tab, pay, layout, want_csum=want_cs)
        v = batch.pack_batch_varlen(tab, flat, lens, layout, want_csum=want_cs, check=False)
        v.check()
        same = torch.equal(fr.view(-1), v.frames) and (
            cs is None or torch.equal(cs.view(torch.int16), v.csum.view(torch.int16)))
        rb = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                               flags=tab.flags.data_ptr(), payload=flat.data_ptr(), len=None, payload_off=None)
        rv = _native.RudpBatch(n=n, payload_len=L, reserved=0, seq=tab.seq.data_ptr(), ack=tab.ack.data_ptr(),
                               flags=tab.flags.data_ptr(), payload=flat.data_ptr(), len=lens.data_ptr(),
                               payload_off=None)
        vf, vo = torch.empty_like(v.frames), torch.empty_like(v.frame_off)
        vc = torch.empty((n,), dtype=torch.uint16, device=device) if want_cs else None
        st = torch.empty((1,), dtype=torch.int32, device=device)
        fns = {
            "encode_fixed_abi": lambda i: lib.rudp_encode(ctypes.byref(rb), fr.data_ptr(),
                                                          cs.data_ptr() if want_cs else None, H, di, sp),
            "encode_varlen_abi": lambda i: lib.rudp_encode_varlen_checked(
                ctypes.byref(rv), flat.numel(), vf.data_ptr(), vf.numel(), vo.data_ptr(),
                vc.data_ptr() if want_cs else None, st.data_ptr(), H, di, sp),
            "encode_fixed_python": lambda i: batch.pack_batch(tab, pay, layout, out=fr, csum_out=cs,
                                                              want_csum=want_cs),
            "encode_varlen_python": lambda i: batch.pack_batch_varlen(tab, flat, lens, layout, want_csum=want_cs,
                                                                      check=False, reuse=v),
        }
        if L == 1:
            o = [torch.empty((n,), dtype=dt, device=device) for dt in
                 (torch.uint16, torch.uint16, torch.uint8, torch.uint8, torch.uint16, torch.uint8)]
            ov = [torch.empty_like(t) for t in o]
            fns["decode_utf8_fixed_abi"] = lambda i: lib.rudp_decode_utf8(
                fr.data_ptr(), None, F, n, cs.data_ptr(), *[t.data_ptr() for t in o[:5]], None, o[5].data_ptr(),
                H, di, sp)
            fns["decode_utf8_varlen_abi"] = lambda i: lib.rudp_decode_varlen_utf8(
                v.frames.data_ptr(), v.frames.numel(), v.frame_off.data_ptr(), F, n, v.csum.data_ptr(),
                *[t.data_ptr() for t in ov], None, H, di, sp)
            fns["decode_utf8_fixed_python"] = lambda i: batch.unpack_batch(fr, layout, csum=cs, utf8=True)
        per = {k: [] for k in fns}
        for r in range(rounds):
            for k, fn in fns.items():
                per[k].append(time_loop(torch, fn, steps, 2 if r == 0 else 1) / steps)
        ms = {k: sorted(x)[len(x) // 2] for k, x in per.items()}
        if int(st.item()):
            raise RuntimeError("the raw varlen encode rejected the bench batch")
        same = same and torch.equal(vf, v.frames)
        enc_bytes = n * algorithmic_bytes_encode(L)  # read L + 5, write L + 7 (frame + csum, or rudp7 frame)
        out[f"encode_1Mx{L}_fixed"] = {
            "ms": ms["encode_fixed_abi"], "vs_varlen_same_bytes": ms["encode_fixed_abi"] / ms["encode_varlen_abi"],
            "roofline_frac": enc_bytes / (ms["encode_fixed_abi"] / 1e3) / 1e9 / HBM_PEAK_GBS,
            "Mpkt_s": n / ms["encode_fixed_abi"] / 1e3, "layout": layout,
            "frames_equal_varlen_path": bool(same), "ms_by_form": ms if L != 1 else
            {k: x for k, x in ms.items() if k.startswith("encode")}}
        if L == 1:
            valid_ok = bool((o[5] == 1).all()) and bool((o[3] == 1).all()) and torch.equal(
                o[0].view(torch.int16), tab.seq.view(torch.int16))
            dec_bytes = n * (F + 2 + 6 + 2 + 1)  # read frame + sideband csum; write seq/ack/flags/ok, csum, valid
            out["decode_utf8_1Mx1_fixed"] = {
                "ms": ms["decode_utf8_fixed_abi"],
                "vs_varlen_same_bytes": ms["decode_utf8_fixed_abi"] / ms["decode_utf8_varlen_abi"],
                "roofline_frac": dec_bytes / (ms["decode_utf8_fixed_abi"] / 1e3) / 1e9 / HBM_PEAK_GBS,
                "Mpkt_s": n / ms["decode_utf8_fixed_abi"] / 1e3, "layout": layout,
                "all_valid_verified_fields_equal": valid_ok,
                "ms_by_form": {k: x for k, x in ms.items() if k.startswith("decode")}}
        del tab, pay, lens, flat, fr, cs, v, vf, vo, vc
    out["note"] = ("fixed-length payloads of 1 and 1000 B (not multiples of 16): the varlen tile kernels with "
                   "implicit offsets (one launch, no scan), against rudp_encode_varlen_checked / "
                   "rudp_decode_varlen_utf8 on the same bytes; *_abi: raw C-ABI calls with preallocated "
                   "outputs (the ratio is theirs), *_python: the Python entries; medians of 5 interleaved "
                   "rounds; 1-char batches are 7-27 MB, resident in the Infinity Cache for both forms")
    torch.cuda.empty_cache()
    return out


def baseline_summary(line):
    """A compact digest of the BASELINE-config legs (C2, C3, C4, C5 on
    one GPU) and the decode legs, appended as the LAST key of the JSON line so a
    reader that keeps only the line's tail still sees each one with its ms,
    roofline fraction and reference-digest result."""
    lg = line.get("legs") or {}

    def pick(key, ms="ms", frac="roofline_frac", chk=None, extra=()):
        d = lg.get(key)
        if not isinstance(d, dict):
            return None
        r = {"ms": round(d[ms], 4) if d.get(ms) is not None else None,
             "frac": round(d[frac], 3) if d.get(frac) is not None else None}
        if chk:
            r["digests"] = d.get(chk)
        for k in extra:
            if k in d:
                r[k] = round(d[k], 3) if isinstance(d[k], float) else d[k]
        return r
    out = {
        "headline_C4_encode_1Mx1472": {"ms": round(line["roofline"]["kernel_ms_per_launch"], 4),
                                       "frac": round(line["roofline"]["frac"], 3),
                                       "matches_reference": line["config"].get("matches_reference")},
        "C2_encode_1Mx1024": pick("encode_1Mx1024", chk="chunks_matching_reference_digests"),
        "C3_encode_1Mx64": pick("encode_1Mx64", chk="chunks_matching_reference_digests",
                                extra=("frac_of_copy_same_bytes",)),
        "C4_roundtrip_1Mx1472": pick("roundtrip_1Mx1472", chk="chunks_matching_reference_digests",
                                     extra=("decode_fields_equal_inputs",)),
        "C5_encode_16Mx1472_1gpu": pick("encode_16Mx1472_C5_1gpu", chk="chunks_matching_reference_digests"),
        "decode_verify_1Mx1472": pick("decode_verify_1Mx1472"),
        "decode_utf8_ascii_1Mx1472": pick("decode_utf8_1Mx1472", extra=("all_valid_and_verified",)),
        "decode_utf8_multibyte_text_1Mx1472": pick("decode_utf8_1Mx1472_multibyte_text",
                                                   extra=("all_valid_and_verified",)),
        "varlen_decode_utf8_text_1Mx1472": pick("varlen_decode_utf8_text_1Mx1472",
                                                extra=("all_valid_and_verified",)),
        "encode_1Mx1_fixed": pick("encode_1Mx1_fixed", extra=("vs_varlen_same_bytes", "frames_equal_varlen_path")),
        "decode_utf8_1Mx1_fixed": pick("decode_utf8_1Mx1_fixed",
                                       extra=("vs_varlen_same_bytes", "all_valid_verified_fields_equal")),
        "encode_1Mx1000_fixed": pick("encode_1Mx1000_fixed",
                                     extra=("vs_varlen_same_bytes", "frames_equal_varlen_path")),
        "varlen_ragged_encode_ms": round(lg["varlen_1M_ragged_0_2944"]["encode_ms"], 4)
        if "varlen_1M_ragged_0_2944" in lg else None,
        "varlen_ragged_decode_frac": round(lg["varlen_1M_ragged_0_2944"]["decode_roofline_frac"], 3)
        if "varlen_1M_ragged_0_2944" in lg else None,
    }
    c5 = lg.get("c5_16Mx1472_strong")
    if c5:
        out["C5_strong"] = {"ms": round(c5["ms"], 4), "GiB_s": round(c5["GiB_s"], 1), "n_gpus": c5["n_gpus"],
                            "per_gpu_frac": round(c5["per_gpu_roofline_frac"], 3),
                            "digests": f"{c5['chunks_matching_reference_digests']}/16"
                            if c5["packets_total"] == C5_PACKETS else c5["chunks_matching_reference_digests"]}
    return {k: v for k, v in out.items() if v is not None}


def e2e_host_decode_legs(torch, batch, frames, n, L, reps=3):
    """The receive side from host memory (north_star: the path starts and ends in a
    socket buffer), through the Python entries: the frames in pinned host memory,
    staged through the GPU by the *_host pipeline, outputs back in host arrays.
    1M x 1472 B rudp7 frames: parse + verify + get_payload()'s strict UTF-8
    (rudp_decode_host with h_valid; utils/reliableUDP.py:118-121, utils/packet.py:73);
    1M one-character rudp5 datagrams packed back to back (a recvmmsg batch): the
    same through rudp_decode_varlen_host, and their encode from packed host
    payloads (rudp_encode_varlen_host)."""
    import numpy as np
    out = {}
    d = batch.unpack_batch(frames, "rudp7", utf8=True)  # first calls: slots, pinned outputs, warm
    d = batch.unpack_batch(frames, "rudp7", utf8=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        d = batch.unpack_batch(frames, "rudp7", utf8=True)
    dt = (time.perf_counter() - t0) / reps
    out["e2e_host_decode_utf8_1Mx1472"] = {
        "GiB_s": n * L / dt / GIB, "ms": dt * 1e3, "pcie_GBs_h2d": n * (L + 7) / dt / 1e9,
        "all_valid_and_verified": bool((d.valid == 1).all()) and bool((d.ok == 1).all()),
        "note": "pinned host frames -> unpack_batch(numpy, utf8=True): rudp_decode_host (H2D, fused "
                "decode + strict UTF-8 kernel, D2H of seq/ack/flags/ok/csum/valid on three streams), "
                "outputs into pinned arrays from torch's caching host allocator"}
    del d
    out.update(e2e_host_varlen_leg(torch, batch, 5))
    return out


def e2e_host_varlen_leg(torch, batch, reps=3):
    """1M one-character rudp5 datagrams packed back to back in pinned host memory
    (a recvmmsg / sendmmsg batch): decode + UTF-8 through rudp_decode_varlen_host
    and encode from packed payloads through rudp_encode_varlen_host, by the Python
    entries."""
    import numpy as np
    out = {}
    m = 1 << 20
    pin = lambda k, dt: torch.empty(k, dtype=dt, pin_memory=True).numpy()  # noqa: E731
    rng = np.random.default_rng(0x5EED0004)
    seq = pin(m, torch.uint16)
    seq[:] = np.arange(m, dtype=np.uint16)
    ack, flg = pin(m, torch.uint16), pin(m, torch.uint8)
    ack[:] = rng.integers(0, 1 << 16, m, dtype=np.uint16)
    flg[:] = 0x40
    pay = pin(m, torch.uint8)
    pay[:] = rng.integers(0x20, 0x7F, m, dtype=np.uint8)
    lens = pin(m, torch.int32)
    lens[:] = 1
    enc = batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True)
    fr, fo, cs = pin(enc.frames.size, torch.uint8), pin(m + 1, torch.int64), pin(m, torch.uint16)
    fr[:], fo[:], cs[:] = enc.frames, enc.frame_off, enc.csum
    # untimed calls of each first: the per-packet outputs come from torch's caching
    # pinned allocator, whose first blocks of a size are fresh hipHostMallocs (a
    # call allocates its outputs while the previous call's result is alive; the
    # bench measured 1.98, 1.46, 0.69 ms for the 3rd-5th encode calls)
    for _ in range(4):
        enc = batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True, out=fr)
    te = []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc = batch.pack_batch_varlen((seq, ack, flg), pay, lens, "rudp5", want_csum=True, out=fr)
        te.append(time.perf_counter() - t0)
    for _ in range(4):
        dv = batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True)
    td = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dv = batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True)
        td.append(time.perf_counter() - t0)
    ok = bool((dv.ok == 1).all()) and bool((dv.valid == 1).all()) and bool(np.array_equal(dv.seq, seq))
    tr = []
    for _ in range(reps):
        t0 = time.perf_counter()
        batch.unpack_batch_varlen(fr, fo, "rudp5", csum=cs, utf8=True, reuse=dv, check=False)
        tr.append(time.perf_counter() - t0)
    ok = ok and bool((dv.ok == 1).all()) and bool((dv.valid == 1).all())
    calls = {"encode": [round(t * 1e3, 3) for t in te], "decode": [round(t * 1e3, 3) for t in td]}
    te, td, tr = (sorted(t)[len(t) // 2] for t in (te, td, tr))
    out["e2e_host_varlen_1M_x_1char"] = {
        "decode_utf8_Mpkt_s": m / td / 1e6, "decode_ms": td * 1e3, "decode_reuse_ms": tr * 1e3,
        "encode_Mpkt_s": m / te / 1e6, "encode_ms": te * 1e3, "calls_ms": calls,
        "decoded_all_valid_and_verified": ok,
        "note": "pinned host buffers: unpack_batch_varlen(numpy, csum, utf8=True) = rudp_decode_varlen_host "
                "(6 B frames + 8 B offsets + 2 B sideband checksum per datagram up, 10 B of fields down); "
                "pack_batch_varlen(numpy, out=pinned) = rudp_encode_varlen_host (10 B up, 6 B frame + 8 B "
                "offset + 2 B checksum down); per-packet outputs from torch's caching pinned allocator "
                "(decode_reuse_ms: into the previous result's arrays, reuse=); medians of 5 calls after 4 untimed ones"}
    return out


def small_batch_calls(torch, batch, device, sizes=(1024, 65536), reps=200):
    """Per-call times at the batch sizes a reference caller produces: one-character
    rudp5 datagrams (utils/reliableUDP.py:11), n per call.  ``us_per_call``: the
    median of 5 runs of `reps` back-to-back sync-free calls on one stream (HIP
    events, outputs reused).  ``us_latency``: wall time of one call plus its
    synchronize (what a caller that waits for every batch sees), median of `reps`
    rounds in which every size and op (and ``floor``: a one-element torch add, the
    box's launch + synchronize floor) takes one turn, so drift of the host or GPU
    state over the leg falls on all of them alike; ``us_latency_event``: the same
    call waited for by an event recorded behind it instead of a device-wide
    synchronize."""
    ops, lasts = {}, []
    for n in sizes:
        tab, pay = batch.synth_batch(n, 1, SEEDS[1472], device=device)
        lens = torch.ones(n, dtype=torch.int32, device=device)
        flat = pay.view(-1)
        enc = batch.pack_batch_varlen(tab, flat, lens, "rudp5", want_csum=True)
        last = {"e": enc, "d": batch.unpack_batch_varlen(enc.frames, enc.frame_off, "rudp5", csum=enc.csum),
                "u": batch.unpack_batch_varlen(enc.frames, enc.frame_off, "rudp5", csum=enc.csum, utf8=True)}
        lasts.append(last)

        def mk(last=last, tab=tab, flat=flat, lens=lens, enc=enc):
            return {
                "encode": lambda: last.__setitem__("e", batch.pack_batch_varlen(
                    tab, flat, lens, "rudp5", want_csum=True, check=False, reuse=last["e"])),
                "decode": lambda: last.__setitem__("d", batch.unpack_batch_varlen(
                    enc.frames, enc.frame_off, "rudp5", csum=enc.csum, check=False, reuse=last["d"])),
                "decode_utf8": lambda: last.__setitem__("u", batch.unpack_batch_varlen(
                    enc.frames, enc.frame_off, "rudp5", csum=enc.csum, check=False, reuse=last["u"], utf8=True)),
                "dedup_window500": lambda: batch.detect_retransmissions(enc.frames, frame_off=enc.frame_off,
                                                                        window=500, check=False),
            }
        ops[n] = mk()
    one = torch.zeros(1, device=device)
    floor = lambda: one.add_(1)  # noqa: E731
    out = {f"n{n}": {} for n in sizes}
    for n in sizes:
        for name, fn in ops[n].items():
            per = sorted(time_loop(torch, lambda i: fn(), reps, 5) / reps * 1e3 for _ in range(5))
            out[f"n{n}"][name] = {"us_per_call": per[2], "Mpkt_s_back_to_back": n / per[2]}
    turns = [("floor", None, floor)] + [(name, n, fn) for n in sizes for name, fn in ops[n].items()]
    lat = {(name, n): [] for name, n, _ in turns}
    lat_ev = {(name, n): [] for name, n, _ in turns}
    ev = torch.cuda.Event()
    for _ in range(reps):
        for name, n, fn in turns:
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            lat[(name, n)].append((time.perf_counter() - t0) * 1e6)
            t0 = time.perf_counter()
            fn()
            ev.record()
            ev.synchronize()
            lat_ev[(name, n)].append((time.perf_counter() - t0) * 1e6)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    for name, n, _ in turns:
        row = out.setdefault("floor", {}) if n is None else out[f"n{n}"].setdefault(name, {})
        row.update({"us_latency": med(lat[(name, n)]), "us_latency_p10_p90": [sorted(lat[(name, n)])[reps // 10],
                                                                             sorted(lat[(name, n)])[reps * 9 // 10]],
                    "us_latency_event": med(lat_ev[(name, n)])})
    for last in lasts:
        last["e"].check()
        last["d"].check()
    out["note"] = ("1-char rudp5 datagrams; Python entries, sync-free, outputs reused; us_per_call: back-to-back "
                   "calls on one stream (HIP events); us_latency: one call + torch.cuda.synchronize (wall), "
                   "every size and op (and the floor: a one-element torch add) taking turns each round; "
                   "us_latency_event: the call + an event recorded behind it, waited for")
    return out


def socket_leg(torch, batch, device, n=1 << 20):
    import socket
    import threading
    from rudp import netio
    tab, pay = batch.synth_batch(n, 1, SEEDS[1472], device=device)
    enc = batch.pack_batch_varlen(tab, pay.view(-1), torch.ones(n, dtype=torch.int32, device=device),
                                  "rudp7")
    frames, off = enc.frames.cpu().numpy(), enc.frame_off.cpu().numpy()
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 27)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    recv = netio.BatchReceiver(rx, max_msgs=1 << 16, slot_bytes=64)
    port = rx.getsockname()[1]
    got = good = batches = 0
    sender = threading.Thread(target=lambda: netio.send_batch(tx, frames, off, "127.0.0.1", port))
    t0 = time.perf_counter()
    sender.start()
    while True:
        k = recv.recv(timeout_ms=300)
        if k == 0:
            break
        dec, _, _ = recv.decode("rudp7", device)
        good += int((dec.ok == 1).sum().item())
        got += k
        batches += 1
    dt = time.perf_counter() - t0 - 0.3  # minus the final idle timeout
    sender.join()
    rx.close()
    tx.close()
    return {"received": got, "verified": good, "batches": batches, "wall_s": dt,
            "Mpkt_s": got / dt / 1e6,
            "note": "loopback kernel UDP stack bound; sendmmsg/recvmmsg 1024 per call"}


def relay_peer(peer_dir: str) -> None:
    """The relay leg's client and server ends, in a process of their own (as
    client.py and server.py are the reference's own processes around proxy.py):
    bind a sink, report its port, read the relay's port, blast the frames in
    4096-datagram sendmmsg bursts (at most 32K datagrams in flight) and count
    what reaches the sink.  Prints one JSON line.  No GPU work."""
    import socket
    import threading

    import numpy as np
    from rudp import _native, netio
    _native.lib()  # load librudp (and torch, which it binds to) before any clock starts
    frames = np.load(Path(peer_dir) / "frames.npy")
    off = np.load(Path(peer_dir) / "off.npy")
    n = off.shape[0] - 1
    sink = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sink.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
    sink.bind(("127.0.0.1", 0))
    print(f"SINK {sink.getsockname()[1]}", flush=True)
    relay_port = int(sys.stdin.readline().split()[1])
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    got = [0]
    rbuf, roff = np.empty((1 << 16) * 64, np.uint8), np.empty((1 << 16) + 1, np.int64)

    def drain():
        while True:
            k = netio.recv_batch(sink, rbuf, roff, slot_bytes=64, timeout_ms=500)
            if k == 0:
                break
            got[0] += k
    t = threading.Thread(target=drain)
    t.start()
    t0 = time.perf_counter()
    for a in range(0, n, 4096):
        while a - got[0] > 32768 and t.is_alive():
            time.sleep(20e-6)
        b = min(n, a + 4096)
        netio.send_batch(tx, frames, off[a:b + 1], "127.0.0.1", relay_port)
    t.join()
    dt = time.perf_counter() - t0 - 0.5  # minus the sink's final idle timeout
    print(json.dumps({"got": got[0], "wall_s": dt}), flush=True)


def relay_leg(torch, batch, device):
    """Datagrams through rudp.relay.Relay in proxy.py's role (proxy.py:126-154):
    a client blasts one-character frames (sendmmsg) at the relay, which forwards
    them to a sink in the server's place; the sink counts what arrives.  The
    client and sink run in a child process (relay_peer), the relay here, as the
    reference runs client.py, proxy.py and server.py as processes of their own.
    Batched relay over 256K datagrams, per-datagram relay over 32K; datagrams/s
    from the first send to the last datagram at the sink, and the relay's
    counters (every datagram distinct: no retransmissions).  Loopback UDP may
    drop under load; the received counts say how many made it."""
    import socket
    import subprocess
    import tempfile

    import numpy as np
    from rudp.relay import Relay
    out = {}
    for name, n, batched in (("batched", 1 << 18, True), ("per_datagram", 1 << 15, False)):
        tab, pay = batch.synth_batch(n, 1, SEEDS[1472], device=device)
        tab.seq.copy_(torch.arange(n, device=device).to(torch.int32).to(torch.uint16))  # distinct frames
        enc = batch.pack_batch_varlen(tab, pay.view(-1), torch.ones(n, dtype=torch.int32, device=device), "rudp5")
        with tempfile.TemporaryDirectory() as tmp:
            np.save(Path(tmp) / "frames.npy", enc.frames.cpu().numpy())
            np.save(Path(tmp) / "off.npy", enc.frame_off.cpu().numpy())
            peer = subprocess.Popen([sys.executable, str(Path(__file__).resolve()), "--relay-peer", tmp],
                                    stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            sink_port = int(peer.stdout.readline().split()[1])
            relay = Relay(sink_port, batched=batched, device=device if batched else None, keep_log=False)
            relay.sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
            relay.start()
            peer.stdin.write(f"RELAY {relay.port}\n")
            peer.stdin.flush()
            res = json.loads(peer.stdout.readline())
            peer.wait(timeout=60)
            relay.stop()
        out[name] = {"sent": n, "relayed_to_sink": res["got"], "wall_s": res["wall_s"],
                     "Mpkt_s": res["got"] / res["wall_s"] / 1e6, "relay_batches": relay.batches,
                     "relay_stats": relay.stats}
    out["note"] = ("client + sink in a child process -> relay (this process) -> sink over loopback, 1-char "
                   "frames in 4096-datagram sendmmsg bursts (at most 32K datagrams in flight); relay without "
                   "its datagram log; batched: recvmmsg of up to 1024 with sources into a pinned ring, "
                   "librudp's dedup stream (500-deep history on the device, no wait per batch), sendmmsg to "
                   "per-datagram destinations on a forwarding thread")
    return out


def config1_loopback():
    """BASELINE config 1: client -> proxy -> server over 127.0.0.1, stop-and-wait, 1 char per
    datagram (rudp.transport over the drop-in Packet, rudp.relay in proxy.py's role; no
    GPU).  Message = bin/input.txt (recorded in tests/golden/wire_trace.json), plus a
    2000-char message for a rate; the relay's counters follow proxy.py:79-94."""
    import threading
    from rudp.relay import Relay
    from rudp.transport import ReliableUDP
    msg = json.loads((REPO / "tests" / "golden" / "wire_trace.json").read_text())["message"]
    out = {}
    for name, m in (("input_txt", msg), ("2000_chars", "x" * 2000)):
        server = ReliableUDP().create()
        server.bind("127.0.0.1", 0)
        relay = Relay(server.socket.getsockname()[1])
        relay.start()
        got = {}
        t = threading.Thread(target=lambda: got.setdefault("m", server.recv()), daemon=True)
        t.start()
        time.sleep(0.05)  # recv() flushes its socket first: let it get there
        client = ReliableUDP(timeout=1).create()
        t0 = time.perf_counter()
        client.send(m, "127.0.0.1", relay.port)
        t.join(timeout=60)
        dt = time.perf_counter() - t0
        relay.stop()
        client.close()
        server.close()
        out[name] = {"ok": got.get("m") == m, "wall_ms": dt * 1e3, "chars_per_s": len(m) / dt,
                     "path": "client -> relay (proxy.py role) -> server", "relay_stats": relay.stats}
    return out


def device_record(torch, rank, local_rank, dev_index):
    """The GPU this rank drives: HIP device index, PCI domain:bus:device, UUID."""
    p = torch.cuda.get_device_properties(dev_index)
    pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return {"rank": rank, "local_rank": local_rank, "device_index": dev_index, "pci": pci,
            "uuid": str(getattr(p, "uuid", "")), "name": p.name}


def read_pmc_traffic(L, n):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    path = REPO / "profiles" / "pmc_encode.json"
    if not path.exists():
        return None, None
    d = json.loads(path.read_text())
    if d.get("L") != L or d.get("n") != n:
        return None, None
    return d.get("hbm_bytes_per_launch"), str(path.relative_to(REPO))


def launch_ranks(n: int, argv, dry_run: bool = False) -> int:
    """`python -m torch.distributed.run --nproc-per-node n` over this script with
    the same arguments, rendezvous on 127.0.0.1 at a free port, as a child process
    whose stdout is ours (rank 0's JSON line passes straight through)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]
    if dry_run:
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU (weak scaling)")
    ap.add_argument("--total-packets", type=int, default=0,
                    help="strong scaling: split this many packets over the ranks (C5: 16777216)")
    ap.add_argument("--payload", type=int, default=1472)
    ap.add_argument("--layout", default="rudp7", choices=["rudp5", "rudp7"])
    ap.add_argument("--no-legs", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="CPU baseline processes (0: one per usable CPU, see usable_cpus())")
    ap.add_argument("--cpu-packets", type=int, default=1 << 15,
                    help="packets per CPU worker at 16 workers, scaled to keep the total (16 x 32768 x ~26 us: about 14 s of CPU work)")
    ap.add_argument("--share-device", action="store_true",
                    help="testing only: every rank uses cuda:0 and gloo (rehearse N>1 on one GPU)")
    ap.add_argument("--dist", action="store_true",
                    help="testing only: the N>1 code path (process group, collectives, C5 strong leg) "
                         "also at N = 1, so the RCCL branch runs on a one-GPU box")
    ap.add_argument("--c5-packets", type=int, default=0,
                    help="testing only: packets of the C5 strong leg (default 16M)")
    ap.add_argument("--relay-peer", metavar="DIR", help=argparse.SUPPRESS)  # relay_leg's child process
    ap.add_argument("--print-launch", action="store_true",
                    help="testing only: with --gpus N > 1 and no launcher, print the rank launcher's "
                         "command instead of running it")
    args = ap.parse_args()
    if args.relay_peer:
        relay_peer(args.relay_peer)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start torch.distributed.run as a CHILD process
        # (before anything touches the GPU; never exec) with this command line,
        # one rank per GPU, and hand back its exit status -- rank 0 prints the line
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.print_launch))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = args.cpu_workers or usable_cpus()["usable"]
        cpu = cpu_baseline(args.payload, max(256, args.cpu_packets * 16 // workers), workers)
        cpu["config1_loopback"] = config1_loopback()

    import torch
    import torch.distributed as dist
    from rudp import batch

    dev_index = 0 if args.share_device else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    distributed = world > 1 or args.dist
    if distributed:
        if args.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    # which physical GPU each rank drives: index, PCI address and UUID, gathered to
    # rank 0 for the line; without --share-device every rank must hold its own GPU
    devices = [device_record(torch, rank, local_rank, dev_index)]
    if distributed:
        gathered = [None] * world
        dist.all_gather_object(gathered, devices[0])
        devices = gathered
    distinct = len({d["pci"] for d in devices}) == len(devices)
    if world > 1 and not args.share_device and not distinct:
        raise SystemExit(f"ranks share a GPU without --share-device: {devices}")

    n, L = args.packets, args.payload
    first = rank * n
    if args.total_packets:
        first, n = rank_slice(rank, world, args.total_packets)
    seed = SEEDS.get(L, 0x5EED0004)
    w = Workload(torch, batch, n, L, args.layout, first, seed, device)
    nsets = len(w.sets)
    for i in range(args.warmup):
        w.encode(batch, i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    stop = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    start.record()
    for i in range(args.steps):
        w.encode(batch, args.warmup + i)
    stop.record()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # every rank's kernel time: the roofline is the slowest GPU's
    wall_max, rank_kernel_ms = over_ranks(torch, dist, world, args.share_device, device, wall,
                                          start.elapsed_time(stop))
    kernel_ms = max(rank_kernel_ms)

    # the timed frames against the reference (BASELINE configs 2-4 by payload size), outside the clock
    head_chk = verify_digests(w, {1024: "C2", 64: "C3", 1472: "C4"}.get(L, ""), first, n)
    del w
    torch.cuda.empty_cache()
    extra = legs(torch, batch, device, max(10, args.steps // 2)) if (
        rank == 0 and not distributed and not args.no_legs) else None
    if distributed and not args.no_legs and not args.total_packets:
        # BASELINE config 5 beside the weak-scaling headline: 16M x 1472 B split
        # over the ranks (strong scaling), same barrier + max-over-ranks clock.
        extra = {"c5_16Mx1472_strong": c5_strong_leg(torch, dist, batch, device, world, rank,
                                                      args.layout, args.share_device,
                                                      total=args.c5_packets or None)}

    if rank == 0:
        # strong scaling: the ranks' slices add up to --total-packets (rank_slice)
        total_payload = (args.total_packets or world * n) * L * args.steps
        per_launch_s = kernel_ms / 1e3 / args.steps  # the slowest rank's
        achieved = n * algorithmic_bytes_encode(L) / per_launch_s / 1e9
        traffic, traffic_src = read_pmc_traffic(L, n)
        line = {
            "metric": "GiB/s payload checksummed+framed (device-resident), 1/2/4/8 MI355X",
            "value": total_payload / wall_max / GIB,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.total_packets else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (on-device splitmix64, ASCII payloads)",
            "config": {
                "workload": f"rudp_encode {args.layout}: checksum+frame {n} x {L} B packets per GPU "
                            f"(BASELINE config 4/5 shape), device-resident",
                "packets_per_gpu": n, "payload_bytes": L, "layout": args.layout,
                "global_batch": world * n, "parallelism": f"packet-slice x{world}, no collective",
                "buffer_sets": nsets,
                "matches_reference": None if head_chk is None else head_chk[0] == head_chk[1] > 0,
                "devices": devices,
                "distinct_gpus": distinct,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": n * algorithmic_bytes_encode(L),
                "kernel_ms_per_launch": per_launch_s * 1e3,
                "kernel_ms_per_launch_by_rank": [k / args.steps for k in rank_kernel_ms],
                "rank_note": "achieved/frac from the slowest rank's HIP-event kernel time",
                "traffic_source": traffic_src,
            },
            "cpu_baseline": cpu,
        }
        if extra is not None:
            line["legs"] = extra
            ceiling = extra.get("d2d_copy_ceiling_GBs")
            if ceiling:
                line["roofline"]["measured_copy_ceiling_GBs"] = ceiling
                line["roofline"]["frac_of_copy_ceiling"] = achieved / ceiling
        line["baseline_legs"] = baseline_summary(line)  # last: visible in any tail of the line
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
