"""Packet-array slicing across GPUs: no exchange step.

Virtual shards on one CPU and a world_size-2 gloo run of the same slicing
rule that bench.py applies per rank (rank r frames packets [r*N, (r+1)*N)).
Concatenated shard outputs must equal the unsharded batch bit for bit; for
variable-length batches the shards' offsets, rebased by rudp.shard, must
equal the unsharded offsets.
"""
import hashlib
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import codec_c, codec_np, synth
from rudp import shard

SEED, N, L = 0x5EED0005, 4096, 1472


def shard_range(rank, world, n_total):
    """bench.py's slicing rule (the one its ranks use for C5)."""
    return bench.rank_slice(rank, world, n_total)


def test_rank_slice_rule():
    assert [bench.rank_slice(r, 8, 1 << 24) for r in (0, 7)] == [(0, 1 << 21), (7 << 21, 1 << 21)]
    # any world size: the slices tile [0, total) in rank order, sizes within one packet
    for world in (1, 2, 3, 5, 6, 7, 8, 16):
        for total in (0, 1, 7, 1000, 1 << 24):
            sl = [bench.rank_slice(r, world, total) for r in range(world)]
            assert sl[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert sum(n for _, n in sl) == total
            assert max(n for _, n in sl) - min(n for _, n in sl) <= 1


@pytest.mark.parametrize("world", [3, 5, 6])
def test_uneven_virtual_shards_concatenate_to_unsharded(world):
    full_fr, _ = codec_c.encode(*synth.synth(SEED, 0, 1000, 64), 7)
    parts = [codec_c.encode(*synth.synth(SEED, *bench.rank_slice(r, world, 1000), 64), 7)[0]
             for r in range(world)]
    assert np.array_equal(np.concatenate(parts), full_fr)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_virtual_shards_concatenate_to_unsharded(world):
    full_fr, full_cs = codec_c.encode(*synth.synth(SEED, 0, N, L), 7)
    parts = []
    for r in range(world):
        first, n = shard_range(r, world, N)
        fr, cs = codec_c.encode(*synth.synth(SEED, first, n, L), 7)
        parts.append((fr, cs))
    assert np.array_equal(np.concatenate([p[0] for p in parts]), full_fr)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), full_cs)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard_range(rank, world, N)
    fr, _ = codec_c.encode(*synth.synth(SEED, first, n, L), 7)
    digest = hashlib.sha256(fr.tobytes()).digest()
    gathered = [None] * world
    dist.all_gather_object(gathered, (first, n, digest))
    import torch
    t = torch.tensor([float(n)])
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # bench.py aggregates units over ranks
    if rank == 0:
        out.put((gathered, float(t.item())))
    dist.destroy_process_group()


def test_gloo_world2_shards_match_unsharded():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert total == N
    full_fr, _ = codec_c.encode(*synth.synth(SEED, 0, N, L), 7)
    per = N // 2
    for first, n, digest in gathered:
        assert digest == hashlib.sha256(full_fr[first:first + n].tobytes()).digest()


def test_payload_spans_is_the_start_end_pair():
    """unpack_batch_varlen's lazy payload spans behave as (start, end)."""
    import torch
    from rudp.batch import PayloadSpans
    off = torch.tensor([0, 3, 10, 10, 17, 30], dtype=torch.int64)
    sp = PayloadSpans(off, 7)
    start, end = sp
    assert torch.equal(start, torch.tensor([3, 10, 10, 17, 24]))
    assert torch.equal(end, off[1:])
    assert torch.equal(sp[0], start) and torch.equal(sp[1], end) and len(sp) == 2
    assert sp.start is sp.start  # computed once


def _varlen_batch(n, seed=0x5EED0006):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 2945, n)
    pay = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq, ack, flags, _ = synth.synth(seed, 0, n, 0)
    bounds = np.concatenate([[0], np.cumsum(lens)])
    pays = [pay[bounds[i]:bounds[i + 1]].tobytes() for i in range(n)]
    return seq, ack, flags, pays


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_varlen_virtual_shards_rebase_to_unsharded(world):
    """Each shard scans its own lengths (offsets from 0); frame_base rebases
    them, and the concatenation is the unsharded batch."""
    n = 1024
    seq, ack, flags, pays = _varlen_batch(n)
    full, full_off, full_cs = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    frames, offs, totals = [], [], []
    for r in range(world):
        first, m = shard.rank_slice(r, world, n)
        fr, off, _ = codec_np.encode_varlen(seq[first:first + m], ack[first:first + m],
                                            flags[first:first + m], pays[first:first + m], 7)
        frames.append(fr)
        offs.append(np.asarray(off, dtype=np.int64))
        totals.append(int(off[-1]))
    assert np.array_equal(np.concatenate(frames), full)
    glob = [o + shard.frame_base(totals, r) for r, o in enumerate(offs)]
    assert np.array_equal(np.concatenate([g[:-1] for g in glob] + [glob[-1][-1:]]), np.asarray(full_off))


def test_rank_slice_rejects_bad_ranks():
    with pytest.raises(ValueError):
        shard.rank_slice(2, 2, 8)
    with pytest.raises(ValueError):
        shard.rank_slice(0, 0, 8)


def _varlen_worker(rank, world, port, out):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 512
    seq, ack, flags, pays = _varlen_batch(n)
    first, m = shard.rank_slice(rank, world, n)
    fr, off, _ = codec_np.encode_varlen(seq[first:first + m], ack[first:first + m], flags[first:first + m],
                                        pays[first:first + m], 7)
    glob = shard.global_frame_offsets(torch.as_tensor(np.asarray(off, dtype=np.int64)))
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, bytes(fr), glob.tolist()))
    if rank == 0:
        out.put(gathered)
    dist.destroy_process_group()


def test_gloo_world2_varlen_global_offsets():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_varlen_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = sorted(q.get(timeout=120))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seq, ack, flags, pays = _varlen_batch(512)
    full, full_off, _ = codec_np.encode_varlen(seq, ack, flags, pays, 7)
    assert b"".join(g[1] for g in gathered) == bytes(full)
    offs = gathered[0][2][:-1] + gathered[1][2]
    assert offs == [int(x) for x in full_off]
