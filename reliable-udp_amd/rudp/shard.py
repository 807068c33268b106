"""Packet-range sharding over ranks: no data-path exchange.

Rank r of `world` frames packets [r*N/world, (r+1)*N/world) of an N-packet
batch.  With fixed-length payloads frame i sits at i*(L+H), so every shard is
independent.  With variable lengths each rank's encode scans its own lengths
(``pack_batch_varlen``), so its frame offsets start at 0; the global offset of
its first frame is the sum of the frame bytes of the ranks before it.  That is
one integer per rank: ``frame_base`` adds them up on the host, and
``global_frame_offsets`` gathers them with one all_gather of a 1-element
tensor (torch.distributed, gloo or RCCL) -- the only communication, and none
of it touches the frames.  Concatenating the shards' frames in rank order
gives the unsharded batch's frames byte for byte, and their global offsets its
offsets (tests/test_sharding.py, tests/test_gpu_varlen.py).
"""
from __future__ import annotations

from typing import Sequence, Tuple


def rank_slice(rank: int, world: int, total: int) -> Tuple[int, int]:
    """(first, count): the packets rank r frames when `total` packets are split
    over `world` ranks, [r*total//world, (r+1)*total//world): any world size,
    shard sizes differing by at most one packet when world does not divide total."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside a world of {world}")
    if total < 0:
        raise ValueError(f"negative packet count {total}")
    first = rank * total // world
    return first, (rank + 1) * total // world - first


def frame_base(shard_frame_bytes: Sequence[int], rank: int) -> int:
    """Global byte offset of rank r's first frame: the frame bytes of ranks < r."""
    return int(sum(int(b) for b in shard_frame_bytes[:rank]))


def global_frame_offsets(frame_off, group=None):
    """This rank's frame offsets (int64 [n + 1], starting at 0, as its encode
    returned them) moved to the unsharded batch's numbering.  Collective: every
    rank of `group` calls it.  The gathered totals travel as CPU tensors on a
    gloo group, as device tensors otherwise."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    on_cpu = dist.get_backend(group) == "gloo"
    total = frame_off[-1:].to(torch.int64)
    if on_cpu:
        total = total.cpu()
    gathered = [torch.empty_like(total) for _ in range(world)]
    dist.all_gather(gathered, total, group=group)
    base = frame_base([int(t.item()) for t in gathered], rank)
    return frame_off + base
