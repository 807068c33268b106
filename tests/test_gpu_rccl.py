"""The RCCL branch of the multi-GPU path, run at world 1 on the one GPU a box has.

Packets shard by slicing: no collective touches the frames.
The only collectives are the benchmark's clock (barrier, MAX of the wall time
over ranks, every rank's kernel time gathered), the device records, the C5
chunk-digest count and shard.global_frame_offsets' one-integer all_gather.
On the driver's 8-GPU node they run over RCCL ("nccl" backend, device
tensors); the CPU suite covers them with gloo (tests/test_sharding.py).  Here
each runs over RCCL with init_process_group("nccl", device_id=cuda:0) at
world 1, in a fresh process launched as torch.distributed.run would.  The
reference has no multi-device counterpart (every Packet is independent,
utils/packet.py:13-16).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent


def _env():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env["PYTHONPATH"] = os.pathsep.join([str(REPO), str(REPO / "reliable-udp_amd"), env.get("PYTHONPATH", "")])
    return env


def test_bench_distributed_path_over_rccl_at_world_1(cuda):
    """bench.py's N > 1 code (process group over RCCL, device records gathered,
    barrier + MAX clock, kernel times gathered, the C5 strong leg with its
    device all_reduce of digest counts) at N = 1."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--dist", "--steps", "5", "--warmup", "2",
                        "--no-cpu-baseline", "--packets", "262144", "--c5-packets", "1048576"],
                       cwd=REPO, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    roof = line["roofline"]
    assert len(roof["kernel_ms_per_launch_by_rank"]) == 1
    assert abs(roof["kernel_ms_per_launch"] - roof["kernel_ms_per_launch_by_rank"][0]) < 1e-9
    c5 = line["legs"]["c5_16Mx1472_strong"]
    assert c5["packets_total"] == 1 << 20 and c5["n_gpus"] == 1
    assert c5["chunks_matching_reference_digests"] == 1 and c5["ranks_bit_exact_vs_reference"] == 1
    assert line["config"]["devices"][0]["device_index"] == 0


_SHARD_SCRIPT = r"""
import torch, torch.distributed as dist
from rudp import batch, shard
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl"
n = 5000
tab, pay = batch.synth_batch(n, 0, 7, device=dev)
g = torch.Generator(device=dev).manual_seed(7)
lens = torch.randint(0, 300, (n,), dtype=torch.int32, device=dev, generator=g)
flat = torch.randint(0, 256, (int(lens.sum().item()),), dtype=torch.uint8, device=dev, generator=g)
res = batch.pack_batch_varlen(tab, flat, lens, "rudp7")
glob = shard.global_frame_offsets(res.frame_off)          # device all_gather of one int64
assert glob.device == dev and torch.equal(glob, res.frame_off)
t = torch.tensor([1.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 1.5
objs = [None]
dist.all_gather_object(objs, {"rank": 0, "frames": int(res.frame_off[-1].item())})
assert objs[0]["frames"] == int(res.frame_off[-1].item())
dist.barrier()
dist.destroy_process_group()
print("rccl-ok")
"""


def test_shard_offsets_and_collectives_over_rccl_at_world_1(cuda):
    r = subprocess.run([sys.executable, "-c", _SHARD_SCRIPT], cwd=REPO, env=_env(), capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0 and "rccl-ok" in r.stdout, r.stderr[-3000:]
