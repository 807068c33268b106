"""bench.py's command line without a GPU: the self-launch of N > 1 ranks and the
compact baseline summary at the end of the JSON line."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def test_gpus_n_without_launcher_starts_torch_distributed_run():
    """--gpus 4 with no WORLD_SIZE: bench.py's own launcher command (a child
    torch.distributed.run over 127.0.0.1, the same arguments)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "4", "--steps", "7", "--print-launch"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(str(REPO / "bench.py"))
    assert cmd[i + 1:i + 5] == ["--gpus", "4", "--steps", "7"]


def test_baseline_summary_is_compact_and_last():
    sys.path.insert(0, str(REPO))
    import bench
    line = {"roofline": {"kernel_ms_per_launch": 0.5166, "frac": 0.75}, "config": {"matches_reference": True},
            "legs": {"encode_1Mx1024": {"ms": 0.35, "roofline_frac": 0.77, "chunks_matching_reference_digests": "1/1"},
                     "roundtrip_1Mx1472": {"ms": 0.73, "roofline_frac": 0.8,
                                           "chunks_matching_reference_digests": "2/2",
                                           "decode_fields_equal_inputs": True},
                     "encode_1Mx1_fixed": {"ms": 0.011, "roofline_frac": 0.17, "vs_varlen_same_bytes": 0.8,
                                           "frames_equal_varlen_path": True}}}
    s = bench.baseline_summary(line)
    assert s["C2_encode_1Mx1024"] == {"ms": 0.35, "frac": 0.77, "digests": "1/1"}
    assert s["C4_roundtrip_1Mx1472"]["decode_fields_equal_inputs"] is True
    assert s["encode_1Mx1_fixed"]["vs_varlen_same_bytes"] == 0.8
    assert "C3_encode_1Mx64" not in s
    assert len(json.dumps(s)) < 2500
