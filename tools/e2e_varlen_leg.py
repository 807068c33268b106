"""The bench's e2e_host_varlen_1M_x_1char leg alone (bench.e2e_host_varlen_leg),
with more calls: python tools/e2e_varlen_leg.py [--reps 7]"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from rudp import batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
print(json.dumps(bench.e2e_host_varlen_leg(torch, batch, args.reps), indent=1))
