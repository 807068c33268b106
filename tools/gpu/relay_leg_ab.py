"""bench.py's relay leg (client + sink in a child process) at 1, 2 and 3
forwarding threads, interleaved twice.  Prints one JSON line."""
import functools
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rudp import batch, relay  # noqa: E402

orig = relay.Relay.__init__
res = {}
for rep in range(2):
    for f in (1, 2, 3):
        relay.Relay.__init__ = functools.partialmethod(orig, forwarders=f)
        out = bench.relay_leg(torch, batch, torch.device("cuda", 0))
        res.setdefault(f, []).append(round(out["batched"]["Mpkt_s"], 4))
        print(f, out["batched"]["Mpkt_s"], out["per_datagram"]["Mpkt_s"], file=sys.stderr, flush=True)
print(json.dumps({"batched_Mpkt_s_by_forwarders": res}))
