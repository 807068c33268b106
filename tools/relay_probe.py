"""Where the batched relay's time goes (bench leg relay_1char, proxy.py's role).

Runs the bench's relay leg shape (one-character datagrams blasted at a batched
rudp.relay.Relay, forwarded to a sink) with timers around the relay thread's
recvmmsg (BatchReceiver.recv), its batch work (Relay._relay_batch: numpy
bookkeeping and the GPU enqueue), the forwarding thread's sendmmsg, and the
sink's recvmmsg.  Prints one JSON line: seconds and calls per phase, and the
datagrams/s.

usage: python tools/relay_probe.py [--n 262144] [--max-msgs 1024] [--switch 0.0002]
"""
from __future__ import annotations

import argparse
import json
import socket
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "reliable-udp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rudp import batch, netio, relay  # noqa: E402

T = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            d = T.setdefault(name, [0.0, 0])
            d[0] += time.perf_counter() - t0
            d[1] += 1
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--max-msgs", type=int, default=1024)
    ap.add_argument("--forwarders", type=int, default=2)
    ap.add_argument("--switch", type=float, default=0.0, help="sys.setswitchinterval (s); 0 keeps the default")
    args = ap.parse_args()
    if args.switch > 0:
        sys.setswitchinterval(args.switch)
    dev = torch.device("cuda", 0)
    n = args.n
    tab, pay = batch.synth_batch(n, 1, 0x5EED0004, device=dev)
    tab.seq.copy_(torch.arange(n, device=dev).to(torch.int32).to(torch.uint16))
    enc = batch.pack_batch_varlen(tab, pay.view(-1), torch.ones(n, dtype=torch.int32, device=dev), "rudp5")
    frames, off = enc.frames.cpu().numpy(), enc.frame_off.cpu().numpy()
    netio.BatchReceiver.recv = timed("relay_recv", netio.BatchReceiver.recv)
    relay.Relay._relay_batch = timed("relay_batch_work", relay.Relay._relay_batch)
    relay.Relay._count_retransmissions = timed("relay_gpu_enqueue", relay.Relay._count_retransmissions)
    send_to = netio.send_batch_to
    netio.send_batch_to = timed("forward_sendmmsg", send_to)
    sink = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sink.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
    sink.bind(("127.0.0.1", 0))
    r = relay.Relay(sink.getsockname()[1], batched=True, device=dev, keep_log=False, max_msgs=args.max_msgs,
                    forwarders=args.forwarders)
    r.sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
    r.start()
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    got = [0]
    rbuf, roff = np.empty((1 << 16) * 64, np.uint8), np.empty((1 << 16) + 1, np.int64)
    sink_recv = timed("sink_recv", netio.recv_batch)

    def drain():
        while True:
            k = sink_recv(sink, rbuf, roff, slot_bytes=64, timeout_ms=500)
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
        netio.send_batch(tx, frames, off[a:b + 1], "127.0.0.1", r.port)
    t.join()
    dt = time.perf_counter() - t0 - 0.5
    r.stop()
    print(json.dumps({"n": n, "switch_s": sys.getswitchinterval(), "forwarders": args.forwarders, "relayed": got[0], "wall_s": dt, "Mpkt_s": got[0] / dt / 1e6,
                      "batches": r.batches, "phases_s_calls": {k: [round(v[0], 4), v[1]] for k, v in T.items()}}))


if __name__ == "__main__":
    main()
