"""Loopback UDP costs behind the relay leg (no GPU): sendmmsg of one-character
datagrams to a drained sink, per datagram, in the shapes the relay and the
socket leg use.

  fixed      one destination (the socket leg's sender)
  per_dgram  a destination per datagram (the relay's forwarder)
  shared     per_dgram from a socket another thread is receiving on at the same
             time (the relay's one socket for both directions)

usage: python tools/udp_probe.py [--n 262144] [--batch 1024]
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

from rudp import _native, netio  # noqa: E402


def sink_socket():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 26)
    s.bind(("127.0.0.1", 0))
    return s


def drain(s, got, stop):
    buf, off = np.empty((1 << 16) * 64, np.uint8), np.empty((1 << 16) + 1, np.int64)
    while not stop.is_set():
        k = netio.recv_batch(s, buf, off, slot_bytes=64, timeout_ms=50)
        got[0] += k


def run(shape, n, batch):
    sink = sink_socket()
    got, stop = [0], threading.Event()
    t = threading.Thread(target=drain, args=(sink, got, stop))
    t.start()
    tx = sink_socket()  # a bound socket, like the relay's
    other_stop = threading.Event()
    feeder = None
    if shape == "shared":  # another thread receives on the sending socket meanwhile
        src = sink_socket()
        rgot = [0]
        feeder = threading.Thread(target=drain, args=(tx, rgot, other_stop))
        feeder.start()

        def feed():
            fr = np.full(batch, 0x41, np.uint8)
            of = np.arange(batch + 1, dtype=np.int64)
            while not other_stop.is_set():
                netio.send_batch(src, fr, of, "127.0.0.1", tx.getsockname()[1])
                time.sleep(0.001)
        feed_t = threading.Thread(target=feed)
        feed_t.start()
    frames = np.full(n, 0x41, np.uint8)
    off = np.arange(n + 1, dtype=np.int64)
    key = netio.addr_key("127.0.0.1", sink.getsockname()[1])
    dst = np.full(batch, key, np.uint64)
    t0 = time.perf_counter()
    for a in range(0, n, batch):
        b = min(n, a + batch)
        while a - got[0] > 32768:
            time.sleep(20e-6)
        if shape == "fixed":
            netio.send_batch(tx, frames, off[a:b + 1], "127.0.0.1", sink.getsockname()[1])
        else:
            netio.send_batch_to(tx, frames, off[a:b + 1], dst[:b - a])
    t_send = time.perf_counter() - t0
    while got[0] < n and time.perf_counter() - t0 < 10:
        time.sleep(1e-4)
    dt = time.perf_counter() - t0
    stop.set()
    other_stop.set()
    t.join()
    if feeder is not None:
        feeder.join()
        feed_t.join()
    return {"sent": n, "got": got[0], "send_s": t_send, "wall_s": dt, "Mpkt_s": got[0] / dt / 1e6,
            "us_per_dgram_send": t_send / n * 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    _native.lib()
    print(json.dumps({s: run(s, args.n, args.batch) for s in ("fixed", "per_dgram", "shared")}))


if __name__ == "__main__":
    main()
