"""A UDP relay in the reference proxy's role, for BASELINE config 1.

Config 1 is client -> proxy.py -> server over 127.0.0.1.  The reference
proxy (proxy.py:126-154) forwards each datagram by its source address,
optionally drops or delays it, and records it (proxy.py:79-94): per-side
sent / received / dropped counters and a retransmission count from
``Packet(data) in self.packets`` over the last MAX_MEMORY = 500 datagrams of
both directions (proxy.py:17, :90-94; Packet.__eq__, utils/packet.py:83-86).
Its curses knobs and matplotlib plot are out of scope; drops here come from a
caller-supplied rule so tests and the bench are deterministic.

The history check is the same relation as the proxy's list scan, kept as a
multiset of keys: two datagrams are Packet-equal (same get_hex(), i.e. same
bit string) exactly when their bytes are equal, except that an empty datagram
parses as the 40-bit zero header (utils/packet.py:16) and so equals five zero
bytes.  O(1) per datagram instead of up to 500 __eq__ calls.
"""
from __future__ import annotations

import socket
import threading
from collections import Counter, deque
from typing import Callable, Dict, List

MAX_MEMORY = 500  # proxy.py:17


class Relay(threading.Thread):
    """Forward between one client and the server at ``server_port``.

    ``drop(direction, index) -> bool`` decides per datagram ("c2s" / "s2c",
    the datagram's index in that direction).  ``log`` keeps every datagram
    seen per direction; ``stats`` mirrors proxy.py's live_stats counters.
    """

    def __init__(self, server_port: int, drop: Callable[[str, int], bool] = lambda d, i: False,
                 host: str = "127.0.0.1"):
        super().__init__(daemon=True)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((host, 0))
        self.sock.settimeout(0.05)
        self.port = self.sock.getsockname()[1]
        self.server = (host, server_port)
        self.client = None
        self.drop = drop
        self.log: Dict[str, List[bytes]] = {"c2s": [], "s2c": []}
        self.stats = {f"{side}_{k}": 0 for side in ("client", "server")
                      for k in ("sent", "received", "dropped", "retransmitted")}
        self._history: deque = deque()
        self._seen: Counter = Counter()
        self.stop_event = threading.Event()

    @property
    def retransmitted(self) -> int:
        return self.stats["client_retransmitted"] + self.stats["server_retransmitted"]

    def _record(self, source: str, data: bytes, dropped: bool) -> None:
        # proxy.py:79-94
        other = "client" if source == "server" else "server"
        key = data if data else bytes(5)  # Packet(b"") is the 40-bit zero header
        self.stats[f"{source}_sent"] += 1
        self.stats[f"{source}_dropped" if dropped else f"{other}_received"] += 1
        if self._seen[key]:
            self.stats[f"{source}_retransmitted"] += 1
        self._history.append(key)
        self._seen[key] += 1
        if len(self._history) > MAX_MEMORY:
            old = self._history.popleft()
            self._seen[old] -= 1

    def run(self) -> None:
        while not self.stop_event.is_set():
            try:
                data, addr = self.sock.recvfrom(1024)  # proxy.py:129
            except socket.timeout:
                continue
            from_server = addr == self.server
            if not from_server:
                self.client = addr
            direction = "s2c" if from_server else "c2s"
            index = len(self.log[direction])
            self.log[direction].append(data)
            dropped = bool(self.drop(direction, index))
            self._record("server" if from_server else "client", data, dropped)
            if not dropped:
                self.sock.sendto(data, self.client if from_server else self.server)

    def stop(self) -> None:
        self.stop_event.set()
        self.join(timeout=2)
        self.sock.close()
