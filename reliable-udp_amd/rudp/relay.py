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

``Relay(..., batched=True)`` is the batched form:
every recvmmsg takes up to ``max_msgs`` datagrams with their source addresses
(rudp_udp_recv_batch_from); the retransmission flags of the whole batch come
from one GPU launch of rudp_dedup_window over the last MAX_MEMORY datagrams
of the earlier batches followed by this batch (the history carried across
batches), and the datagrams that are not dropped leave in one sendmmsg with
per-datagram destinations (rudp_udp_send_batch_to).  Same forwarding, log and
counters as the per-datagram loop.
"""
from __future__ import annotations

import socket
import threading
from collections import Counter, deque
from typing import Callable, Dict, List, Optional

import numpy as np

MAX_MEMORY = 500  # proxy.py:17
SLOT_BYTES = 1024  # recvfrom(1024), proxy.py:129


class Relay(threading.Thread):
    """Forward between one client and the server at ``server_port``.

    ``drop(direction, index) -> bool`` decides per datagram ("c2s" / "s2c",
    the datagram's index in that direction; None: nothing is dropped).
    ``log`` keeps every datagram seen per direction (``keep_log=False``: only
    the per-direction counts, for throughput runs); ``stats`` mirrors
    proxy.py's live_stats counters.
    """

    def __init__(self, server_port: int, drop: Optional[Callable[[str, int], bool]] = None,
                 host: str = "127.0.0.1", batched: bool = False, device=None, max_msgs: int = 1024,
                 keep_log: bool = True):
        super().__init__(daemon=True)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((host, 0))
        self.sock.settimeout(0.05)
        self.port = self.sock.getsockname()[1]
        self.server = (host, server_port)
        self.client = None
        self.drop = drop
        self.keep_log = keep_log
        self.log: Dict[str, List[bytes]] = {"c2s": [], "s2c": []}
        self.seen = {"c2s": 0, "s2c": 0}  # datagrams per direction (the drop rule's index)
        self.stats = {f"{side}_{k}": 0 for side in ("client", "server")
                      for k in ("sent", "received", "dropped", "retransmitted")}
        self._history: deque = deque()
        self._seen: Counter = Counter()
        self.stop_event = threading.Event()
        self.batched = batched
        self.batches = 0
        if batched:
            import torch
            self._device = torch.device(device) if device is not None else torch.device("cuda", 0)
            self._max_msgs = max_msgs
            from .netio import addr_key
            self._server_key = addr_key(host, server_port)
            self._client_key = None
            # the last MAX_MEMORY datagrams (both directions), packed, for the next batch's check
            self._hist_frames = np.zeros(0, np.uint8)
            self._hist_off = np.zeros(1, np.int64)

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

    def _dup_flags(self, frames: np.ndarray, off: np.ndarray) -> np.ndarray:
        """Retransmission flags of a batch (frames[off[i]:off[i+1]], i < k) against the
        carried history and the batch's own earlier datagrams: one GPU launch of the
        proxy's `Packet(data) in self.packets` (proxy.py:90), window MAX_MEMORY."""
        import torch
        from . import batch
        k = off.shape[0] - 1
        h = self._hist_off.shape[0] - 1
        body = frames[off[0]:off[k]]
        # one spare byte keeps the buffer non-empty when every datagram is empty
        allf = np.concatenate([self._hist_frames, body, np.zeros(1, np.uint8)])
        allo = np.concatenate([self._hist_off, self._hist_off[-1] + (off[1:] - off[0])])
        d_frames = torch.from_numpy(allf).to(self._device)
        d_off = torch.from_numpy(allo).to(self._device)
        dup = batch.detect_retransmissions(d_frames, frame_off=d_off, window=MAX_MEMORY).cpu().numpy()[h:]
        # carry the last MAX_MEMORY datagrams into the next batch
        keep = min(MAX_MEMORY, h + k)
        first = h + k - keep
        self._hist_frames = allf[allo[first]:allo[-1]].copy()
        self._hist_off = allo[first:] - allo[first]
        return dup.astype(bool)

    def _relay_batch(self, frames: np.ndarray, off: np.ndarray, src: np.ndarray) -> None:
        """Record and forward one received batch (the per-datagram loop's work, batched)."""
        from . import netio
        k = off.shape[0] - 1
        from_server = src == self._server_key
        n_s = int(from_server.sum())
        first = {"s2c": self.seen["s2c"], "c2s": self.seen["c2s"]}
        self.seen["s2c"] += n_s
        self.seen["c2s"] += k - n_s
        dropped = np.zeros(k, bool)
        if self.keep_log or self.drop is not None:
            idx = {"s2c": first["s2c"], "c2s": first["c2s"]}
            for i in range(k):
                direction = "s2c" if from_server[i] else "c2s"
                if self.keep_log:
                    self.log[direction].append(frames[off[i]:off[i + 1]].tobytes())
                if self.drop is not None:
                    dropped[i] = bool(self.drop(direction, idx[direction]))
                idx[direction] += 1
        # the client is the source of the latest client datagram (proxy.py:133-135):
        # a server datagram goes to the client known when it arrived
        pos = np.where(~from_server, np.arange(k), -1)
        last = np.maximum.accumulate(pos)
        prev = np.uint64(self._client_key or 0)
        to_client = np.where(last >= 0, src[np.maximum(last, 0)], prev)
        dst = np.where(from_server, to_client, np.uint64(self._server_key)).astype(np.uint64)
        if n_s < k:
            self._client_key = int(src[pos.max()])
            self.client = netio.key_addr(self._client_key)
        dup = self._dup_flags(frames, off)
        # proxy.py:79-94, summed over the batch
        for side, m in (("server", from_server), ("client", ~from_server)):
            other = "client" if side == "server" else "server"
            self.stats[f"{side}_sent"] += int(m.sum())
            self.stats[f"{side}_dropped"] += int((m & dropped).sum())
            self.stats[f"{other}_received"] += int((m & ~dropped).sum())
            self.stats[f"{side}_retransmitted"] += int((m & dup).sum())
        # a server datagram before any client one has nowhere to go (dst 0: not sent)
        send = ~dropped & (dst != 0)
        if send.any():
            lens = np.diff(off)
            body = frames[off[0]:off[k]]
            out = body[np.repeat(send, lens)] if body.size else body
            out_off = np.concatenate([[0], np.cumsum(lens[send])]).astype(np.int64)
            netio.send_batch_to(self.sock, out, out_off, dst[send])
        self.batches += 1

    def _run_batched(self) -> None:
        from . import netio
        frames = np.empty(self._max_msgs * SLOT_BYTES, np.uint8)
        off = np.empty(self._max_msgs + 1, np.int64)
        src = np.empty(self._max_msgs, np.uint64)
        while not self.stop_event.is_set():
            k = netio.recv_batch(self.sock, frames, off, slot_bytes=SLOT_BYTES, max_msgs=self._max_msgs,
                                 timeout_ms=50, sources=src)
            if k:
                self._relay_batch(frames, off[:k + 1], src[:k])

    def run(self) -> None:
        if self.batched:
            self._run_batched()
            return
        while not self.stop_event.is_set():
            try:
                data, addr = self.sock.recvfrom(1024)  # proxy.py:129
            except socket.timeout:
                continue
            from_server = addr == self.server
            if not from_server:
                self.client = addr
            direction = "s2c" if from_server else "c2s"
            index = self.seen[direction]
            self.seen[direction] += 1
            if self.keep_log:
                self.log[direction].append(data)
            dropped = bool(self.drop(direction, index)) if self.drop is not None else False
            self._record("server" if from_server else "client", data, dropped)
            if not dropped:
                self.sock.sendto(data, self.client if from_server else self.server)

    def stop(self) -> None:
        self.stop_event.set()
        self.join(timeout=2)
        self.sock.close()
