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
into a pinned receive ring (rudp.netio.BatchReceiver, rudp_udp_recv_batch_from),
and the datagrams that are not dropped leave in one sendmmsg with
per-datagram destinations (rudp_udp_send_batch_to), on a forwarding thread
of their own so the kernel's per-datagram send cost overlaps the next
recvmmsg (the receive slot stays held until its datagrams are sent; one
thread, so each direction keeps its order).  The retransmission flags of a
batch come from librudp's dedup stream (rudp_dedup_stream_push): one GPU
launch of rudp_dedup_window's rule over the last MAX_MEMORY datagrams of the
earlier batches followed by this batch, the history kept on the device, the
flags summed into per-side device counters, all enqueued from C with no wait
for the GPU; the counters are read when ``stats`` is.  Forwarding does not
depend on the flags (the proxy only counts retransmissions, proxy.py:90-91).
Same forwarding, log and counters as the per-datagram loop.
"""
from __future__ import annotations

import ctypes
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
                 keep_log: bool = True, forwarders: int = 1):
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
        self._stats = {f"{side}_{k}": 0 for side in ("client", "server")
                       for k in ("sent", "received", "dropped", "retransmitted")}
        self._history: deque = deque()
        self._seen: Counter = Counter()
        self.stop_event = threading.Event()
        self.errors: List[BaseException] = []  # forwarding-thread failures (the relay keeps going)
        self.batched = batched
        self.batches = 0
        # Batched: sendmmsg threads (batches leave in the order the threads
        # reach the kernel, as the reference's executor workers send them,
        # proxy.py:127, :154).  One is the default: the hop costs ~1.2 us per
        # datagram in the kernel's send path of the one socket, and 2 or 3
        # threads on it measured no faster (0.64-0.79 vs 0.78 M/s,
        # profiles/r04/sweeps/relay_forwarders.json).
        self.forwarders = max(1, int(forwarders))
        if batched:
            import torch
            self._device = torch.device(device) if device is not None else torch.device("cuda", 0)
            self._max_msgs = max_msgs
            from .netio import addr_key
            self._server_key = addr_key(host, server_port)
            self._client_key = None
            self._stream = torch.cuda.Stream(self._device)
            from . import _native
            h = ctypes.c_void_p()
            _native.check(_native.lib().rudp_dedup_stream_create(
                MAX_MEMORY, max_msgs, SLOT_BYTES, self._device.index or 0, self._stream.cuda_stream, ctypes.byref(h)))
            self._dstream = h

    def __del__(self):
        h = getattr(self, "_dstream", None)
        if h is not None and h.value:
            from . import _native
            _native.lib().rudp_dedup_stream_destroy(h)
            self._dstream = None

    @property
    def stats(self) -> Dict[str, int]:
        """proxy.py's live_stats counters.  Batched: the GPU's retransmission counts
        are folded in here (one synchronization with the relay's stream)."""
        if self.batched:
            from . import _native
            acc = (ctypes.c_uint64 * 2)()
            _native.check(_native.lib().rudp_dedup_stream_counts(self._dstream, acc))
            return {**self._stats, "client_retransmitted": int(acc[0]), "server_retransmitted": int(acc[1])}
        return dict(self._stats)

    @property
    def retransmitted(self) -> int:
        st = self.stats
        return st["client_retransmitted"] + st["server_retransmitted"]

    def _record(self, source: str, data: bytes, dropped: bool) -> None:
        # proxy.py:79-94
        other = "client" if source == "server" else "server"
        key = data if data else bytes(5)  # Packet(b"") is the 40-bit zero header
        self._stats[f"{source}_sent"] += 1
        self._stats[f"{source}_dropped" if dropped else f"{other}_received"] += 1
        if self._seen[key]:
            self._stats[f"{source}_retransmitted"] += 1
        self._history.append(key)
        self._seen[key] += 1
        if len(self._history) > MAX_MEMORY:
            old = self._history.popleft()
            self._seen[old] -= 1

    def _count_retransmissions(self, frames: np.ndarray, off: np.ndarray, side: np.ndarray) -> None:
        """Enqueue the batch's retransmission check (the proxy's `Packet(data) in
        self.packets`, proxy.py:90, window MAX_MEMORY) and its per-side count
        (side 1: from the server) through librudp's dedup stream; frames are
        copied out of ``frames`` before the call returns, nothing waits for the GPU."""
        from . import _native
        k = off.shape[0] - 1
        off = np.ascontiguousarray(off, dtype=np.uint64)
        side = np.ascontiguousarray(side, dtype=np.uint8)
        _native.check(_native.lib().rudp_dedup_stream_push(
            self._dstream, frames.ctypes.data if frames.size else None, off.ctypes.data, k, side.ctypes.data, None))

    def _relay_batch(self, frames: np.ndarray, off: np.ndarray, src: np.ndarray, rx=None, send_q=None) -> None:
        """Record and forward one received batch (the per-datagram loop's work,
        batched).  ``rx``: the BatchReceiver whose last batch this is (its pinned
        slot is copied to the device asynchronously); else ``frames`` is copied
        from wherever it lives.  ``send_q``: hand the sendmmsg to the forwarding
        thread (holding rx's slot until it has run); else send here."""
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
        self._count_retransmissions(frames, off, from_server)
        # proxy.py:79-94 (retransmissions: on the device, _count_retransmissions)
        for side, m in (("server", from_server), ("client", ~from_server)):
            other = "client" if side == "server" else "server"
            self._stats[f"{side}_sent"] += int(m.sum())
            self._stats[f"{side}_dropped"] += int((m & dropped).sum())
            self._stats[f"{other}_received"] += int((m & ~dropped).sum())
        # a server datagram before any client one has nowhere to go (dst 0: not sent)
        send = ~dropped & (dst != 0)
        if send.all():
            out, out_off, out_dst = frames, off, dst  # (offsets into frames, as sendmmsg reads them)
        elif send.any():
            lens = np.diff(off)
            body = frames[off[0]:off[k]]
            out = body[np.repeat(send, lens)] if body.size else body
            out_off = np.concatenate([[0], np.cumsum(lens[send])]).astype(np.int64)
            out_dst = dst[send]
        else:
            out = None
        if out is not None:
            if send_q is not None:
                send_q.put((out, out_off, out_dst, rx.hold() if rx is not None else None))
            else:
                netio.send_batch_to(self.sock, out, out_off, out_dst)
        self.batches += 1

    def _forward(self, q, rx) -> None:
        """The forwarding thread: sendmmsg each batch handed over, in order, then
        give its receive slot back."""
        from . import netio
        while True:
            item = q.get()
            if item is None:
                return
            out, out_off, out_dst, slot = item
            try:
                netio.send_batch_to(self.sock, out, out_off, out_dst)
            except OSError as e:
                if not self.stop_event.is_set():  # (a socket closed under a stopping relay is expected)
                    self.errors.append(e)         # anything else: kept for the caller, the relay goes on
            except Exception as e:  # noqa: BLE001 -- recorded; the slot is still given back
                self.errors.append(e)   # (KeyboardInterrupt / SystemExit propagate after the finally)
            finally:
                if slot is not None:
                    rx.release(slot)

    def _run_batched(self) -> None:
        import queue
        from . import netio
        rx = netio.BatchReceiver(self.sock, max_msgs=self._max_msgs, slot_bytes=SLOT_BYTES, slots=2 + 2 * self.forwarders,
                                 device=self._device, stream=self._stream, with_sources=True)
        q: "queue.Queue" = queue.Queue()
        fwd = [threading.Thread(target=self._forward, args=(q, rx), daemon=True) for _ in range(self.forwarders)]
        for t in fwd:
            t.start()
        try:
            while not self.stop_event.is_set():
                k = rx.recv(timeout_ms=50)
                if k:
                    self._relay_batch(rx.frames, rx.frame_off[:k + 1], rx.sources, rx=rx, send_q=q)
        finally:
            for _ in fwd:
                q.put(None)
            for t in fwd:
                t.join()

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
