"""Batched UDP socket I/O (recvmmsg / sendmmsg) at the host boundary, over loopback."""
import socket
import threading

import numpy as np
import pytest

from oracle import codec_np, synth
from rudp import netio
from rudp.packet import Packet


def udp_pair(rcvbuf=1 << 25):
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, rcvbuf)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    return rx, tx, rx.getsockname()[1]


def frames_for(n, L_max, seed=5):
    rng = np.random.default_rng(seed)
    seq, ack, flags, _ = synth.synth(seed, 0, n, 0)
    pays = [bytes(rng.integers(0, 128, rng.integers(0, L_max), dtype=np.uint8)) for _ in range(n)]
    return codec_np.encode_varlen(seq, ack, flags, pays, 5)


def receive_all(rx, n, slot=1024, timeout_ms=2000):
    frames = np.empty(n * slot, np.uint8)
    off = np.empty(n + 1, np.int64)
    out, got = [], 0
    while got < n:
        k = netio.recv_batch(rx, frames, off, slot_bytes=slot, max_msgs=n - got, timeout_ms=timeout_ms)
        if k == 0:
            break
        out += [bytes(frames[off[i]:off[i + 1]]) for i in range(k)]
        got += k
    return out


def test_send_recv_roundtrip_in_order():
    n = 20000
    fr, off, _ = frames_for(n, 60)
    rx, tx, port = udp_pair()
    t = threading.Thread(target=lambda: netio.send_batch(tx, fr, off, "127.0.0.1", port))
    t.start()
    got = receive_all(rx, n)
    t.join()
    want = [bytes(fr[off[i]:off[i + 1]]) for i in range(n)]
    assert got == want
    # each frame still parses with the drop-in, like utils/reliableUDP.py:119 would
    assert int(Packet(got[123]).get_header_field("seq_num", 10)) == int.from_bytes(want[123][:2], "big")
    rx.close()
    tx.close()


def test_truncation_like_recvfrom_1024():
    rx, tx, port = udp_pair()
    big = bytes(range(256)) * 8  # 2048 B
    tx.sendto(big, ("127.0.0.1", port))
    tx.sendto(b"", ("127.0.0.1", port))
    tx.sendto(b"abc", ("127.0.0.1", port))
    got = receive_all(rx, 3)
    assert got == [big[:1024], b"", b"abc"]
    rx.close()
    tx.close()


def test_timeout_and_nonblocking():
    rx, tx, port = udp_pair()
    frames = np.empty(4096, np.uint8)
    off = np.empty(5, np.int64)
    assert netio.recv_batch(rx, frames, off, timeout_ms=50) == 0
    assert netio.recv_batch(rx, frames, off, timeout_ms=0) == 0
    with pytest.raises(TypeError):
        netio.recv_batch(rx, frames.astype(np.int8), off)
    with pytest.raises(ValueError):
        netio.send_batch(tx, frames[:10], np.array([0, 20], np.int64), "127.0.0.1", port)
    rx.close()
    tx.close()
