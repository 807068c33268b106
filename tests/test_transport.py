"""Config 1: client -> relay -> server over 127.0.0.1 with the drop-in codec.

rudp.transport.ReliableUDP (the caller, counterpart of utils/reliableUDP.py)
moves bin/input.txt's message through rudp.relay.Relay, which plays proxy.py's
role (forward both ways, record, optionally drop).  Every datagram on the wire is
compared with the trace captured from the reference (tests/golden/
wire_trace.json, ISN 0x0e1b), and the relay checks each one with the drop-in
Packet the way proxy.py:81,90 does.
"""
import socket
import threading
import time

import pytest

from rudp.packet import Packet
from rudp.relay import Relay
from rudp.transport import ReliableUDP


def run_transfer(message, isn, drop=None, client_timeout=1, codec_device=None, batched=False):
    server = ReliableUDP().create()
    server.bind("127.0.0.1", 0)
    sport = server.socket.getsockname()[1]
    relay = Relay(sport, drop or (lambda d, i: False), batched=batched,
                  device="cuda:0" if batched else None)
    relay.start()
    got = {}
    t = threading.Thread(target=lambda: got.setdefault("msg", server.recv()), daemon=True)
    t.start()
    time.sleep(0.05)  # recv() flushes its socket on entry (reliableUDP.py:112)
    client = ReliableUDP(timeout=client_timeout, isn_source=lambda: isn,
                         codec_device=codec_device).create()
    t0 = time.perf_counter()
    client.send(message, "127.0.0.1", relay.port)
    t.join(timeout=30)
    dt = time.perf_counter() - t0
    time.sleep(0.05)
    relay.stop()
    client.close()
    server.close()
    return got.get("msg"), relay, dt


def test_config1_wire_trace_matches_reference(wire_trace):
    msg, relay, _ = run_transfer(wire_trace["message"], wire_trace["isn"])
    assert msg == wire_trace["message"]
    assert [d.hex() for d in relay.log["c2s"]] == wire_trace["client_to_server"]
    assert [d.hex() for d in relay.log["s2c"]] == wire_trace["server_to_client"]
    assert relay.retransmitted == 0
    n_c, n_s = len(wire_trace["client_to_server"]), len(wire_trace["server_to_client"])
    assert relay.stats == {"client_sent": n_c, "client_received": n_s, "client_dropped": 0,
                           "client_retransmitted": 0, "server_sent": n_s, "server_received": n_c,
                           "server_dropped": 0, "server_retransmitted": 0}


def test_config1_survives_drops(wire_trace):
    # drop the 2nd data frame once and the first server ACK once: the sender
    # times out and retransmits; the relay's __eq__ check sees the retransmits
    dropped = set()

    def drop(direction, index):
        key = (direction, index)
        if key in {("c2s", 1), ("s2c", 0)} and key not in dropped:
            dropped.add(key)
            return True
        return False
    msg, relay, _ = run_transfer(wire_trace["message"], wire_trace["isn"], drop=drop,
                                 client_timeout=0.1)
    assert msg == wire_trace["message"]
    assert relay.retransmitted >= 2


@pytest.mark.parametrize("message", ["", "x", "héllo ✓", "a" * 300])
def test_config1_messages(message):
    msg, _, _ = run_transfer(message, isn=4999, client_timeout=0.2)
    # the reference server returns what it assembled; an empty message carries no payload
    assert msg == message


@pytest.mark.gpu
def test_config1_gpu_framed_sender_matches_reference_trace(wire_trace):
    """The sender's data frames come from one GPU varlen launch; the wire
    trace is still the reference's, byte for byte."""
    msg, relay, _ = run_transfer(wire_trace["message"], wire_trace["isn"], codec_device="cuda:0")
    assert msg == wire_trace["message"]
    assert [d.hex() for d in relay.log["c2s"]] == wire_trace["client_to_server"]
    assert [d.hex() for d in relay.log["s2c"]] == wire_trace["server_to_client"]


@pytest.mark.gpu
@pytest.mark.parametrize("message", ["", "x", "héllo ✓ 𝄞", "a" * 300])
def test_config1_gpu_framed_sender_messages(message):
    """Multi-byte UTF-8 and the empty message, with drops forcing
    retransmissions of GPU-framed rows."""
    for isn in (1, 4999):
        dropped = set()

        def drop(direction, index):
            if index % 7 == 3 and (direction, index) not in dropped:
                dropped.add((direction, index))
                return True
            return False
        msg, relay, _ = run_transfer(message, isn=isn, drop=drop, client_timeout=0.1,
                                     codec_device="cuda:0")
        assert msg == message
        # every data frame on the wire equals the scalar drop-in's frame for its pointer
        from rudp.packet import Packet
        for frame in relay.log["c2s"]:
            p = Packet(frame)
            seq = int(p.get_header_field("seq_num", base=10))
            ptr = (seq - isn) % 65536
            if p.get_header_field("ack", base=2) == "1":
                continue  # the final ACK (:87-93) is scalar
            q = Packet()
            q.set_header_field("seq_num", str(isn + ptr), base=10)
            q.set_header_field("ack_num", "0", base=10)
            if ptr == 0:
                q.set_header_field("syn", "1", base=2)
            if ptr >= len(message) - 1:
                q.set_header_field("fin", "1", base=2)
            q.set_payload(message[ptr:ptr + 1])
            assert frame == q.to_byte(), (message, isn, ptr)


@pytest.mark.gpu
@pytest.mark.parametrize("isn", [1, 5000, 65500])
def test_gpu_frame_table_rows_equal_scalar_packets(isn):
    """Row p of the GPU frame table == the scalar Packet the reference builds
    for pointer p (utils/reliableUDP.py:53-61), seq wrapping past 2^16."""
    message = "ab✓𝄞" + "z" * 100
    r = ReliableUDP(isn_source=lambda: isn, codec_device="cuda:0")
    data, off = r._gpu_frames(message, isn)
    assert len(off) == len(message) + 2
    for ptr in range(len(message) + 1):
        q = Packet()
        q.set_header_field("seq_num", str(isn + ptr), base=10)
        q.set_header_field("ack_num", "0", base=10)
        if ptr == 0:
            q.set_header_field("syn", "1", base=2)
        if ptr >= len(message) - 1:
            q.set_header_field("fin", "1", base=2)
        q.set_payload(message[ptr:ptr + 1])
        assert data[off[ptr]:off[ptr + 1]] == q.to_byte(), ptr


def test_relay_history_equals_proxy_list_scan():
    """The relay's keyed history gives the proxy's `Packet(data) in self.packets`
    answer (proxy.py:81-94, 500 deep) on datagrams with repeats, empty ones and
    ones that differ only in length."""
    import random as _r
    from rudp.relay import MAX_MEMORY, Relay
    rng = _r.Random(7)
    pool = [b"", bytes(5), b"\x00", bytes(6), b"\x01\x02\x03\x04\x05", b"\x01\x02\x03\x04\x05a"] + \
        [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 9))) for _ in range(40)]
    seq = [rng.choice(pool) for _ in range(3000)]
    relay = Relay(9)  # never started: only its bookkeeping is used
    want, history = [], []
    for i, data in enumerate(seq):
        pkt = Packet(data)
        want.append(pkt in history)
        history.append(pkt)
        if len(history) > MAX_MEMORY:
            history.pop(0)
        before = relay.retransmitted
        relay._record("client", data, False)
        assert (relay.retransmitted - before == 1) == want[-1], i
    relay.sock.close()
    assert any(want) and not all(want)


def test_receiver_answers_previous_peer_across_recv_calls():
    """The receiver keeps its peer across recv() calls, as the reference keeps
    self.target_addr (utils/reliableUDP.py:18, :131, :140-146): a stray non-SYN
    datagram at the start of a later recv() -- here the previous sender's last
    frame, resent late -- is ACKed to that sender (ack = 0 + 0: no transfer yet),
    and the next transfer still goes through."""
    from rudp.transport import ACK, build, parse
    server = ReliableUDP().create()
    server.bind("127.0.0.1", 0)
    sport = server.socket.getsockname()[1]
    got = []
    t = threading.Thread(target=lambda: got.append(server.recv()), daemon=True)
    t.start()
    time.sleep(0.05)
    client = ReliableUDP(timeout=0.2, isn_source=lambda: 100).create()
    client.send("hi", "127.0.0.1", sport)
    t.join(timeout=30)
    assert got == ["hi"]
    t2 = threading.Thread(target=lambda: got.append(server.recv()), daemon=True)
    t2.start()
    time.sleep(0.05)
    late = build(100 + 1, 0, 0x20, "i")          # the first transfer's FIN frame, again
    client.socket.sendto(late, ("127.0.0.1", sport))
    client.socket.settimeout(5)
    data, _ = client.socket.recvfrom(1024)
    reply = parse(data)
    assert reply.flags == ACK and reply.ack == 0 and reply.seq == 0
    other = ReliableUDP(timeout=0.2, isn_source=lambda: 200).create()
    other.send("ok", "127.0.0.1", sport)
    t2.join(timeout=30)
    assert got == ["hi", "ok"]
    for s in (client, other, server):
        s.close()


# ------------------------------------------------------------ batched relay
@pytest.mark.gpu
def test_batched_relay_wire_trace_and_drops(wire_trace):
    """Config 1 through the batched relay (recvmmsg with sources, GPU retransmission
    flags, sendmmsg with per-datagram destinations): the reference wire trace and
    counters without drops; the message survives drops, whose retransmissions the
    GPU check counts."""
    msg, relay, _ = run_transfer(wire_trace["message"], wire_trace["isn"], batched=True)
    assert msg == wire_trace["message"]
    assert [d.hex() for d in relay.log["c2s"]] == wire_trace["client_to_server"]
    assert [d.hex() for d in relay.log["s2c"]] == wire_trace["server_to_client"]
    n_c, n_s = len(wire_trace["client_to_server"]), len(wire_trace["server_to_client"])
    assert relay.stats == {"client_sent": n_c, "client_received": n_s, "client_dropped": 0,
                           "client_retransmitted": 0, "server_sent": n_s, "server_received": n_c,
                           "server_dropped": 0, "server_retransmitted": 0}
    assert relay.batches > 0
    dropped = set()

    def drop(direction, index):
        key = (direction, index)
        if key in {("c2s", 1), ("s2c", 0)} and key not in dropped:
            dropped.add(key)
            return True
        return False
    msg, relay, _ = run_transfer(wire_trace["message"], wire_trace["isn"], drop=drop, client_timeout=0.1,
                                 batched=True)
    assert msg == wire_trace["message"] and relay.retransmitted >= 2


@pytest.mark.gpu
def test_batched_relay_counters_equal_scalar_relay():
    """Batches of 1..700 datagrams with repeats inside and across batches (the
    500-deep history carried over), empty datagrams and drops: the batched relay's
    counters, log and forwarded datagrams equal the per-datagram relay's."""
    import random as _r

    import numpy as np
    from rudp import netio
    rng = _r.Random(11)
    sink_srv = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sink_srv.bind(("127.0.0.1", 0))
    sink_cli = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sink_cli.bind(("127.0.0.1", 0))
    for s_ in (sink_srv, sink_cli):
        s_.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 24)
    srv_port, cli_port = sink_srv.getsockname()[1], sink_cli.getsockname()[1]
    pool = [b"", bytes(5), b"\x00", bytes(6)] + [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 12)))
                                                  for _ in range(300)]
    seq = []
    for _ in range(4000):
        r = rng.random()
        if r < 0.3 and seq:
            seq.append(seq[-rng.randint(1, min(len(seq), 800))])
        else:
            seq.append(rng.choice(pool))
    from_server = [rng.random() < 0.4 for _ in seq]
    from_server[0] = False  # the client speaks first
    drops = {i for i in range(len(seq)) if rng.random() < 0.1}
    index = {"c2s": 0, "s2c": 0}
    order = []
    for i, fs in enumerate(from_server):
        d = "s2c" if fs else "c2s"
        order.append((d, index[d]))
        index[d] += 1
    drop_set = {order[i] for i in drops}
    rule = lambda d, i: (d, i) in drop_set  # noqa: E731
    scalar = Relay(srv_port, rule)
    batched = Relay(srv_port, rule, batched=True, device="cuda:0")
    cli_key = netio.addr_key("127.0.0.1", cli_port)
    pos = 0
    while pos < len(seq):
        k = min(rng.randint(1, 700), len(seq) - pos)
        part = seq[pos:pos + k]
        frames = np.frombuffer(b"".join(part), np.uint8) if any(part) else np.zeros(0, np.uint8)
        off = np.concatenate([[0], np.cumsum([len(p) for p in part])]).astype(np.int64)
        src = np.array([batched._server_key if from_server[pos + j] else cli_key for j in range(k)], np.uint64)
        batched._relay_batch(frames, off, src)
        pos += k
    for i, data in enumerate(seq):
        d, j = order[i]
        scalar.log[d].append(data)
        scalar._record("server" if from_server[i] else "client", data, (d, j) in drop_set)
    assert batched.stats == scalar.stats
    assert batched.log == scalar.log
    assert batched.retransmitted > 100
    # what reached the two sinks: every non-dropped datagram of its direction, in order
    want = {"s2c": [], "c2s": []}
    for i, data in enumerate(seq):
        if i not in drops:
            want[order[i][0]].append(data)
    for sink, d in ((sink_srv, "c2s"), (sink_cli, "s2c")):
        sink.settimeout(0.5)
        got = []
        try:
            while True:
                got.append(sink.recvfrom(2048)[0])
        except socket.timeout:
            pass
        assert got == want[d], d
    for s_ in (scalar.sock, batched.sock, sink_srv, sink_cli):
        s_.close()
