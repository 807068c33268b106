"""Stop-and-wait transfer of one message over UDP: the codec's caller (config 1).

The reference's only production caller of utils/packet.py is its
utils/reliableUDP.py (class ReliableUDP, :8-202), which does not parse below
Python 3.12 (PEP 701 f-string at :50).  This module is written from the
protocol it implements and the wire trace captured from it
(tests/golden/wire_trace.json): the same public surface, the same bytes on the
wire, organised as two loops, one per role.

Protocol (one character of payload per datagram, utils/reliableUDP.py:11):

* sender — draws an ISN in [1, 5000]; frame k carries message[k] with
  seq = ISN + k, ack 0, SYN on k = 0 and FIN on the last character (an empty
  message is one SYN|FIN frame).  It waits ``timeout`` seconds for a reply
  whose ack_num is ISN + k + len(payload); other replies are ignored, a
  timeout resends frame k.  Twenty sends without progress abort the transfer.
  An ACK moves k to ack_num - ISN.  After the last frame it keeps waiting for
  the receiver's FIN, answers it with ACK(seq = ISN + k, ack = peer seq + 1)
  and returns.
* receiver — answers the sender of the last SYN it accepted (kept across
  recv() calls, so a stray frame before the next SYN is ACKed there); accepts
  a SYN (unless it repeats the previous transfer's ISN) as
  a new transfer and then the frame whose seq - ISN equals the characters
  received so far; every datagram is answered with ACK(ack = ISN + characters
  received).  After accepting a FIN frame it sends FIN|ACK(ack = ISN + length)
  up to twenty times, half a second apart, until an ACK with ack_num 1 comes
  back, and returns the message.

``ReliableUDP(codec_device="cuda:0")`` frames the sender's data frames on the
GPU: every frame a transfer can send is known once the ISN is drawn, so one
pack_batch_varlen launch (rudp5, the reference's 5-byte layout) builds the
table and each send, retransmissions included, takes row k.  Same wire bytes.
"""
from __future__ import annotations

import ipaddress
import random
from socket import AF_INET, SOCK_DGRAM, socket
from typing import Any, Callable, NamedTuple, Optional

from .batch import ACK, FIN, SYN
from .packet import Packet

MAX_DATAGRAM = 1024   # recvfrom size of the reference (utils/reliableUDP.py:9)
MAX_SENDS = 20        # sends without progress before giving up (:10)
CHUNK = 1             # characters per datagram (:11)
FIN_WAIT_S = 0.5      # receiver's wait for the final ACK (:166)


class Reply(NamedTuple):
    seq: int
    ack: int
    flags: int
    payload: str


def build(seq: int, ack: int, flags: int, payload: str = "") -> bytes:
    """One frame through the drop-in codec (seq/ack taken mod 2^16 as
    set_header_field keeps the low 16 bits, utils/packet.py:56)."""
    p = Packet()
    p.set_header_field("seq_num", str(seq), base=10)
    p.set_header_field("ack_num", str(ack), base=10)
    for name, bit in (("syn", SYN), ("ack", ACK), ("fin", FIN)):
        if flags & bit:
            p.set_header_field(name, "1", base=2)
    p.set_payload(payload)
    return p.to_byte()


def parse(data: bytes) -> Reply:
    p = Packet(data)
    flags = sum(bit for name, bit in (("syn", SYN), ("ack", ACK), ("fin", FIN))
                if p.get_header_field(name, base=2) == "1")
    return Reply(int(p.get_header_field("seq_num", base=10)), int(p.get_header_field("ack_num", base=10)),
                 flags, p.get_payload() or "")


class ReliableUDP:
    BUFFER_SIZE = MAX_DATAGRAM
    RETRIES = MAX_SENDS
    PAYLOAD_SIZE = CHUNK

    def __init__(self, timeout=1, isn_source: Optional[Callable[[], int]] = None,
                 codec_device: Optional[str] = None):
        self.socket: socket
        self.retransmission_timeout = timeout
        self._draw_isn = isn_source or (lambda: random.randint(1, 5000))
        self._codec_device = codec_device
        self._last_isn: Optional[int] = None  # the previous transfer's ISN (a repeated SYN is ignored)
        # the sender of the last SYN, kept across recv() calls as the reference
        # keeps self.target_addr (utils/reliableUDP.py:18, :131 only ever set it):
        # a stray non-SYN datagram at the start of a later recv() is answered there
        self._peer: Any = None

    # ------------------------------------------------------------ socket
    def create(self):
        self.socket = socket(AF_INET, SOCK_DGRAM)
        return self

    def bind(self, ip, port):
        self.socket.bind((str(ipaddress.ip_address(ip)), port))

    def close(self):
        self.socket.close()

    def flush_recv_buffer(self):
        """Drop whatever is queued on the socket (stale replies of an earlier transfer)."""
        self.socket.setblocking(False)
        try:
            while True:
                self.socket.recvfrom(65535)
        except BlockingIOError:
            pass
        finally:
            self.socket.setblocking(True)

    def _receive(self, timeout: Optional[float]):
        """(Reply, addr), or None when nothing arrived within `timeout` seconds."""
        self.socket.settimeout(timeout)
        try:
            data, addr = self.socket.recvfrom(MAX_DATAGRAM)
        except TimeoutError:
            return None
        return parse(data), addr

    # ------------------------------------------------------------ sender
    def send(self, message: str, ip, port) -> None:
        self.flush_recv_buffer()
        try:
            self._transmit(message, (str(ipaddress.ip_address(ip)), port))
        finally:
            self.flush_recv_buffer()

    def _transmit(self, message: str, dest) -> None:
        isn = self._draw_isn()
        table = self._gpu_frames(message, isn) if self._codec_device else None
        k, sends_left = 0, MAX_SENDS
        expect = None  # (ack_num that acknowledges the outstanding frame, it was the last one)
        while True:
            if expect is None:  # (re)send frame k
                n = CHUNK if k < len(message) else 0
                last = k + n >= len(message)
                if sends_left < 1:
                    if not last:
                        print(f"\033[91mAborted after {MAX_SENDS * self.retransmission_timeout} seconds "
                              f"({MAX_SENDS} sends of character {k} unacknowledged)\033[0m")
                    return
                if table is not None:
                    frame = table[0][table[1][k]:table[1][k + 1]]
                else:
                    flags = (SYN if k == 0 else 0) | (FIN if last else 0)
                    frame = build(isn + k, 0, flags, message[k:k + n])
                self.socket.sendto(frame, dest)
                sends_left -= 1
                expect = (isn + k + n, last)
            got = self._receive(self.retransmission_timeout)
            if got is None:
                expect = None  # timeout: resend
                continue
            reply = got[0]
            if reply.ack != expect[0]:
                continue  # not for the outstanding frame
            if reply.flags & ACK:
                k = reply.ack - isn
            if reply.flags & FIN:
                self.socket.sendto(build(isn + k, reply.seq + 1, ACK), dest)
                return
            if expect[1]:
                expect = (isn + k, True)  # everything is sent: wait for the FIN
            else:
                expect, sends_left = None, MAX_SENDS

    def _gpu_frames(self, message: str, isn: int):
        """Frames for k = 0..len(message) in one GPU launch: (bytes, offsets)."""
        import numpy as np
        import torch
        from . import batch
        dev = torch.device(self._codec_device)
        n = len(message) + 1  # k = len(message): the header-only FIN frame a late resend carries
        k = np.arange(n, dtype=np.int64)
        seq = ((isn + k) & 0xFFFF).astype(np.uint16)
        flags = (np.where(k == 0, SYN, 0) | np.where(k >= len(message) - 1, FIN, 0)).astype(np.uint8)
        lens = np.array([len(c.encode()) for c in message] + [0], dtype=np.int32)
        payload = np.frombuffer(bytearray(message.encode()), dtype=np.uint8)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        res = batch.pack_batch_varlen((t(seq), t(np.zeros(n, np.uint16)), t(flags)), t(payload), t(lens),
                                      "rudp5", want_csum=False)
        return res.frames.cpu().numpy().tobytes(), res.frame_off.cpu().tolist()

    # ----------------------------------------------------------- receiver
    def recv(self) -> str:
        self.flush_recv_buffer()
        isn, text, peer = 0, "", self._peer
        received = 0  # characters accepted so far (the next in-order frame is isn + received)
        while True:
            reply, addr = self._receive(None)
            syn = bool(reply.flags & SYN)
            in_order = (received == 0 and syn) or reply.seq - isn == received
            repeated_syn = syn and reply.seq == self._last_isn
            finished = False
            if syn and not repeated_syn:  # a new transfer starts here
                isn, received, peer, text = reply.seq, 0, addr, ""
                self._peer = peer
            if (in_order or syn) and not repeated_syn:
                text += reply.payload
                received = len(text)
                finished = bool(reply.flags & FIN)
            if peer is None:  # nothing to answer yet
                text = ""
                continue
            self.socket.sendto(build(0, isn + len(text), ACK), peer)
            if finished:
                break
        for _ in range(MAX_SENDS):
            self.socket.sendto(build(0, isn + len(text), FIN | ACK), peer)
            got = self._receive(FIN_WAIT_S)
            if got is not None and got[0].flags & ACK and got[0].ack == 1:
                break
        self._last_isn = isn
        self.flush_recv_buffer()
        return text
