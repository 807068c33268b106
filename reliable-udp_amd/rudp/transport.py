"""Stop-and-wait ARQ over UDP: the caller of the codec (config 1).

Counterpart of the reference's utils/reliableUDP.py (class ReliableUDP,
:8-202), which is the only production caller of utils/packet.py.  It is
rewritten here because the reference file does not parse below Python 3.12
(PEP 701 f-string at :50).  It stays scalar Python, like the reference: one
character per datagram (:11), so every frame is 5-9 bytes and by default goes
through the host-side drop-in rudp.packet.Packet.

Same public surface: ReliableUDP(timeout).create() / bind(ip, port) /
send(message, ip, port) / recv() / close() / flush_recv_buffer().  Same
protocol and wire bytes: the states of the reference's FSM tables (:96-107 and
:186-199) are the methods below, with the same transitions, retry counts,
timeouts and header values.  The config-1 wire trace (tests/golden/
wire_trace.json, captured from the reference) is reproduced byte for byte.

``ReliableUDP(codec_device="cuda:0")`` moves the sender's data frames
(:53-61) onto the GPU codec: every frame send() can emit is known once the
ISN is drawn (pointer p: seq = ISN + p, ack 0, SYN at p = 0, FIN from the last
character on, payload message[p]), so send() frames the whole message in one
pack_batch_varlen launch (rudp5, the reference's 5-byte layout) and each
SEND_DATA step, retransmissions included, sends row p of that table.  The
bytes on the wire are the same.
"""
from __future__ import annotations

import ipaddress
import random
from socket import AF_INET, SOCK_DGRAM, socket
from typing import Any, Callable, Optional

from .packet import Packet


class ReliableUDP:
    BUFFER_SIZE = 1024      # utils/reliableUDP.py:9
    RETRIES = 20            # :10
    PAYLOAD_SIZE = 1        # :11

    def __init__(self, timeout=1, isn_source: Optional[Callable[[], int]] = None,
                 codec_device: Optional[str] = None):
        self.socket: socket
        self.message_pointer = 0
        self.random_number = 0
        self.prev_random_number = None
        self.target_addr: Any = None
        self.retransmission_timeout = timeout
        # the ISN draw of :41; injectable so a test can pin the wire trace
        self._isn = isn_source or (lambda: random.randint(1, 5000))
        self._codec_device = codec_device
        self._frames: Optional[tuple] = None  # (bytes, offsets) of the pre-framed message

    def create(self):
        self.socket = socket(AF_INET, SOCK_DGRAM)
        return self

    def bind(self, ip, port):
        self.socket.bind((str(ipaddress.ip_address(ip)), port))

    def flush_recv_buffer(self):
        try:
            self.socket.setblocking(False)
            while self.socket.recvfrom(65535):
                continue
        except BlockingIOError:
            pass
        finally:
            self.socket.setblocking(True)

    def close(self):
        self.socket.close()

    # ------------------------------------------------------------- sender
    def send(self, message, ip, port):
        """utils/reliableUDP.py:38-108 — SEND_DATA <-> WAIT_ACK -> SEND_ACK -> EXIT."""
        self.flush_recv_buffer()
        self.message_pointer = 0
        self.random_number = self._isn()
        self._frames = self._frame_message(message) if self._codec_device else None
        dest = (str(ip), port)
        state, args = "SEND_DATA", (ReliableUDP.RETRIES,)
        while True:
            if state == "SEND_DATA":
                step = self._send_data(message, dest, *args)
            elif state == "WAIT_ACK":
                step = self._wait_ack(message, *args)
            else:  # SEND_ACK
                self._send_final_ack(ip, port, *args)
                break
            if step is None:  # EXIT after the retries ran out
                break
            state, args = step[0], step[1:]
        self.flush_recv_buffer()

    def _frame_message(self, message):
        """Frames for pointer values 0..len(message), in one GPU launch."""
        import numpy as np
        import torch
        from . import batch
        dev = torch.device(self._codec_device)
        n = len(message) + 1  # p = len(message): the header-only FIN frame (empty payload)
        p = np.arange(n, dtype=np.int64)
        seq = ((self.random_number + p) & 0xFFFF).astype(np.uint16)
        flags = np.where(p == 0, 0x80, 0) | np.where(p >= len(message) - 1, 0x20, 0)
        lens = np.array([len(c.encode()) for c in message] + [0], dtype=np.int32)
        payload = np.frombuffer(bytearray(message.encode()), dtype=np.uint8)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        res = batch.pack_batch_varlen((t(seq), t(np.zeros(n, np.uint16)), t(flags.astype(np.uint8))),
                                      t(payload), t(lens), "rudp5", want_csum=False)
        return res.frames.cpu().numpy().tobytes(), res.frame_off.cpu().tolist()

    def _send_data(self, message, dest, retries):
        # :43-62
        end = min(self.message_pointer + ReliableUDP.PAYLOAD_SIZE, len(message))
        is_first = self.message_pointer == 0
        is_last = end == len(message)
        if retries < 1:
            if not is_last:
                sent = message[:self.message_pointer]
                tail = f"\n'{sent}'" if self.message_pointer > 0 else ""
                print(f"\033[91mAborted after {ReliableUDP.RETRIES * self.retransmission_timeout} "
                      f"seconds ({ReliableUDP.RETRIES} retries * {self.retransmission_timeout} "
                      f"second timeout) {tail} \033[0m")
            return None
        if self._frames is not None:
            data, off = self._frames
            frame = data[off[self.message_pointer]:off[self.message_pointer + 1]]
        else:
            p = Packet()
            p.set_header_field("seq_num", str(self.message_pointer + self.random_number), base=10)
            p.set_header_field("ack_num", "0", base=10)
            if is_first:
                p.set_header_field("syn", "1", base=2)
            if is_last:
                p.set_header_field("fin", "1", base=2)
            p.set_payload(message[self.message_pointer:end])
            frame = p.to_byte()
        self.socket.sendto(frame, dest)
        return ("WAIT_ACK", is_last, end - self.message_pointer, retries - 1)

    def _wait_ack(self, message, is_last, payload_length, retries):
        # :64-85
        try:
            self.socket.settimeout(self.retransmission_timeout)
            data, _ = self.socket.recvfrom(ReliableUDP.BUFFER_SIZE)
            p = Packet(data)
            ack_num = int(p.get_header_field("ack_num", base=10))
            seq_num = int(p.get_header_field("seq_num", base=10))
            is_valid = ack_num == self.random_number + self.message_pointer + payload_length
            is_ack = is_valid and p.get_header_field("ack", base=2) == "1"
            is_fin = is_valid and p.get_header_field("fin", base=2) == "1"
            if not is_valid:
                return ("WAIT_ACK", is_last, payload_length, retries)
            if is_ack:
                self.message_pointer = ack_num - self.random_number
            if is_fin:
                return ("SEND_ACK", seq_num)
            if is_last:
                return ("WAIT_ACK", True, 0, retries)
            return ("SEND_DATA", ReliableUDP.RETRIES)
        except TimeoutError:
            return ("SEND_DATA", retries)

    def _send_final_ack(self, ip, port, last_seq_num):
        # :87-93
        p = Packet()
        p.set_header_field("seq_num", str(self.random_number + self.message_pointer), base=10)
        p.set_header_field("ack_num", str(last_seq_num + 1), base=10)
        p.set_header_field("ack", "1", base=2)
        self.socket.sendto(p.to_byte(), (str(ipaddress.ip_address(ip)), port))

    # ----------------------------------------------------------- receiver
    def recv(self):
        """utils/reliableUDP.py:111-199 — RECEIVE_DATA <-> SEND_ACK -> SEND_FIN <-> WAIT_ACK."""
        self.flush_recv_buffer()
        self.message_pointer = 0
        self.random_number = 0
        state, args = "RECEIVE_DATA", ("",)
        while True:
            if state == "RECEIVE_DATA":
                state, *args = self._receive_data(*args)
            elif state == "SEND_ACK":
                state, *args = self._send_ack(*args)
            elif state == "SEND_FIN":
                state, *args = self._send_fin(*args)
            elif state == "WAIT_ACK":
                state, *args = self._wait_fin_ack(*args)
            else:  # EXIT
                return self._clean_up(*args)

    def _receive_data(self, buffer=""):
        # :116-137
        self.socket.settimeout(None)
        data, addr = self.socket.recvfrom(ReliableUDP.BUFFER_SIZE)
        p = Packet(data)
        seq_num = int(p.get_header_field("seq_num", base=10))
        payload = p.get_payload() or ""
        is_last_message = p.get_header_field("fin", base=2) == "1"
        is_syn = p.get_header_field("syn", base=2) == "1"
        is_valid = (self.message_pointer == 0 and is_syn) or \
            seq_num - self.random_number == self.message_pointer
        is_new_connection = is_syn and not is_valid
        is_duplicate_syn = is_syn and seq_num == self.prev_random_number
        if is_syn and not is_duplicate_syn:
            self.random_number = seq_num
            self.message_pointer = 0
            self.target_addr = addr
            buffer = ""
        if (is_valid or is_new_connection) and not is_duplicate_syn:
            self.message_pointer = len(buffer + payload)
            return ("SEND_ACK", buffer + payload, is_last_message)
        return ("SEND_ACK", buffer, False)

    def _send_ack(self, acknowledged_message, is_last_message):
        # :139-150
        if not self.target_addr:
            return ("RECEIVE_DATA", "")
        p = Packet()
        p.set_header_field("ack", "1", base=2)
        p.set_header_field("seq_num", "0", base=10)
        p.set_header_field("ack_num", str(self.random_number + len(acknowledged_message)), base=10)
        self.socket.sendto(p.to_byte(), self.target_addr)
        if is_last_message:
            return ("SEND_FIN", acknowledged_message, 20)
        return ("RECEIVE_DATA", acknowledged_message)

    def _send_fin(self, message, retries):
        # :152-162
        if retries < 1:
            return ("EXIT", message)
        p = Packet()
        p.set_header_field("fin", "1", base=2)
        p.set_header_field("ack", "1", base=2)
        p.set_header_field("seq_num", "0", base=10)
        p.set_header_field("ack_num", str(self.random_number + len(message)), base=10)
        self.socket.sendto(p.to_byte(), self.target_addr)
        return ("WAIT_ACK", message, retries - 1)

    def _wait_fin_ack(self, message, retries):
        # :164-176
        try:
            self.socket.settimeout(0.5)
            data, _ = self.socket.recvfrom(ReliableUDP.BUFFER_SIZE)
            p = Packet(data)
            is_ack = p.get_header_field("ack", base=2) == "1"
            ack_num = int(p.get_header_field("ack_num", base=10))
            if is_ack and ack_num == 1:
                return ("EXIT", message)
            return ("SEND_FIN", message, retries)
        except TimeoutError:
            return ("SEND_FIN", message, retries)

    def _clean_up(self, message):
        # :178-183
        self.message_pointer = 0
        self.prev_random_number = self.random_number
        self.random_number = 0
        self.flush_recv_buffer()
        return message
