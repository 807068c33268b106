"""Drop-in replacement for the reference module utils/packet.py.

Same public surface: the module global ``custom_header`` (utils/packet.py:3-10)
and class ``Packet`` (utils/packet.py:12-86) with identical method names,
signatures, return types, attribute names and exceptions, so that
utils/reliableUDP.py and proxy.py run unchanged against it.

The reference keeps the datagram as a Python ``str`` of '0'/'1' characters
(utils/packet.py:16) and converts to and from it on every call.  This class
keeps the same logical bit string as an ``int`` plus a bit count, so parsing,
field access and serialising are integer shifts and ``int.to_bytes`` instead
of string building: same results, including the reference's edge cases
(truncated fields of short frames, low-bit truncation on set, the
empty-payload no-op, strict UTF-8 payloads, non-byte-aligned header
definitions).  A value that is not made of binary digits (e.g. a negative
number, which the reference splices in as '...b101') switches the instance to
an explicit string so later calls fail exactly where the reference fails.

This is the scalar, per-datagram API and stays on the host: one GPU launch
costs more than framing a 5-9 byte datagram.  Batches go to the HIP kernels
through rudp.batch.pack_batch / unpack_batch.
"""
from typing import Optional, Union

custom_header = {
    "seq_num": 2,
    "ack_num": 2,
    "syn": 1 / 8,
    "ack": 1 / 8,
    "fin": 1 / 8,
    "offset": 5 / 8,  # pads the header to 40 bits (utils/packet.py:9)
}

_BINARY_DIGITS = frozenset("01")


def _is_binary(s: str) -> bool:
    return not (set(s) - _BINARY_DIGITS)


class Packet:
    def __init__(self, packet: Optional[bytes] = None, header_definition=custom_header):
        # utils/packet.py:13-16
        self.header_definition = header_definition
        self.header_length_bits = int(sum(header_definition.values()) * 8)
        self._raw = None  # str form, only when the bits are not all binary digits
        if packet:
            digits = packet.hex()
            self._v = int(digits, 16)
            self._n = len(digits) * 4
        else:
            self._v = 0
            self._n = self.header_length_bits if self.header_length_bits > 0 else 0

    # -- the reference's public attribute `binary` (utils/packet.py:16) -------
    @property
    def binary(self) -> str:
        if self._raw is not None:
            return self._raw
        return format(self._v, "0%db" % self._n) if self._n else ""

    @binary.setter
    def binary(self, bits: str) -> None:
        if isinstance(bits, str) and _is_binary(bits):
            self._raw = None
            self._v = int(bits, 2) if bits else 0
            self._n = len(bits)
        else:
            self._raw = bits

    def _cut(self, start, stop):
        """(value, length) of self.binary[start:stop], Python slice rules."""
        a, b, _ = slice(start, stop).indices(self._n)
        length = b - a if b > a else 0
        if not length:
            return 0, 0
        return (self._v >> (self._n - b)) & ((1 << length) - 1), length

    # -- utils/packet.py:19-26 -------------------------------------------------
    def get_header_field_position(self, field_name):
        bit_pointer = 0
        for key, size in self.header_definition.items():
            width = int(size * 8)
            if key == field_name:
                return (bit_pointer, bit_pointer + width)
            bit_pointer += width
        raise ValueError(f"Field '{field_name}' not found in header definition")

    # -- utils/packet.py:29-40 -------------------------------------------------
    def get_header_field(self, field_name: str, base: int = 16):
        bit_start, bit_end = self.get_header_field_position(field_name)
        if self._raw is not None:
            bits = self._raw[bit_start:bit_end]
            if base == 2:
                return bits
            if base == 10:
                return str(int(bits, 2))
            if base == 16:
                return hex(int(bits, 2))[2:]
            raise ValueError("Unsupported base")
        value, length = self._cut(bit_start, bit_end)
        if base == 2:
            return format(value, "0%db" % length) if length else ""
        if base not in (10, 16):
            raise ValueError("Unsupported base")
        if not length:
            int("", 2)  # the reference parses an empty slice: same ValueError
        return str(value) if base == 10 else format(value, "x")

    # -- utils/packet.py:43-57 -------------------------------------------------
    def set_header_field(self, field_name: str, value: str, base=16):
        bit_start, bit_end = self.get_header_field_position(field_name)
        if base == 16:
            bits = bin(int(value, 16))[2:]
        elif base == 10:
            bits = bin(int(value))[2:]
        elif base == 2:
            bits = value
        else:
            raise ValueError("Unsupported base")
        width = bit_end - bit_start
        bits = bits.zfill(width)[-width:]  # keeps the low `width` bits
        if self._raw is None and _is_binary(bits):
            head, head_n = self._cut(None, bit_start)
            tail, tail_n = self._cut(bit_end, None)
            field = int(bits, 2) if bits else 0
            self._v = (((head << len(bits)) | field) << tail_n) | tail
            self._n = head_n + len(bits) + tail_n
        else:
            whole = self.binary
            self.binary = whole[:bit_start] + bits + whole[bit_end:]

    # -- utils/packet.py:60-65 -------------------------------------------------
    def set_payload(self, data: str):
        if len(data) == 0:
            return  # the reference keeps any previous payload
        raw = data.encode()
        if self._raw is not None:
            self.binary = self._raw[:self.header_length_bits] + format(
                int.from_bytes(raw, "big"), "0%db" % (8 * len(raw)))
            return
        head, head_n = self._cut(None, self.header_length_bits)
        self._v = (head << (8 * len(raw))) | int.from_bytes(raw, "big")
        self._n = head_n + 8 * len(raw)

    # -- utils/packet.py:68-73 -------------------------------------------------
    def get_payload(self) -> Union[str, None]:
        if self._raw is not None:
            bits = self._raw[self.header_length_bits:]
            if len(bits) == 0:
                return None
            return bytes.fromhex(hex(int(bits, 2))[2:].zfill(len(bits) // 4)).decode()
        value, length = self._cut(self.header_length_bits, None)
        if not length:
            return None
        if length % 8 == 0:
            return value.to_bytes(length // 8, "big").decode()
        return bytes.fromhex(format(value, "x").zfill(length // 4)).decode()

    # -- utils/packet.py:76-77 -------------------------------------------------
    def get_hex(self) -> str:
        if self._raw is not None:
            return hex(int(self._raw, 2))[2:].zfill(len(self._raw) // 4)
        if not self._n:
            int("", 2)  # empty bit string: the reference's ValueError
        return format(self._v, "x").zfill(self._n // 4)

    # -- utils/packet.py:80-81 -------------------------------------------------
    def to_byte(self) -> bytes:
        if self._raw is None and self._n and self._n % 8 == 0:
            return self._v.to_bytes(self._n // 8, "big")
        return bytes.fromhex(self.get_hex())

    # -- utils/packet.py:83-86 -------------------------------------------------
    def __eq__(self, value: object) -> bool:
        if isinstance(value, Packet):
            if self._raw is None and value._raw is None and self._n == value._n and self._n:
                return self._v == value._v
            return value.get_hex() == self.get_hex()
        return False
