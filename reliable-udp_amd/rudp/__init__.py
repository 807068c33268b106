"""rudp — MI355X-native Reliable-UDP wire codec.

``rudp.packet``  scalar drop-in for the reference's utils/packet.py
                 (``Packet``, ``custom_header``), host-side.
``rudp.batch``   batched frame/checksum/parse/verify on gfx950 through the
                 C ABI of librudp.so (include/rudp.h).
"""
from .packet import Packet, custom_header  # noqa: F401

__all__ = ["Packet", "custom_header", "pack_batch", "unpack_batch", "synth_batch",
           "HeaderTable", "make_flags"]


def __getattr__(name):
    # The batch API pulls in numpy and (on first call) torch + librudp.so;
    # importing rudp for the scalar Packet alone stays dependency-free.
    if name in ("pack_batch", "unpack_batch", "synth_batch", "HeaderTable", "make_flags",
                "DecodedBatch"):
        from . import batch
        return getattr(batch, name)
    raise AttributeError(name)
