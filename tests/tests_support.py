"""Shared helpers for the golden-vector tests (no reference code in here)."""
from __future__ import annotations

# Header definitions the scripted edge cases use, by name.
ONE_BIT = {"a": 1 / 8}                                    # non-byte-aligned header
ZERO_WIDTH = {"seq_num": 2, "z": 0, "ack_num": 2}         # a zero-width field


def definition(custom_header, name):
    if name == "ref":
        return custom_header
    if name == "rudp7":
        return {**custom_header, "checksum": 2}
    if name == "one_bit":
        return ONE_BIT
    if name == "zero_width":
        return ZERO_WIDTH
    raise KeyError(name)


def run_script(Packet, custom_header, steps):
    """Execute one scripted case on a Packet class; returns per-step outcomes.

    Each outcome is {"ok": value} or {"exc": exception type name, "msg": str}.
    The same function produced tests/golden/edge_cases.json from the
    reference utils/packet.py, so a drop-in must reproduce it exactly.
    """
    out = []
    p = None
    for st in steps:
        op = st[0]
        try:
            if op == "new":
                raw = bytes.fromhex(st[1]) if st[1] is not None else None
                d = definition(custom_header, st[2])
                p = Packet(raw) if d is custom_header else Packet(raw, header_definition=d)
                res = None
            elif op == "get":
                res = p.get_header_field(st[1], st[2])
            elif op == "set":
                res = p.set_header_field(st[1], st[2], st[3])
            elif op == "pos":
                res = list(p.get_header_field_position(st[1]))
            elif op == "set_payload":
                res = p.set_payload(st[1])
            elif op == "get_payload":
                res = p.get_payload()
            elif op == "get_hex":
                res = p.get_hex()
            elif op == "to_byte":
                res = p.to_byte().hex()
            elif op == "binary":
                res = p.binary
            elif op == "hlb":
                res = p.header_length_bits
            elif op == "eq_hex":
                res = p == Packet(bytes.fromhex(st[1]))
            elif op == "eq_other":
                res = p == st[1]
            else:
                raise AssertionError(op)
            out.append({"ok": res})
        except Exception as e:  # noqa: BLE001 - the exception IS the recorded result
            out.append({"exc": type(e).__name__, "msg": str(e)})
    return out


def replay(Packet, custom_header, case):
    return run_script(Packet, custom_header, case["steps"])
