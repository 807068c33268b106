"""rudp.packet (the scalar drop-in) against the reference's recorded behaviour.

The drop-in must reproduce utils/packet.py exactly: results, attribute values
and exception types + messages.  Pinned by the golden script
results the reference produced, plus randomized op sequences checked against
the bit-string restatement in oracle/.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import small_lengths
from oracle.bitstring_packet import BitstringPacket, REF_HEADER
from rudp import packet as dropin
from tests_support import replay, run_script


def test_module_surface():
    assert dropin.custom_header == REF_HEADER
    assert list(dropin.custom_header) == ["seq_num", "ack_num", "syn", "ack", "fin", "offset"]
    p = dropin.Packet()
    for attr in ("header_definition", "header_length_bits", "binary"):
        assert hasattr(p, attr)
    with pytest.raises(TypeError):
        hash(p)  # __eq__ without __hash__, like the reference


def test_edge_cases_match_reference(edge_cases):
    for case in edge_cases:
        assert replay(dropin.Packet, dropin.custom_header, case) == case["results"], case["name"]


def test_golden_frames_through_dropin(golden_small):
    for L in small_lengths(golden_small):
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        for i in range(len(g["seq"])):
            s, a, f = int(g["seq"][i]), int(g["ack"][i]), int(g["flags"][i])
            # encode as utils/reliableUDP.py:53-61 does
            p = dropin.Packet()
            p.set_header_field("seq_num", str(s), base=10)
            p.set_header_field("ack_num", str(a), base=10)
            p.set_header_field("syn", str(f >> 7 & 1), base=2)
            p.set_header_field("ack", str(f >> 6 & 1), base=2)
            p.set_header_field("fin", str(f >> 5 & 1), base=2)
            p.set_header_field("offset", format(f & 31, "b"), base=2)
            p.set_payload(g["payload"][i].tobytes().decode())
            assert p.to_byte() == g["frames5"][i].tobytes()
            # decode as utils/reliableUDP.py:118-123 does
            q = dropin.Packet(g["frames7"][i].tobytes(), header_definition={**dropin.custom_header, "checksum": 2})
            assert int(q.get_header_field("seq_num", base=10)) == s
            assert int(q.get_header_field("checksum", base=16), 16) == int(g["csum"][i])
            assert q.get_payload() == (g["payload"][i].tobytes().decode() if L else None)
            assert q == dropin.Packet(g["frames7"][i].tobytes())


def test_full_range_frames_parse_like_reference(golden_small):
    for L in small_lengths(golden_small):
        fr = golden_small[f"L{L}_full_frames5"]
        ref = golden_small[f"L{L}_full_fields5"]
        for i in range(len(fr)):
            p = dropin.Packet(fr[i].tobytes())
            assert int(p.get_header_field("seq_num", 10)) == ref[i, 0]
            assert int(p.get_header_field("ack_num", 10)) == ref[i, 1]
            flags = (int(p.get_header_field("syn", 2)) << 7 | int(p.get_header_field("ack", 2)) << 6
                     | int(p.get_header_field("fin", 2)) << 5 | int(p.get_header_field("offset", 2), 2))
            assert flags == ref[i, 2]
            assert p.get_hex() == fr[i].tobytes().hex()


# ---------------------------------------------------------------- properties
FIELDS = ["seq_num", "ack_num", "syn", "ack", "fin", "offset", "checksum", "bogus"]
_value = st.one_of(
    st.integers(min_value=-70000, max_value=1 << 20).map(str),
    st.sampled_from(["0", "1", "101", "ffff", "0x1f", "-a", "", "x", "  7 "]),
    st.text(alphabet="01", min_size=0, max_size=20),
)
_op = st.one_of(
    st.tuples(st.just("get"), st.sampled_from(FIELDS), st.sampled_from([2, 10, 16, 8])),
    st.tuples(st.just("set"), st.sampled_from(FIELDS), _value, st.sampled_from([2, 10, 16, 3])),
    st.tuples(st.just("set_payload"), st.text(max_size=12)),
    st.tuples(st.just("get_payload")),
    st.tuples(st.just("get_hex")),
    st.tuples(st.just("to_byte")),
    st.tuples(st.just("binary")),
    st.tuples(st.just("eq_hex"), st.binary(min_size=1, max_size=8).map(bytes.hex)),
)
_start = st.one_of(st.none().map(lambda _: None), st.binary(max_size=12).map(bytes.hex))


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(start=_start, rudp7=st.booleans(), ops=st.lists(_op, max_size=10))
def test_random_op_sequences_match_bitstring_port(start, rudp7, ops):
    steps = [["new", start, "rudp7" if rudp7 else "ref"]] + [list(o) for o in ops]
    ours = run_script(dropin.Packet, dropin.custom_header, steps)
    theirs = run_script(BitstringPacket, REF_HEADER, steps)
    assert ours == theirs


@settings(max_examples=200, deadline=None)
@given(frame=st.binary(max_size=64))
def test_parse_any_bytes_matches_bitstring_port(frame):
    steps = [["new", frame.hex(), "ref"], ["get", "seq_num", 10], ["get", "ack_num", 16],
             ["get", "syn", 2], ["get", "offset", 10], ["get_payload"], ["get_hex"], ["to_byte"],
             ["binary"]]
    assert run_script(dropin.Packet, dropin.custom_header, steps) == \
        run_script(BitstringPacket, REF_HEADER, steps)


def test_binary_setter_roundtrip():
    p = dropin.Packet()
    p.binary = "0" * 40 + format(ord("A"), "08b")
    assert p.get_payload() == "A"
    p.binary = "10x"
    with pytest.raises(ValueError):
        p.get_hex()


def test_thread_safety_smoke():
    # The proxy builds Packets from ThreadPoolExecutor workers (proxy.py:127, :154):
    # instances share no state.
    from concurrent.futures import ThreadPoolExecutor
    frames = [bytes([i, i, 0, 0, 0x40, 65 + i % 26]) for i in range(200)]

    def work(b):
        return dropin.Packet(b).get_payload()
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(work, frames))
    assert got == [chr(65 + i % 26) for i in range(200)]
