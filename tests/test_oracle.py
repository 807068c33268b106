"""The oracle pinned against the reference's own outputs (tests/golden/).

Golden vectors were produced by the reference utils/packet.py in the build
container (tests/golden/make_golden.py).  The checksum VALUE has no
reference counterpart (the reference computes none); it is pinned by the
RFC 1071 known answer only.
"""
import numpy as np
import pytest

from conftest import small_lengths
from oracle import bitstring_packet as bp
from oracle import codec_np, synth


def test_rfc1071_known_answer():
    # RFC 1071 §3 example: sum 0xddf2, checksum 0x220d
    assert codec_np.inet_checksum(bytes.fromhex("0001f203f4f5f6f7")) == 0x220D
    assert codec_np.inet_checksum(b"") == 0xFFFF
    # odd length: trailing byte is the high half of a zero-padded word
    assert codec_np.inet_checksum(b"\x01") == (~0x0100) & 0xFFFF


def test_frame_checksum_verifies_to_all_ones():
    seq, ack, flags, pay = synth.synth(7, 0, 50, 33, ascii=False)
    fr, cs = codec_np.encode(seq, ack, flags, pay, 7)
    # rudp7: recomputing over the frame with the field zeroed gives the field back
    assert np.array_equal(codec_np.frame_checksums(fr, 7), cs)
    # identical value in both layouts (payload at an odd offset either way)
    _, cs5 = codec_np.encode(seq, ack, flags, pay, 5)
    assert np.array_equal(cs5, cs)
    for i in range(5):
        assert codec_np.inet_checksum(fr[i, :5].tobytes() + fr[i, 7:].tobytes()) == cs[i]


@pytest.mark.parametrize("layout", [5, 7])
def test_numpy_encode_matches_reference_frames(golden_small, layout):
    for L in small_lengths(golden_small):
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        fr, cs = codec_np.encode(g["seq"], g["ack"], g["flags"], g["payload"], layout)
        assert np.array_equal(fr, g[f"frames{layout}"]), f"L={L}"
        assert np.array_equal(cs, g["csum"]), f"L={L}"


@pytest.mark.parametrize("layout", [5, 7])
def test_numpy_decode_matches_reference_fields(golden_small, layout):
    for L in small_lengths(golden_small):
        fr = golden_small[f"L{L}_full_frames{layout}"]
        ref = golden_small[f"L{L}_full_fields{layout}"]
        seq, ack, flags, ok, cs, pay = codec_np.decode(fr, layout)
        assert np.array_equal(seq, ref[:, 0]) and np.array_equal(ack, ref[:, 1])
        assert np.array_equal(flags, ref[:, 2])
        if layout == 7:
            assert np.array_equal(cs, ref[:, 3]) and ok.all()
        assert np.array_equal(pay, fr[:, layout:])


def test_bitstring_port_matches_reference_frames(golden_small):
    for L in small_lengths(golden_small):
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        for i in range(0, len(g["seq"]), 5):
            args = (int(g["seq"][i]), int(g["ack"][i]), int(g["flags"][i]), g["payload"][i].tobytes())
            assert bp.encode_like_reference(*args) == g["frames5"][i].tobytes()
            assert bp.encode_like_reference(*args, csum=int(g["csum"][i])) == g["frames7"][i].tobytes()
            seq, ack, flags, cs, payload = bp.decode_like_reference(g["frames7"][i].tobytes(), rudp7=True)
            assert (seq, ack, flags, cs) == (args[0], args[1], args[2], int(g["csum"][i]))
            assert payload == (args[3].decode() if L else None)


def test_bitstring_port_matches_reference_edge_cases(edge_cases):
    from tests_support import replay
    for case in edge_cases:
        assert replay(bp.BitstringPacket, bp.REF_HEADER, case) == case["results"], case["name"]


def test_synth_is_counter_based():
    a = synth.synth(0x5EED, 0, 300, 37, ascii=True)
    b = synth.synth(0x5EED, 100, 150, 37, ascii=True)
    for x, y in zip(a, b):
        assert np.array_equal(x[100:250], y)
    seq, ack, flags, pay = a
    assert (pay < 0x80).all()
    assert set(np.unique(flags)) <= {0x00, 0x80, 0x20, 0xA0, 0x40, 0x60}
    k, isn = synth.keys(0x5EED)
    assert 1 <= isn <= 5000 and seq[0] == isn
    # splitmix64 reference value (Vigna's splitmix64 with state 0: first output)
    assert synth.mix64_int(0x9E3779B97F4A7C15) == 0xE220A8397B1DCDAF


def test_wire_trace_matches_reference_call_pattern(wire_trace):
    msg, isn = wire_trace["message"], wire_trace["isn"]
    for ptr, hexframe in enumerate(wire_trace["client_to_server"][:-1]):
        flags = (0x80 if ptr == 0 else 0) | (0x20 if ptr == len(msg) - 1 else 0)
        assert bp.encode_like_reference(isn + ptr, 0, flags, msg[ptr].encode()).hex() == hexframe


def test_c_restatement_matches_numpy_and_goldens(golden_small):
    from oracle import codec_c
    assert codec_c.inet_checksum(bytes.fromhex("0001f203f4f5f6f7")) == 0x220D
    for L in small_lengths(golden_small):
        g = {k.split("_", 1)[1]: v for k, v in golden_small.items() if k.startswith(f"L{L}_")}
        for layout in (5, 7):
            fr, cs = codec_c.encode(g["seq"], g["ack"], g["flags"], g["payload"], layout)
            assert np.array_equal(fr, g[f"frames{layout}"]) and np.array_equal(cs, g["csum"])
            full = g[f"full_frames{layout}"]
            seq, ack, flags, ok, cs2 = codec_c.decode(full, layout)
            want = codec_np.decode(full, layout)
            for a, b in zip((seq, ack, flags, ok, cs2), want[:5]):
                assert np.array_equal(a, b)
    for F in range(0, 7):
        fr = np.arange(9 * F, dtype=np.uint8).reshape(9, F)
        for layout in (5, 7):
            got = codec_c.decode(fr, layout)
            want = codec_np.decode(fr, layout)
            for a, b in zip(got, want[:5]):
                assert np.array_equal(a, b), (F, layout)


@pytest.mark.slow
@pytest.mark.parametrize("name,layout", [("C3", 5), ("C3", 7), ("C4", 7)])
def test_c_oracle_reproduces_reference_digest(digests, name, layout):
    """The C restatement frames BASELINE config chunk 0 exactly as utils/packet.py did."""
    import hashlib

    from oracle import codec_c
    cfg = digests[name]
    seq, ack, flags, pay = synth.synth(cfg["seed"], 0, cfg["chunk"], cfg["L"])
    fr, cs = codec_c.encode(seq, ack, flags, pay, layout)
    assert hashlib.sha256(fr.tobytes()).hexdigest() == cfg["layouts"][str(layout)]["frames"][0]
    assert hashlib.sha256(cs.astype("<u2").tobytes()).hexdigest() == cfg["layouts"][str(layout)]["csum"][0]


def test_varlen_oracle_matches_reference(golden_varlen):
    from conftest import split_by_lengths
    g = golden_varlen
    pays, _ = split_by_lengths(g["payload"], g["lengths"])
    for layout in (5, 7):
        fr, off, cs = codec_np.encode_varlen(g["seq"], g["ack"], g["flags"], pays, layout)
        assert np.array_equal(fr, g[f"frames{layout}"]) and np.array_equal(cs, g["csum"])
        assert off[-1] == len(fr) and np.array_equal(np.diff(off), g["lengths"] + layout)
        seq, ack, flags, ok, cs2 = codec_np.decode_varlen(fr, off, layout,
                                                           g["csum"] if layout == 5 else None)
        assert np.array_equal(seq, g["seq"]) and np.array_equal(flags, g["flags"])
        assert (ok == 1).all() and np.array_equal(cs2, g["csum"])


def test_utf8_oracle_matches_reference_get_payload(golden_varlen):
    from conftest import split_by_lengths
    g = golden_varlen
    bodies, _ = split_by_lengths(g["utf8_bodies"], g["utf8_lengths"])
    frames = [b"\x00\x01\x00\x02\x40" + b for b in bodies]
    off = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.int64)
    flat = np.frombuffer(b"".join(frames), np.uint8)
    assert np.array_equal(codec_np.utf8_valid(flat, off, 5), g["utf8_valid"])


def test_proxy_dedup_oracle_matches_reference(golden_dedup):
    from conftest import split_by_lengths
    frames, _ = split_by_lengths(golden_dedup["frames"], golden_dedup["lengths"])
    assert bp.proxy_retransmitted(frames, 500) == golden_dedup["dup"].tolist()


def test_proxy_dedup_with_dropin_packet(golden_dedup):
    """The proxy's own loop (proxy.py:90-94) over the drop-in Packet gives the same flags."""
    from conftest import split_by_lengths
    from rudp.packet import Packet
    frames, _ = split_by_lengths(golden_dedup["frames"], golden_dedup["lengths"])
    history, dup = [], []
    for data in frames:
        pkt = Packet(data)
        dup.append(1 if pkt in history else 0)
        history.append(pkt)
        if len(history) > 500:
            history.pop(0)
    assert dup == golden_dedup["dup"].tolist()
