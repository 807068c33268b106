"""Generate the committed golden fixtures from the REFERENCE utils/packet.py.

Runs only in the build container, where /root/reference exists; the GPU box
and the tests read the fixtures this writes, never the reference.  Imports the
reference module from its own path (nothing is copied) and records:

  edge_cases.json   scripted calls on the reference Packet (every edge case
                    of SURVEY.md §8a a2-a9) with their results / exceptions
  frames_small.npz  fixed-length batches framed by the reference, per payload
                    length and layout, plus reference-decoded fields of
                    full-range (0x00-0xFF) frames
  digests.json      SHA-256 digests of reference-framed full-size batches
                    (BASELINE configs C2-C5), per 2^20-packet chunk
  wire_trace.json   frames of the config-1 exchange (utils/reliableUDP.py
                    call pattern, message bin/input.txt, ISN 0x0e1b)

The rudp7 checksum field VALUE is build-defined (the reference has none): it
comes from oracle/codec_np.py and is only *framed* by the reference.

usage: python tests/golden/make_golden.py [--skip-digests] [--jobs 8]
       python tests/golden/make_golden.py --only-digests --configs C2,C3
         (recomputes those configs' digests, every layout, and merges them into
         the existing digests.json; the other configs' entries are kept)
"""
from __future__ import annotations

import argparse
import hashlib
import importlib.util
import json
import os
import sys
import time
from multiprocessing import Pool
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
REF_PACKET = Path("/root/reference/utils/packet.py")

from oracle import codec_np, synth  # noqa: E402

# BASELINE.json configs; seeds fixed per config index.
CONFIGS = {
    "C2": dict(seed=0x5EED0002, n=1 << 20, L=1024, layouts=(5, 7)),
    "C3": dict(seed=0x5EED0003, n=1 << 20, L=64, layouts=(5, 7)),
    "C4": dict(seed=0x5EED0004, n=1 << 20, L=1472, layouts=(5, 7)),
    "C5": dict(seed=0x5EED0005, n=1 << 24, L=1472, layouts=(5, 7)),
}
DIGEST_CHUNK = 1 << 20
SMALL_LENGTHS = (0, 1, 2, 3, 15, 16, 17, 31, 48, 64, 100, 1024, 1472)
SMALL_SEED = 0x5EED1000


def load_reference():
    spec = importlib.util.spec_from_file_location("reference_packet", REF_PACKET)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


REF = None


def ref():
    global REF
    if REF is None:
        REF = load_reference()
    return REF


def rudp7_definition(mod):
    return {**mod.custom_header, "checksum": 2}


# ------------------------------------------------------------- framing by ref
def ref_encode(mod, seq, ack, flags, payload: bytes, layout: int, csum: int) -> bytes:
    """One frame through the reference API, call pattern of utils/reliableUDP.py:53-61."""
    p = mod.Packet(header_definition=rudp7_definition(mod)) if layout == 7 else mod.Packet()
    p.set_header_field("seq_num", str(int(seq)), base=10)
    p.set_header_field("ack_num", str(int(ack)), base=10)
    if flags & 0x80:
        p.set_header_field("syn", "1", base=2)
    if flags & 0x40:
        p.set_header_field("ack", "1", base=2)
    if flags & 0x20:
        p.set_header_field("fin", "1", base=2)
    if flags & 0x1F:
        p.set_header_field("offset", format(flags & 0x1F, "b"), base=2)
    if layout == 7:
        p.set_header_field("checksum", format(int(csum), "x"), base=16)
    p.set_payload(payload.decode("ascii"))
    return p.to_byte()


def ref_decode_fields(mod, frame: bytes, layout: int):
    p = mod.Packet(frame, header_definition=rudp7_definition(mod)) if layout == 7 else mod.Packet(frame)
    seq = int(p.get_header_field("seq_num", base=10))
    ack = int(p.get_header_field("ack_num", base=10))
    flags = (int(p.get_header_field("syn", base=2), 2) << 7 | int(p.get_header_field("ack", base=2), 2) << 6
             | int(p.get_header_field("fin", base=2), 2) << 5 | int(p.get_header_field("offset", base=2), 2))
    cs = int(p.get_header_field("checksum", base=16), 16) if layout == 7 else -1
    return seq, ack, flags, cs, p.get_hex()


def ref_encode_batch(seq, ack, flags, payload, layout, csum) -> np.ndarray:
    mod = ref()
    n, L = payload.shape
    out = bytearray()
    for i in range(n):
        out += ref_encode(mod, seq[i], ack[i], flags[i], payload[i].tobytes(), layout, csum[i])
    return np.frombuffer(bytes(out), dtype=np.uint8).reshape(n, L + layout)


# ---------------------------------------------------------------- edge cases
sys.path.insert(0, str(HERE.parent))
from tests_support import run_script  # noqa: E402

EDGE_SCRIPTS = [
    ("default_header", [["new", None, "ref"], ["to_byte"], ["get_hex"], ["binary"], ["hlb"],
                        ["get_payload"], ["get", "seq_num", 16], ["get", "syn", 2]]),
    ("fields_syn_fin", [["new", None, "ref"], ["set", "seq_num", "1234", 16],
                        ["set", "ack_num", "abcd", 16], ["set", "syn", "1", 2], ["set", "fin", "1", 2],
                        ["to_byte"], ["get", "seq_num", 10], ["get", "ack_num", 16],
                        ["get", "syn", 2], ["get", "ack", 2], ["get", "fin", 10], ["get", "offset", 2]]),
    ("wrap_mod_2_16", [["new", None, "ref"], ["set", "seq_num", "70000", 10], ["get", "seq_num", 10],
                       ["set", "ack_num", "ffff1", 16], ["get", "ack_num", 16], ["to_byte"]]),
    ("flag_low_bit", [["new", None, "ref"], ["set", "syn", "101", 2], ["get", "syn", 2],
                      ["set", "offset", "11111111", 2], ["get", "offset", 10], ["to_byte"]]),
    ("hex_prefix", [["new", None, "ref"], ["set", "seq_num", "0x1f", 16], ["get", "seq_num", 10]]),
    ("int_value_base10", [["new", None, "ref"], ["set", "seq_num", 513, 10], ["get", "seq_num", 16]]),
    ("negative_corrupts", [["new", None, "ref"], ["set", "seq_num", "-5", 10], ["binary"],
                           ["get", "ack_num", 10], ["get", "seq_num", 2], ["get", "seq_num", 10],
                           ["get_hex"], ["to_byte"], ["set_payload", "hi"], ["get_payload"],
                           ["set", "seq_num", "7", 10], ["get_hex"], ["to_byte"]]),
    ("negative_hex", [["new", None, "ref"], ["set", "ack_num", "-a", 16], ["get", "ack_num", 2],
                      ["eq_hex", "0000000000"]]),
    ("non_binary_base2", [["new", None, "ref"], ["set", "fin", "x", 2], ["get", "fin", 2],
                          ["get_hex"]]),
    ("short_frame", [["new", "010203", "ref"], ["get", "seq_num", 10], ["get", "ack_num", 10],
                     ["get", "ack_num", 2], ["get", "syn", 2], ["get", "syn", 10], ["get", "fin", 16],
                     ["get_payload"], ["get_hex"], ["to_byte"]]),
    ("short_frame_set", [["new", "0102", "ref"], ["set", "fin", "1", 2], ["binary"], ["get_hex"],
                         ["set_payload", "Z"], ["get_hex"], ["get_payload"]]),
    ("one_byte_frame", [["new", "ff", "ref"], ["get", "seq_num", 10], ["get", "seq_num", 16],
                        ["set", "ack_num", "3", 10], ["get_hex"]]),
    ("empty_bytes", [["new", "", "ref"], ["to_byte"], ["get_payload"]]),
    ("payload_roundtrip", [["new", None, "ref"], ["set", "seq_num", "3611", 10],
                           ["set_payload", "t"], ["to_byte"], ["get_payload"], ["get", "seq_num", 10]]),
    ("payload_empty_noop", [["new", None, "ref"], ["set_payload", "abc"], ["set_payload", ""],
                            ["get_payload"], ["to_byte"]]),
    ("payload_replace", [["new", None, "ref"], ["set_payload", "abcdef"], ["set_payload", "xy"],
                         ["get_payload"], ["to_byte"], ["set", "seq_num", "1", 10], ["to_byte"]]),
    ("payload_leading_nul", [["new", "0001000200" + "0000" + "41", "ref"], ["get_payload"],
                             ["get_hex"], ["to_byte"]]),
    ("payload_utf8", [["new", None, "ref"], ["set_payload", "é€"], ["to_byte"],
                      ["get_payload"]]),
    ("payload_bad_utf8", [["new", "00010000" + "40" + "ff", "ref"], ["get", "ack", 2],
                          ["get_payload"], ["get_hex"]]),
    ("parse_header_only", [["new", "0e1b000080", "ref"], ["get_payload"], ["get", "syn", 2]]),
    ("parse_trace_frame", [["new", "0e200000200a", "ref"], ["get", "seq_num", 10],
                           ["get", "fin", 2], ["get_payload"], ["eq_hex", "0e200000200a"],
                           ["eq_hex", "0e200000200b"], ["eq_other", "0e200000200a"]]),
    ("unknown_field", [["new", None, "ref"], ["get", "nope", 16], ["set", "nope", "1", 16],
                       ["pos", "nope"], ["pos", "fin"]]),
    ("unsupported_base", [["new", None, "ref"], ["get", "seq_num", 8], ["set", "seq_num", "1", 8],
                          ["get", "seq_num", 2]]),
    ("non_byte_aligned", [["new", None, "one_bit"], ["hlb"], ["set_payload", "A"], ["get_hex"],
                          ["to_byte"], ["binary"], ["get", "a", 2]]),
    ("non_byte_aligned_parse", [["new", "c1", "one_bit"], ["get", "a", 10], ["get_payload"]]),
    ("zero_width_field", [["new", None, "zero_width"], ["hlb"], ["set", "z", "101", 2], ["binary"],
                          ["get_hex"], ["get", "ack_num", 10]]),
    ("rudp7_checksum_field", [["new", None, "rudp7"], ["hlb"], ["set", "seq_num", "1", 10],
                              ["set", "checksum", "beef", 16], ["set_payload", "ab"], ["to_byte"],
                              ["get", "checksum", 16], ["get_payload"]]),
    ("rudp7_parse", [["new", "0001000000beef6162", "rudp7"], ["get", "checksum", 10],
                     ["get", "seq_num", 10], ["get_payload"]]),
]


def make_edge_cases(mod):
    cases = []
    for name, steps in EDGE_SCRIPTS:
        res = run_script(mod.Packet, mod.custom_header, steps)
        cases.append({"name": name, "steps": steps, "results": res})
    return cases


# --------------------------------------------------------------- small frames
def make_small(mod):
    arrays = {}
    for L in SMALL_LENGTHS:
        n = 64 if L <= 100 else 24
        seq, ack, flags, pay = synth.synth(SMALL_SEED + L, 0, n, L, ascii=True)
        # make every flag/offset combination appear on top of the synthetic mix
        flags = flags.copy()
        flags[:8] = np.array([0x00, 0x80, 0x40, 0x20, 0xE0, 0xA0, 0x60, 0x1F], np.uint8)
        _, csum = codec_np.encode(seq, ack, flags, pay, 5)
        f5 = ref_encode_batch(seq, ack, flags, pay, 5, csum)
        f7 = ref_encode_batch(seq, ack, flags, pay, 7, csum)
        arrays.update({f"L{L}_seq": seq, f"L{L}_ack": ack, f"L{L}_flags": flags,
                       f"L{L}_payload": pay, f"L{L}_frames5": f5, f"L{L}_frames7": f7,
                       f"L{L}_csum": csum})
        # full-range payloads: framed by numpy, fields decoded by the reference
        sq, ak, fl, pb = synth.synth(SMALL_SEED + 0x800 + L, 0, n, L, ascii=False)
        for layout in (5, 7):
            fr, _ = codec_np.encode(sq, ak, fl, pb, layout)
            dec = np.array([ref_decode_fields(mod, fr[i].tobytes(), layout)[:4] for i in range(n)],
                           dtype=np.int64).reshape(n, 4)
            hexes = [ref_decode_fields(mod, fr[i].tobytes(), layout)[4] for i in range(n)]
            assert all(h == fr[i].tobytes().hex() for i, h in enumerate(hexes))
            arrays[f"L{L}_full_frames{layout}"] = fr
            arrays[f"L{L}_full_fields{layout}"] = dec
    return arrays


# ------------------------------------------------------------ varlen batches
UTF8_CASES = [
    b"", b"a", b"\x00", b"\x7f", b"\xc2\x80", b"\xdf\xbf", b"\xe0\xa0\x80", b"\xef\xbf\xbf",
    b"\xf0\x90\x80\x80", b"\xf4\x8f\xbf\xbf", b"\xf0\x9f\x98\x80", b"\xed\x9f\xbf",
    b"\x80", b"\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xc2", b"\xe0\x80\x80", b"\xe0\x9f\xbf",
    b"\xed\xa0\x80", b"\xed\xbf\xbf", b"\xe2\x82", b"\xf0\x80\x80\x80", b"\xf0\x8f\xbf\xbf",
    b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xff", b"\xfe", b"a\xc3\xa9b", b"a\xc3b",
    b"\xe2\x82\xac\xe2\x82", b"\xf0\x9f\x98", b"\xc3\xa9\xc3\xa9\xc3\xa9\xc3",
]


def make_varlen(mod):
    import random
    rng = random.Random(0x5EED2000)
    alphabet = "abcxyz019 \n\t~" + "éßñ" + "€中文字" + "😀🚀" + "\u0000\u007f\u0080\u07ff\u0800\uffff"
    texts = [""] + ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 40))) for _ in range(399)]
    pays = [t.encode() for t in texts]
    n = len(pays)
    seq, ack, flags, _ = synth.synth(0x5EED3000, 0, n, 0)
    fr5, off5, cs = codec_np.encode_varlen(seq, ack, flags, pays, 5)
    ref5, ref7 = bytearray(), bytearray()
    for i, t in enumerate(texts):
        for layout, buf in ((5, ref5), (7, ref7)):
            p = mod.Packet(header_definition=rudp7_definition(mod)) if layout == 7 else mod.Packet()
            p.set_header_field("seq_num", str(int(seq[i])), base=10)
            p.set_header_field("ack_num", str(int(ack[i])), base=10)
            for bit, name in ((0x80, "syn"), (0x40, "ack"), (0x20, "fin")):
                if flags[i] & bit:
                    p.set_header_field(name, "1", base=2)
            if layout == 7:
                p.set_header_field("checksum", format(int(cs[i]), "x"), base=16)
            p.set_payload(t)
            buf += p.to_byte()
    # payload validity exactly as the reference's get_payload reports it
    rnd = [bytes(rng.randrange(256) for _ in range(rng.randint(0, 12))) for _ in range(300)]
    cases = UTF8_CASES + rnd
    valid = []
    for body in cases:
        q = mod.Packet(b"\x00\x01\x00\x02\x40" + body)
        try:
            q.get_payload()
            valid.append(1)
        except UnicodeDecodeError:
            valid.append(0)
    return {
        "seq": seq, "ack": ack, "flags": flags,
        "payload": np.frombuffer(b"".join(pays), np.uint8),
        "lengths": np.array([len(p) for p in pays], np.int32),
        "frames5": np.frombuffer(bytes(ref5), np.uint8), "frames7": np.frombuffer(bytes(ref7), np.uint8),
        "csum": cs,
        "utf8_bodies": np.frombuffer(b"".join(cases), np.uint8),
        "utf8_lengths": np.array([len(c) for c in cases], np.int32),
        "utf8_valid": np.array(valid, np.uint8),
    }


# ------------------------------------------------------- proxy retransmission
def make_dedup(mod):
    """Datagram sequence with retransmissions; dup flags from the reference
    Packet.__eq__ under the proxy's list logic (proxy.py:90-94, window 500)."""
    import random
    rng = random.Random(0x5EED4000)
    pool = [b"", b"\x00" * 5, b"\x00" * 4, b"\x00" * 6, b"\x01", b"\x00\x01",
            bytes.fromhex("0e1b00008074"), bytes.fromhex("0e1c00000065"), bytes.fromhex("00000e1c40")]
    pool += [bytes(rng.randrange(256) for _ in range(rng.randint(1, 30))) for _ in range(150)]
    seq = []
    for _ in range(3000):
        r = rng.random()
        if r < 0.3 and seq:        # retransmit something recent (inside or just outside the window)
            seq.append(seq[-rng.randint(1, min(len(seq), 700))])
        elif r < 0.4:              # the edge cases: empty vs zero header, short frames
            seq.append(rng.choice(pool[:9]))
        else:                      # a fresh datagram
            seq.append(bytes(rng.randrange(256) for _ in range(rng.randint(1, 30))))
    history, dup = [], []
    for data in seq:
        pkt = mod.Packet(data)
        dup.append(1 if pkt in history else 0)
        history.append(pkt)
        if len(history) > 500:
            history.pop(0)
    return {"frames": np.frombuffer(b"".join(seq), np.uint8),
            "lengths": np.array([len(d) for d in seq], np.int32),
            "dup": np.array(dup, np.uint8)}


# -------------------------------------------------------------------- digests
def _digest_task(args):
    cfg, layout, chunk_index = args
    c = CONFIGS[cfg]
    first = chunk_index * DIGEST_CHUNK
    n = min(DIGEST_CHUNK, c["n"] - first)
    h_frames = hashlib.sha256()
    h_csum = hashlib.sha256()
    step = 1 << 15
    for a in range(0, n, step):
        m = min(step, n - a)
        seq, ack, flags, pay = synth.synth(c["seed"], first + a, m, c["L"], ascii=True)
        _, csum = codec_np.encode(seq, ack, flags, pay, 5)
        fr = ref_encode_batch(seq, ack, flags, pay, layout, csum)
        h_frames.update(fr.tobytes())
        h_csum.update(csum.astype("<u2").tobytes())
    return cfg, layout, chunk_index, h_frames.hexdigest(), h_csum.hexdigest()


def make_digests(jobs: int, configs=None):
    """Digests of the named configs (all of CONFIGS when None), every layout."""
    configs = list(CONFIGS) if configs is None else configs
    tasks = []
    for cfg in configs:
        c = CONFIGS[cfg]
        chunks = (c["n"] + DIGEST_CHUNK - 1) // DIGEST_CHUNK
        for layout in c["layouts"]:
            tasks += [(cfg, layout, k) for k in range(chunks)]
    out = {cfg: dict(seed=CONFIGS[cfg]["seed"], n=CONFIGS[cfg]["n"], L=CONFIGS[cfg]["L"],
                     chunk=DIGEST_CHUNK, layouts={}) for cfg in configs}
    t0 = time.time()
    with Pool(jobs) as pool:
        for i, (cfg, layout, k, hf, hc) in enumerate(pool.imap_unordered(_digest_task, tasks)):
            d = out[cfg]["layouts"].setdefault(str(layout), {"frames": {}, "csum": {}})
            d["frames"][str(k)] = hf
            d["csum"][str(k)] = hc
            print(f"  [{i + 1}/{len(tasks)}] {cfg} rudp{layout} chunk {k} ({time.time() - t0:.0f}s)",
                  flush=True)
    for cfg in out:
        for layout, d in out[cfg]["layouts"].items():
            for kind in ("frames", "csum"):
                parts = [d[kind][str(k)] for k in range(len(d[kind]))]
                d[kind] = parts
                d[kind + "_all"] = hashlib.sha256("".join(parts).encode()).hexdigest()
    return out


# ----------------------------------------------------------------- wire trace
def make_wire_trace(mod):
    """Frames of config 1 (client -> server, message bin/input.txt, ISN 0x0e1b).

    Built with the reference Packet in the exact call order of
    utils/reliableUDP.py (send_data :53-61, server send_ack :142-146,
    send_fin :156-161, client final send_ack :88-92); matches the trace
    captured on a live run.
    """
    message = Path("/root/reference/bin/input.txt").read_text()
    isn = 0x0E1B
    c2s, s2c = [], []
    for ptr in range(len(message)):
        p = mod.Packet()
        p.set_header_field("seq_num", str(ptr + isn), base=10)
        p.set_header_field("ack_num", "0", base=10)
        if ptr == 0:
            p.set_header_field("syn", "1", base=2)
        if ptr + 1 == len(message):
            p.set_header_field("fin", "1", base=2)
        p.set_payload(message[ptr:ptr + 1])
        c2s.append(p.to_byte().hex())
        a = mod.Packet()
        a.set_header_field("ack", "1", base=2)
        a.set_header_field("seq_num", "0", base=10)
        a.set_header_field("ack_num", str(isn + ptr + 1), base=10)
        s2c.append(a.to_byte().hex())
    f = mod.Packet()
    f.set_header_field("fin", "1", base=2)
    f.set_header_field("ack", "1", base=2)
    f.set_header_field("seq_num", "0", base=10)
    f.set_header_field("ack_num", str(isn + len(message)), base=10)
    s2c.append(f.to_byte().hex())
    last = mod.Packet()
    last.set_header_field("seq_num", str(isn + len(message)), base=10)
    last.set_header_field("ack_num", str(0 + 1), base=10)
    last.set_header_field("ack", "1", base=2)
    c2s.append(last.to_byte().hex())
    return {"message": message, "isn": isn, "client_to_server": c2s, "server_to_client": s2c}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-digests", action="store_true")
    ap.add_argument("--only-digests", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--configs", default="", help="comma-separated subset of CONFIGS to (re)digest and merge")
    args = ap.parse_args()
    mod = ref()
    if not args.only_digests:
        (HERE / "edge_cases.json").write_text(json.dumps(make_edge_cases(mod), indent=1) + "\n")
        np.savez_compressed(HERE / "frames_small.npz", **make_small(mod))
        (HERE / "wire_trace.json").write_text(json.dumps(make_wire_trace(mod), indent=1) + "\n")
        np.savez_compressed(HERE / "varlen.npz", **make_varlen(mod))
        np.savez_compressed(HERE / "dedup.npz", **make_dedup(mod))
        print("wrote edge_cases.json, frames_small.npz, wire_trace.json, varlen.npz, dedup.npz")
    if not args.skip_digests:
        path = HERE / "digests.json"
        if args.configs:
            sel = [c for c in args.configs.split(",") if c]
            old = json.loads(path.read_text()) if path.exists() else {}
            new = make_digests(args.jobs, sel)
            for cfg in sel:  # a layout digested before must come out the same again
                for layout, d in old.get(cfg, {}).get("layouts", {}).items():
                    if layout in new[cfg]["layouts"] and new[cfg]["layouts"][layout] != d:
                        raise SystemExit(f"{cfg} rudp{layout}: recomputed digests differ from the committed ones")
            old.update(new)
            digests = {cfg: old[cfg] for cfg in CONFIGS if cfg in old}
        else:
            digests = make_digests(args.jobs)
        path.write_text(json.dumps(digests, indent=1) + "\n")
        print("wrote digests.json")


if __name__ == "__main__":
    main()
