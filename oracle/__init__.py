"""ORACLE — test infrastructure only, never the product.

CPU restatements of the reference's hot path (reotam5/Reliable-UDP
utils/packet.py, as called from utils/reliableUDP.py), used as the checker for
the HIP kernels in reliable-udp_amd/.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import anything from here.

  bitstring_packet.py  the reference's bit-string Packet algorithm restated
                       (timed as bench.py's cpu_baseline, kind "port")
  codec_np.py          numpy batch frame/checksum/parse/verify
  synth.py             numpy restatement of the device synthetic generator
  codec_ref.c          plain-C batch restatement (full-size diffs)

Parity pinning: framing/decode are pinned to golden vectors and SHA-256
digests produced by the reference utils/packet.py itself in the build
container (tests/golden/make_golden.py).  The checksum VALUE is build-defined
(the reference has none) and is pinned only by the RFC 1071 known answer
(00 01 f2 03 f4 f5 f6 f7 -> 0x220d) — "parity unpinned" against the
reference for that field.
"""
