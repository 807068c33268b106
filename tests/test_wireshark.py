"""The reconciled Wireshark dissector agrees with the codec.

tools/wireshark/rudp.lua is generated from rudp.packet.custom_header; these
checks keep the committed copy current and pin its field masks and offsets to
the constants the kernels pack (utils/packet.py:3-10: 5-bit offset, no RST;
the reference's wireshark.lua:11-12 used RST 0x10 and offset 0x0F).
No Lua interpreter exists in this image, so the dissector itself is not run.
"""
import re
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tools" / "wireshark"))

import gen_dissector  # noqa: E402
from oracle import codec_np  # noqa: E402
from rudp import batch  # noqa: E402


def test_committed_dissector_is_current():
    assert (REPO / "tools/wireshark/rudp.lua").read_text() == gen_dissector.render()


def test_field_table_matches_codec():
    from rudp.packet import custom_header
    fields, h = gen_dissector.field_table({**custom_header, "checksum": 2})
    assert h == batch.layout_header_len("rudp7")
    t = {name: (off, n, mask) for name, off, n, mask in fields}
    assert t["seq_num"] == (0, 2, None) and t["ack_num"] == (2, 2, None)
    assert t["syn"] == (4, 1, batch.SYN) and t["ack"] == (4, 1, batch.ACK)
    assert t["fin"] == (4, 1, batch.FIN) and t["offset"] == (4, 1, batch.OFFSET_MASK)
    assert t["checksum"] == (5, 2, None)
    _, h5 = gen_dissector.field_table(custom_header)
    assert h5 == batch.layout_header_len("rudp5")


def test_lua_masks_and_no_rst():
    text = (REPO / "tools/wireshark/rudp.lua").read_text()
    masks = dict(re.findall(r'"rudp\.flags\.(\w+)".*?0x([0-9A-F]{2})\)', text))
    assert masks == {"syn": "80", "ack": "40", "fin": "20", "offset": "1F"}
    assert "rudp.flags.rst" not in text and "0x0F" not in text


def test_checksum_status_matches_oracle(golden_small):
    """The Lua's 'Good' test is inet_checksum(frame, field zeroed) == field; the
    golden rudp7 frames satisfy it and a flipped byte breaks it (oracle restatement)."""
    key = next(k for k in golden_small if k.endswith("_frames7") and "full" not in k)
    fr = golden_small[key].copy()
    stored = fr[:, 5].astype(np.uint16) << 8 | fr[:, 6]
    assert np.array_equal(codec_np.frame_checksums(fr, 7), stored)
    fr[0, 2] ^= 1  # a header byte outside the checksum field
    assert codec_np.frame_checksums(fr, 7)[0] != stored[0]
