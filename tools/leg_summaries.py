"""Turn tools/gpu/profile_legs.sh's rocprofv3 output (gpurun_out/<prefix>_*) into
profiles/<round>/<leg>_summary.json + _kernel_stats.csv (tools/prof_summary.py),
one per timed bench leg, with the run's own HIP-event time per call beside
the trace's per-dispatch median.

usage: python tools/leg_summaries.py --prefix p4 --round r04 [--out gpurun_out] [leg ...]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent

# tag: (summary name, kernels (a call's chain), n, L, algorithmic bytes per unit)
LEGS = {
    "enc1472": ("encode_1Mx1472", "encode_tile_kernel", 1 << 20, 1472, 2956),
    "enc1024": ("encode_1Mx1024", "encode_tile_kernel", 1 << 20, 1024, 2060),
    "enc64": ("encode_1Mx64", "encode_tile_kernel", 1 << 20, 64, 140),
    "dec1472": ("decode_verify_1Mx1472", "decode_tile_kernel", 1 << 20, 1472, 1485),
    # parse + verify + strict UTF-8 in one pass: the valid flag is one more byte written
    "decu8_1472": ("decode_utf8_1Mx1472", "decode_tile_kernel", 1 << 20, 1472, 1486),
    # the same on valid multi-byte text (every chunk through the table check)
    "decu8text": ("decode_utf8_1Mx1472_multibyte_text", "decode_tile_kernel", 1 << 20, 1472, 1486),
    "enc16M": ("encode_16Mx1472", "encode_tile_kernel", 1 << 24, 1472, 2956),
    "venc1472": ("encode_varlen_1Mx1472", "scan_block_sums_kernel<8u>,scan_block_bases_kernel,scan_apply_kernel,"
                 "encode_varlen_tile_kernel", 1 << 20, 1472, 2968),
    "vdec1472": ("decode_varlen_1Mx1472", "decode_varlen_tile_kernel", 1 << 20, 1472, 1495),
    "vdecu8_1472": ("decode_varlen_utf8_1Mx1472", "decode_varlen_tile_kernel", 1 << 20, 1472, 1496),
    "vencrag": ("encode_varlen_ragged_0_2944", "scan_block_sums_kernel<8u>,scan_block_bases_kernel,"
                "scan_apply_kernel,encode_varlen_tile_kernel", 1 << 20, 1473, None),
    "vdecrag": ("decode_varlen_ragged_0_2944", "decode_varlen_tile_kernel", 1 << 20, 1473, None),
    "vdecu8rag": ("decode_varlen_utf8_ragged_0_2944", "decode_varlen_tile_kernel", 1 << 20, 1473, None),
    "utf8": ("utf8_validate_1Mx1472", "validate_utf8_tile_kernel", 1 << 20, 1472, 1480),
    "dedup": ("proxy_dedup_1M_window500", "dedup_small_kernel", 1 << 20, 1, 15),
    # (round 6: pass 1 also leaves 4-bit length codes, the framing kernel's mode 4; the setup's
    # fixed-length encode of the same payloads is mode 3 and stays out of the sums)
    "venc1c": ("encode_varlen_small_1Mx1char", "scan_block_sums_kernel<4u>|encode_varlen_small_kernel<5, 4u, 4>",
               1 << 20, 1, 26),
    # fixed-length batches off the 16-B grid (round 6): the varlen tiles with implicit offsets.
    # encode 2L + 10 (run_kernel frames rudp5 without the sideband checksum: read L + 5, write L + 5);
    # rudp7 2L + 12; decode + UTF-8 read F = 6,
    # write seq/ack/flags/ok/csum/valid 9
    "senc1c": ("encode_fixed_1Mx1char", "encode_varlen_small_kernel<5, 4u, 3>|", 1 << 20, 1, 12),
    "sdecu8_1c": ("decode_utf8_fixed_1Mx1char", "decode_varlen_small_kernel<5, 4u, true, true>|", 1 << 20, 1, 15),
    "senc1000": ("encode_fixed_1Mx1000", "encode_varlen_tile_kernel", 1 << 20, 1000, 2012),
    "vdec1c": ("decode_varlen_small_1Mx1char", "decode_varlen_small_kernel", 1 << 20, 1, 24),
    "vdecu8_1c": ("decode_varlen_utf8_small_1Mx1char", "decode_varlen_small_kernel", 1 << 20, 1, 25),
}


def event_ms(log: Path):
    for line in reversed(log.read_text().splitlines()):
        if line.startswith("{") and "ms_per_launch" in line:
            d = json.loads(line)
            return d["ms_per_launch"], d.get("payload_bytes")
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", type=Path, default=REPO / "gpurun_out")
    ap.add_argument("--prefix", required=True)
    ap.add_argument("--round", required=True)
    ap.add_argument("legs", nargs="*")
    args = ap.parse_args()
    for tag, (name, kernels, n, L, per_unit) in LEGS.items():
        if args.legs and tag not in args.legs:
            continue
        P = args.prefix
        kt = args.out / f"{P}_{tag}_kt"
        if not kt.exists():
            print(f"skip {tag}: no {kt}", file=sys.stderr)
            continue
        ms, pay = event_ms(args.out / f"{P}_{tag}_kt.log")
        if per_unit is None:  # ragged (mean 1473.1 B): as the equal-length legs, per the run's payload bytes
            # encode: read L + len 4 + table 5, write L + 7 + frame_off 8; decode: read L + 7 + frame_off 8,
            # write seq/ack/flags/ok/csum 8
            per_unit = 2 * pay / n + 24 if tag.startswith("venc") else pay / n + (24 if "u8" in tag else 23)
        cmd = [sys.executable, str(REPO / "tools/prof_summary.py"), "--round", args.round, "--tag", name,
               "--kt", str(kt), "--fetch", str(args.out / f"{P}_{tag}_fetch"),
               "--write", str(args.out / f"{P}_{tag}_write"), "--kernel", kernels, "--n", str(n), "--L", str(L),
               "--alg-bytes-per-unit", str(per_unit)]
        if ms is not None:
            cmd += ["--event-ms", str(ms)]
        if tag == "enc1472":
            cmd += ["--pmc-out", str(REPO / "profiles/pmc_encode.json")]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
        print(tag, name, "ok", file=sys.stderr)


if __name__ == "__main__":
    main()
