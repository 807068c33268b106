"""The C ABI library loads and exports what include/rudp.h declares.

CPU-only: no compute call reaches a device here; only the argument checks
that run before any HIP call are exercised.
"""
import ctypes
import re

import numpy as np
import pytest

from conftest import REPO
from rudp import _native
from rudp import batch


def declared_functions():
    text = (REPO / "include" / "rudp.h").read_text()
    return set(re.findall(r"^RUDP_API\s+(?:int|const char\*)\s+(rudp_\w+)\s*\(", text, flags=re.M))


def test_header_and_binding_agree():
    assert declared_functions() == set(_native.EXPORTS)


def _dynamic_symbols(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True, text=True, check=True)
    return {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}


def test_library_exports_every_declared_symbol():
    lib = _native.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.rudp_abi_version() == _native.ABI_VERSION


def test_product_library_exports_only_the_abi():
    """librudp.so carries the include/rudp.h ABI and nothing of the diagnostics
    (no rudpx_* knobs, timelines or copy kernels); librudp_tools.so adds them."""
    prod = {s for s in _dynamic_symbols(_native.LIB_PATH) if s.startswith(("rudp", "rudpx"))}
    assert prod == declared_functions()
    tools = {s for s in _dynamic_symbols(_native.TOOLS_LIB_PATH) if s.startswith("rudpx_")}
    assert {"rudpx_tune", "rudpx_encode_trace", "rudpx_stamp", "rudpx_copy_vpt"} <= tools


def test_internals_stay_inside_each_library():
    """Both builds hide everything but their entry points; what the HIP runtime
    needs exported (kernel handles) lives in a namespace per build (rudp::,
    rudp_tools::), so the product and diagnostics libraries in one process can
    never bind to each other's kernels or functions (their argument structs
    differ), whatever the load flags."""
    prod = _dynamic_symbols(_native.LIB_PATH)
    tools = _dynamic_symbols(_native.TOOLS_LIB_PATH)
    assert not any("rudp_tools" in s for s in prod)
    assert not any(s.startswith("_ZN4rudp") and not s.startswith("_ZN10rudp_tools") for s in tools)
    internal = {s for s in prod if s.startswith("_ZN4rudp")}
    assert not (internal & tools)
    # functions: the entry points only (no internal C++ function of librudp is exported)
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    funcs = {ln.split()[-1] for ln in out.splitlines() if ln.split()[1:2] == ["T"]}
    assert funcs == declared_functions()


def test_batch_struct_layout():
    # struct rudp_batch: u64, u32, u32, then 6 pointers
    assert ctypes.sizeof(_native.RudpBatch) == 8 + 4 + 4 + 6 * 8
    assert _native.RudpBatch.seq.offset == 16


def test_argument_errors_before_device():
    lib = _native.lib()
    assert lib.rudp_encode(None, None, None, 7, 0, None) == _native.EINVAL
    assert b"NULL" in lib.rudp_last_error()
    b = _native.RudpBatch(n=1, payload_len=4)
    assert lib.rudp_encode(ctypes.byref(b), None, None, 6, 0, None) == _native.EINVAL
    assert b"layout" in lib.rudp_last_error()
    lens = (ctypes.c_uint32 * 1)(4)
    b.len = ctypes.cast(lens, ctypes.c_void_p)
    assert lib.rudp_encode(ctypes.byref(b), None, None, 7, 0, None) == _native.ENOTSUP
    assert lib.rudp_decode(None, None, 10, 1, None, None, None, None, None, None, None, 9, 0,
                           None) == _native.EINVAL
    off = (ctypes.c_uint64 * 1)(0)
    offp = ctypes.cast(off, ctypes.c_void_p)
    # variable-length decode is zero-copy: a payload_out buffer is refused
    assert lib.rudp_decode(None, offp, 10, 1, None, None, None, None, None, None, offp, 7, 0,
                           None) == _native.ENOTSUP
    assert lib.rudp_decode(None, offp, 10, 1, None, None, None, None, None, None, None, 7, 0,
                           None) == _native.EINVAL
    assert lib.rudp_encode_varlen(ctypes.byref(_native.RudpBatch(n=1)), None, None, None, 7, 0,
                                  None) == _native.EINVAL
    assert b"len" in lib.rudp_last_error()
    assert lib.rudp_validate_utf8(None, None, 10, 1, 7, None, 0, None) == _native.EINVAL
    out5 = (ctypes.c_int64 * 5)(9, 9, 9, 9, 9)
    assert lib.rudp_varlen_bounds(None, None, 0, out5, 0, None) == 0 and list(out5) == [0] * 5
    assert lib.rudp_varlen_bounds(None, None, 4, out5, 0, None) == _native.EINVAL
    assert lib.rudp_varlen_bounds(None, None, 4, None, 0, None) == _native.EINVAL
    assert lib.rudp_frame_off_bounds(None, 4, out5, 0, None) == _native.EINVAL
    # the sync-free varlen entries need their status word and offsets
    b1 = ctypes.byref(_native.RudpBatch(n=1))
    assert lib.rudp_encode_varlen_checked(b1, 0, None, 0, None, None, None, 7, 0, None) == _native.EINVAL
    assert b"d_status" in lib.rudp_last_error()
    assert lib.rudp_decode_varlen_checked(None, 0, None, 0, 1, None, None, None, None, None, None, None, 7, 0,
                                          None) == _native.EINVAL
    assert lib.rudp_frame_off_check(None, 1, 0, None, 0, None) == _native.EINVAL
    # empty batches are a successful no-op, no device needed
    assert lib.rudp_encode(ctypes.byref(_native.RudpBatch(n=0)), None, None, 5, 0, None) == 0
    assert lib.rudp_synth(1, 0, 0, 16, 1, None, None, None, None, 0, None) == 0


def test_error_mapping():
    with pytest.raises(ValueError, match="layout"):
        b = _native.RudpBatch(n=1, payload_len=4)
        _native.check(_native.lib().rudp_encode(ctypes.byref(b), None, None, 6, 0, None))


def test_python_api_validation():
    seq = np.zeros(3, np.uint16)
    with pytest.raises(ValueError, match="layout"):
        batch.pack_batch((seq, seq, np.zeros(3, np.uint8)), np.zeros((3, 4), np.uint8), "rudp6")
    with pytest.raises(TypeError, match="uint16"):
        batch.pack_batch((seq.astype(np.int32), seq, np.zeros(3, np.uint8)),
                         np.zeros((3, 4), np.uint8))
    with pytest.raises(ValueError, match="entries"):
        batch.pack_batch((seq[:2], seq, np.zeros(3, np.uint8)), np.zeros((3, 4), np.uint8))
    with pytest.raises(ValueError, match="in-band"):
        batch.unpack_batch(np.zeros((3, 20), np.uint8), "rudp7", csum=seq)
    assert batch.make_flags(syn=1, fin=1) == 0xA0
    assert batch.make_flags(ack=1, offset=0x3F) == 0x5F


def _code_object_kernels(path):
    """Kernel names of the gfx950 code objects in a library's offload bundles
    (one per translation unit in .hip_fatbin: __CLANG_OFFLOAD_BUNDLE__, entry
    count, then per entry offset / size / triple), read from each code
    object's symbol table by llvm-readelf: names ending in .kd are kernel
    descriptors."""
    import struct
    import subprocess
    import tempfile
    data = path.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, at = [], data.find(magic)
    while at >= 0:
        (count,) = struct.unpack_from("<Q", data, at + len(magic))
        pos = at + len(magic) + 8
        for _ in range(count):
            off, size, tlen = struct.unpack_from("<QQQ", data, pos)
            triple = data[pos + 24:pos + 24 + tlen].decode()
            pos += 24 + tlen
            if "gfx950" in triple and size:
                objs.append(data[at + off:at + off + size])
        at = data.find(magic, at + 1)
    assert objs, "no gfx950 code object"
    readelf = next((p for p in ("/opt/rocm/lib/llvm/bin/llvm-readelf", "/opt/rocm/llvm/bin/llvm-readelf")
                    if __import__("os").path.exists(p)), None)
    if readelf is None:
        pytest.skip("llvm-readelf not found")
    names = set()
    for co in objs:
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            out = subprocess.run([readelf, "--syms", "--wide", f.name], capture_output=True, text=True,
                                 check=True).stdout
        names |= {ln.split()[-1][:-3] for ln in out.splitlines() if ln.split() and ln.split()[-1].endswith(".kd")}
    return names


def test_product_code_object_ships_only_measured_forms():
    """Kernel forms measured slower than the defaults live in the
    diagnostics build only: the byte-span decode (index pass and span kernel),
    the decode tile reading four chunks at a time (R4) and the two-wave
    (128-thread) decode tiles.  librudp.so's code object has none of them;
    librudp_tools.so keeps them for the A/B tools and their tests."""
    prod = _code_object_kernels(_native.LIB_PATH)
    assert any("decode_varlen_tile_kernel" in k for k in prod)
    losing = [k for k in prod if "decode_span_index_kernel" in k or "decode_varlen_span_kernel" in k
              or re.search(r"decode_varlen_tile_kernelILi[57]ELb[01]ELj(128ELb0|256ELb1)E", k)]
    assert not losing, losing
    # fixed-length batches that miss the fixed tiles take the varlen tiles with
    # implicit offsets (round 6): the one-wave-per-packet byte kernels are gone
    assert not [k for k in prod if "encode_bytes_kernel" in k or "decode_bytes_kernel" in k]
    assert any("copy_payloads_kernel" in k for k in prod)
    tools = _code_object_kernels(_native.TOOLS_LIB_PATH)
    assert any("decode_varlen_span_kernel" in k for k in tools)
    assert any(re.search(r"decode_varlen_tile_kernelILi7ELb0ELj128ELb0E", k) for k in tools)
