"""Compile librudp.so (the HIP kernels + C ABI) for gfx950, in-tree.

hipcc cross-compiles without a GPU, so this runs in the build container and
the resulting ``rudp/librudp.so`` travels with the repo snapshot to the GPU
box.  Objects go to ``reliable-udp_amd/build/``; a source is rebuilt only when
it or a header is newer than its object.

The same sources also build ``rudp/librudp_tools.so`` with RUDP_TOOLS=1
(objects in ``build/tools/``): the diagnostics build tools/ and the tests of
the non-default kernel forms load (``_native.tools_lib()``), with the
rudpx_* sweep knobs, tile timelines and copy ceilings.  The product library
has none of them.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent                      # reliable-udp_amd/
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
BUILD = ROOT / "build"
LIB = PKG_DIR / "librudp.so"
TOOLS_LIB = PKG_DIR / "librudp_tools.so"
SOURCES = ("encode.hip", "decode.hip", "synth.hip", "varlen.hip", "dedup.hip", "bounds.hip", "scan.hip", "device_pool.hip", "capi.hip",
           "tuning.hip", "netio.cpp")
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: librudp.so cannot be built")


def _newest_header() -> float:
    hdrs = list(CSRC.glob("*.hpp")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hdrs), default=0.0)


def _build_one(lib: Path, objdir: Path, defines, force: bool, verbose: bool, hipcc: str, hdr_time: float,
               pool: ThreadPoolExecutor):
    objdir.mkdir(parents=True, exist_ok=True)
    # host code hidden by default: only the RUDP_API entry points leave the .so, so the
    # product and diagnostics builds (same C++ names, different struct layouts) can
    # never interpose on each other, even under RTLD_GLOBAL or a profiler's preload
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-mcode-object-version=5", "-Xarch_host", "-fvisibility=hidden", f"-I{INCLUDE}", *defines]

    def compile_one(src: str) -> Path:
        s = CSRC / src
        o = objdir / (Path(src).stem + ".o")
        if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_time):
            if s.suffix == ".cpp":  # host-only C++ (no HIP): plain g++
                cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-fvisibility=hidden",
                       f"-I{INCLUDE}", *defines, "-c", str(s), "-o", str(o)]
            else:
                cmd = [hipcc, *flags, "-c", str(s), "-o", str(o)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
        return o

    futs = [pool.submit(compile_one, src) for src in SOURCES]

    def link() -> Path:
        objs = [f.result() for f in futs]
        if force or not lib.exists() or lib.stat().st_mtime < max(o.stat().st_mtime for o in objs):
            cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link of {lib.name} failed:\n{r.stderr}")
        return lib
    return link


def build(force: bool = False, verbose: bool = False, tools: bool = True) -> Path:
    """Build (if stale) and return the path of librudp.so; with ``tools`` also
    the diagnostics build librudp_tools.so."""
    hipcc = _hipcc()
    hdr_time = _newest_header()
    jobs = max(1, min(2 * len(SOURCES), os.cpu_count() or 1))
    with ThreadPoolExecutor(max_workers=jobs) as pool:
        links = [_build_one(LIB, BUILD, [], force, verbose, hipcc, hdr_time, pool)]
        if tools:
            links.append(_build_one(TOOLS_LIB, BUILD / "tools", ["-DRUDP_TOOLS=1"], force, verbose, hipcc,
                                    hdr_time, pool))
        for link in links:
            link()
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, tools="--no-tools" not in sys.argv))
