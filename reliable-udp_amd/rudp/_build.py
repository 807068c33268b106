"""Compile librudp.so (the HIP kernels + C ABI) for gfx950, in-tree.

hipcc cross-compiles without a GPU, so this runs in the build container and
the resulting ``rudp/librudp.so`` travels with the repo snapshot to the GPU
box.  Objects go to ``reliable-udp_amd/build/``; a source is rebuilt only when
it or a header is newer than its object.
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


def build(force: bool = False, verbose: bool = False) -> Path:
    """Build (if stale) and return the path of librudp.so."""
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr_time = _newest_header()
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-mcode-object-version=5", f"-I{INCLUDE}"]

    def compile_one(src: str) -> Path:
        s = CSRC / src
        o = BUILD / (Path(src).stem + ".o")
        if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_time):
            if s.suffix == ".cpp":  # host-only C++ (no HIP): plain g++
                cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-Wall",
                       f"-I{INCLUDE}", "-c", str(s), "-o", str(o)]
            else:
                cmd = [hipcc, *flags, "-c", str(s), "-o", str(o)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    if force or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
               "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of librudp.so failed:\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
