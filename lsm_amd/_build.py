"""Build liblsmblk.so (HIP kernels for gfx950 + the per-entry host half) in-tree."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SO = os.path.join(PKG, "liblsmblk.so")
SOURCES = [os.path.join(PKG, "csrc", f) for f in ("lsmblk_gpu.hip", "lsmblk_compact.hip", "lsmblk_sst.hip", "lsmblk_host.cpp")]
HEADERS = [os.path.join(ROOT, "include", "lsmblk.h"), os.path.join(PKG, "csrc", "lsmblk_dev.hpp")]


def needs_build():
    if not os.path.exists(SO):
        return True
    t = os.path.getmtime(SO)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return SO
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function",
           "-I" + os.path.join(ROOT, "include"), *SOURCES, "-o", SO + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(SO + ".tmp", SO)
    return SO


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(SO)
