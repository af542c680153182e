"""Build liblsmblk.so (HIP kernels for gfx950 + the per-entry host half) in-tree.

Two libraries from the same sources:
  * liblsmblk.so       the product (-DLSMBLK_DIAG_BUILD=0): ablation masks compiled out;
  * liblsmblk_diag.so  diagnostics (-DLSMBLK_DIAG_BUILD=1): the kernels honour the timing-only
                       ablation masks of LSMBLK_DEBUG_DECODE_SKIP (bench.py --ablate loads it).
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SO = os.path.join(PKG, "liblsmblk.so")
DIAG_SO = os.path.join(PKG, "liblsmblk_diag.so")
SOURCES = [os.path.join(PKG, "csrc", f) for f in ("lsmblk_gpu.hip", "lsmblk_compact.hip", "lsmblk_sst.hip", "lsmblk_host.cpp")]
HEADERS = [os.path.join(ROOT, "include", "lsmblk.h"), os.path.join(PKG, "csrc", "lsmblk_dev.hpp")]


def src_sha():
    """sha256 of the kernel sources and the ABI header (profiles/traffic.json is stamped with it)."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(SOURCES + HEADERS):
        h.update(os.path.basename(p).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()


def needs_build(so=SO):
    if not os.path.exists(so):
        return True
    t = os.path.getmtime(so)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def _cmd(so, diag):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    return [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-Wall", "-Wshadow", "-Wno-unused-function", f"-DLSMBLK_DIAG_BUILD={1 if diag else 0}",
            "-I" + os.path.join(ROOT, "include"), *SOURCES, "-o", so + ".tmp"]


def build(force=False, verbose=False, diag=True):
    """Compile the product library (and the diagnostics one) when a source is newer; the two
    compiles run side by side."""
    jobs = [(so, d) for so, d in ((SO, False), (DIAG_SO, True)) if (d is False or diag) and (force or needs_build(so))]
    procs = []
    for so, d in jobs:
        cmd = _cmd(so, d)
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((so, subprocess.Popen(cmd)))
    failed = [so for so, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc -> {failed}")
    for so, _ in procs:
        os.replace(so + ".tmp", so)
    return SO


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(SO)
