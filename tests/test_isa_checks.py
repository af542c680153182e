"""Static checks on the gfx950 ISA of the product kernels (CPU only: hipcc cross-compiles).

decode_lag_kernel issues a block's staging loads by inline asm (the waitcnt pass does not see
them).  That is sound only if no instruction reads or writes their
destination registers before the inline-asm `s_waitcnt vmcnt` that lands them, on every CFG
path, and if no VALU write of an SGPR they read comes within 5 wait states of them (a hazard
the compiler's hazard pass does not check inside inline asm)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _isa(tmp_path, src):
    out = tmp_path / (src + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include", "-DLSMBLK_DIAG_BUILD=0",
                    "--offload-device-only", "-S", "-o", str(out), os.path.join(ROOT, "lsm_amd", "csrc", src)],
                   check=True, capture_output=True, cwd=str(tmp_path))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_inline_asm_loads_are_landed_before_use(tmp_path):
    out = _isa(tmp_path, "lsmblk_gpu.hip")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_inflight_check.py"), str(out),
                        "decode_lag_kernel"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asm loads" in r.stdout and "OK" in r.stdout, r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_every_inline_asm_site_is_checked(tmp_path):
    """Every function with inline asm in the product sources passes the checks, and every asm
    instruction is of a kind the checker covers (a new kind of site fails until classified)."""
    paths = [str(_isa(tmp_path, f)) for f in ("lsmblk_gpu.hip", "lsmblk_compact.hip", "lsmblk_sst.hip")]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_inflight_check.py"), "--all", *paths],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    # decode_lag_kernel (staging loads), the crc / bloom kernels (SDWA), plan / large merge-tile waits
    for k in ("decode_lag_kernel", "crc_kernel", "plan_walk_kernel", "merge_big_kernel", "sst_bloom_kernel"):
        assert k in r.stdout, r.stdout
