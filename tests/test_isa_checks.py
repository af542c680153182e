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


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_inline_asm_loads_are_landed_before_use(tmp_path):
    out = tmp_path / "lsmblk_gpu.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include", "--offload-device-only",
                    "-S", "-o", str(out), os.path.join(ROOT, "lsm_amd", "csrc", "lsmblk_gpu.hip")],
                   check=True, capture_output=True, cwd=str(tmp_path))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_inflight_check.py"), str(out),
                        "decode_lag_kernel"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asm loads" in r.stdout and "OK" in r.stdout, r.stdout
