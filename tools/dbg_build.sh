#!/bin/bash
# Debug build of liblsmblk.so with device printf (never shipped): tools/dbg_build.sh OUT.so
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DLSMBLK_DEVICE_DEBUG -Iinclude \
  lsm_amd/csrc/lsmblk_gpu.hip lsm_amd/csrc/lsmblk_host.cpp -o "$1"
