#!/bin/bash
# build a debug variant of liblsmblk.so with extra -D flags: tools/dbg_build.sh -DFOO
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function "$@" -Iinclude lsm_amd/csrc/lsmblk_gpu.hip lsm_amd/csrc/lsmblk_host.cpp -o lsm_amd/liblsmblk.so
