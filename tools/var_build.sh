#!/bin/bash
# Build a variant of liblsmblk.so with extra -D flags (experiments): tools/var_build.sh NAME -DFOO=1 ...
# -> lsm_amd/var_NAME.so, selected at run time by LSMBLK_SO_OVERRIDE
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wshadow -Wno-unused-function -DLSMBLK_DIAG_BUILD=${DIAG:-0} "$@" -Iinclude \
  lsm_amd/csrc/lsmblk_gpu.hip lsm_amd/csrc/lsmblk_compact.hip lsm_amd/csrc/lsmblk_sst.hip lsm_amd/csrc/lsmblk_host.cpp \
  -o lsm_amd/var_$NAME.so
