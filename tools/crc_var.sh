#!/bin/bash
# GPU box: tools/crc_time.py for the default library and each variant named (lsm_amd/var_NAME.so)
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 120 python3 tools/crc_time.py || exit 1
for v in "$@"; do
  LSMBLK_SO_OVERRIDE=$PWD/lsm_amd/var_$v.so timeout -k 10 120 python3 tools/crc_time.py || exit 1
done
