#!/bin/bash
# GPU box: TCC read requests (all / DRAM-destined / 64 B / 128 B) of the decode kernels at one lag
# usage: tools/dram_pass.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
  --kernel-include-regex "decode_lag_kernel|decode_kernel|dec_count_staged_kernel|emit_kernel" \
  -d gpurun_out/dram_$TAG -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie "$@" \
  > /dev/null 2> gpurun_out/dram_$TAG.err || { echo "pmc failed"; tail -3 gpurun_out/dram_$TAG.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/dram_$TAG
