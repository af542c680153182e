#!/bin/bash
# GPU box: HBM traffic counters of config M's large-block kernels (emit_big, decode_lag), one pass each
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex "emit_big_kernel|decode_lag_kernel" \
    -d gpurun_out/tm_$i -o run -f csv -- python3 bench.py --config M --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie \
    > /dev/null 2> gpurun_out/tm_$i.err || { echo "pmc $c failed"; tail -3 gpurun_out/tm_$i.err; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/tm_$i
done
