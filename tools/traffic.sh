#!/bin/bash
# GPU-box: FETCH_SIZE and WRITE_SIZE passes over the default bench workload -> traffic json
set -o pipefail
OUT=${1:-gpurun_out/traffic.json}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex "dec_count_kernel|dec_count_staged_kernel|decode_kernel|decode_lag_kernel|plan_adj_kernel|plan_walk_kernel|emit_kernel|crc_kernel|agg_tile_kernel" \
    -d gpurun_out/traffic/$c -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie > /dev/null 2> gpurun_out/traffic_$c.err || { echo "pmc $c failed"; exit 1; }
done
python3 tools/traffic.py gpurun_out/traffic U 1048576 "$OUT"
