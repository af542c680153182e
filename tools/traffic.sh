#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (each its own run) over every bench config's workload
# -> traffic json stamped with the kernel-source sha (bench.py reports traffic only on a match)
# usage: tools/traffic.sh OUT_JSON [COMMIT] [CONFIGS...]
set -o pipefail
OUT=${1:-gpurun_out/traffic.json}
COMMIT=${2:-unknown}
shift 2
CFGS=${@:-U Z M C}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
args=()
for cfg in $CFGS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/traffic_$cfg/$c -o run -f csv -- python3 bench.py --config $cfg \
      --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie --no-oracle-check > /dev/null 2> gpurun_out/traffic_${cfg}_$c.err \
      || { echo "pmc $cfg $c failed"; tail -3 gpurun_out/traffic_${cfg}_$c.err; exit 1; }
  done
  args+=("$cfg=gpurun_out/traffic_$cfg")
done
python3 tools/traffic.py "$OUT" "$COMMIT" "${args[@]}"
