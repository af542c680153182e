#!/bin/bash
# GPU box: decode A/B -- the lagged decode at several lags against the two-pass path (U, 20 steps)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --no-oracle-check --no-pcie --steps 20 "$@" \
    > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.log || { echo "$n failed"; tail -5 gpurun_out/ab_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in r['kernels_ms'].items()}, d['config']['roundtrip_bit_exact'])"
}
for v in "$@"; do
  case $v in
    two) run two --decode-two-pass || exit 1 ;;
    lag*) run $v --decode-lag ${v#lag} || exit 1 ;;
    *) run $v || exit 1 ;;
  esac
done
