#!/bin/bash
# GPU box: bench every variant .so named on the command line (plus the default build):
#   tools/var_bench.sh base v1 v2 ...   ("base" = lsm_amd/liblsmblk.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  so=lsm_amd/var_$v.so; [ "$v" = base ] && so=lsm_amd/liblsmblk.so
  LSMBLK_SO_OVERRIDE=$PWD/$so timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --no-oracle-check \
    --steps 20 $BENCH_ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.log || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/var_$v.json')); r=d['roofline']
print('$v', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in r['kernels_ms'].items()}, d['config'].get('roundtrip_bit_exact', d['config'].get('oracle_checked')))"
done
