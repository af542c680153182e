#!/bin/bash
# GPU box: decode lag x variant sweep (timing only; the headline bench checks every block).
#   tools/lag_sweep.sh "base sc1" "0 6144 8192"     (lag 0 = the default, 40 MiB of blocks)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in $1; do
  so=lsm_amd/var_$v.so; [ "$v" = base ] && so=lsm_amd/liblsmblk.so
  for lag in $2; do
    la=""; [ "$lag" != 0 ] && la="--decode-lag $lag"
    LSMBLK_SO_OVERRIDE=$PWD/$so timeout -k 10 120 python3 -u bench.py --no-extras --no-cpu-baseline --no-oracle-check \
      --no-pcie --steps 20 $la $BENCH_ARGS > gpurun_out/lag_${v}_$lag.json 2> gpurun_out/lag_${v}_$lag.log
    rc=$?; [ $rc -le 1 ] || exit 1  # (1: the line printed, round trip not bit-exact -- timing probes)
    python3 -c "
import json; d=json.load(open('gpurun_out/lag_${v}_$lag.json')); r=d['roofline']
print('$v lag $lag', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in r['kernels_ms'].items()})"
  done
done
