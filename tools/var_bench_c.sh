#!/bin/bash
# GPU box: config C (compaction) for the default build and each variant named (lsm_amd/var_NAME.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  so=lsm_amd/var_$v.so; [ "$v" = base ] && so=lsm_amd/liblsmblk.so
  LSMBLK_SO_OVERRIDE=$PWD/$so timeout -k 10 300 python3 -u bench.py --config C --no-cpu-baseline --steps 5 --warmup 2 \
    > gpurun_out/varc_$v.json 2> gpurun_out/varc_$v.log || exit 1
  python3 -c "
import json
for l in open('gpurun_out/varc_$v.json'):
    if l.startswith('{'):
        d = json.loads(l); print('$v', d['value'], d['ms_per_step'], d['stage_ms'], d['config']['compaction_bit_exact'])"
done
