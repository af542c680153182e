#!/bin/bash
# GPU box: large-block decode ablations on config M (diagnostics only)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for m in 1024 2048 4096 7168; do
  timeout -k 10 200 python3 -u bench.py --config M --no-extras --no-cpu-baseline --no-oracle-check --steps 10 --ablate $m \
    > gpurun_out/ablm_$m.json 2> gpurun_out/ablm_$m.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ablm_$m.json'))['ablation_decode_ms_by_skip_mask']; print($m, d['0'], d['$m'])"
done
