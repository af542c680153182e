#!/bin/bash
# GPU box: parity tests, then a short bench per config: tools/bench_cfgs.sh TAG [U Z M ...]
# Prints GiB/s and per-kernel ms for each config.
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for cfg in "${@:-U}"; do
  timeout -k 10 300 python3 bench.py --config "$cfg" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json'));r=d['roofline'];print('$cfg',d['value'],'GiB/s',r['kernels_ms'],'ok',d['config'].get('roundtrip_bit_exact'))"
done
