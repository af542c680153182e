#!/bin/bash
# GPU-box dev cycle: GPU parity tests, then a short bench (per-kernel ms from HIP events).
# usage: tools/dev_gpu.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print(d['value'],'GiB/s',d['ms_per_step'],'ms',r['kernels_ms'],'ok',d['config'].get('roundtrip_bit_exact'))"
