#!/bin/bash
# GPU-box helper: parity tests, then a rocprofv3 kernel-trace of a short bench run.
# usage: tools/prof_bench.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/tests_$TAG.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench rc=$?"
cat gpurun_out/bench_$TAG.json
head -6 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -d, -f1-4
