#!/bin/bash
# GPU box: GPU tests at the working tree's build, then U A/B (plan helper variant p1 vs h0), alternating
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 90 --timeout-method thread > gpurun_out/tests_exp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_exp.log; exit 1; }
tail -1 gpurun_out/tests_exp.log
bash tools/var_bench.sh h0 p1 h0 p1 || exit 1
BENCH_ARGS="--config Z" bash tools/var_bench.sh h0 p1 || exit 1
