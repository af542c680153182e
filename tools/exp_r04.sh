#!/bin/bash
# GPU box: GPU tests at the working tree's build, then A/B: config M (base vs h0), config C (h0 vs merge-tile variants)
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 90 --timeout-method thread > gpurun_out/tests_exp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_exp.log; exit 1; }
tail -1 gpurun_out/tests_exp.log
timeout -k 10 120 ./tools/copy_probe > gpurun_out/copy_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/copy_probe.txt
BENCH_ARGS="--config M" bash tools/var_bench.sh base h0 || exit 1
bash tools/var_bench_c.sh h0 mA mB mC mD || exit 1
