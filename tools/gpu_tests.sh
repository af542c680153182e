#!/bin/bash
# GPU box: the GPU test suite (one process, per-test timeout), log under gpurun_out/
#   tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
exit $rc
