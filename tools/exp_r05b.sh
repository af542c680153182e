#!/bin/bash
# plan walk: LDS padding (at most two walker workgroups per CU) A/B + per-segment traces
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u bench.py --no-extras --no-cpu-baseline --no-pcie --no-oracle-check --steps 5 --trace-plan > gpurun_out/e5_trace_base.log 2>&1 || exit 1
LSMBLK_SO_OVERRIDE=$PWD/lsm_amd/var_paddiag.so timeout -k 10 120 python3 -u bench.py --no-extras --no-cpu-baseline --no-pcie --no-oracle-check --steps 5 --trace-plan > gpurun_out/e5_trace_pad.log 2>&1 || exit 1
grep plan_trace gpurun_out/e5_trace_base.log gpurun_out/e5_trace_pad.log
bash tools/var_bench.sh base pad base pad || exit 1
BENCH_ARGS="--config Z" bash tools/var_bench.sh base pad base pad
