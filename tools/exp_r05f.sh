#!/bin/bash
# large-block count from the staged tail + one 32-byte window per entry: decode tests, then A/B
# (M and U) against the previous build (var_head)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh r05f2 "decode or large or malformed or configs or roundtrip or golden or verify or framed or crc" || exit 1
BENCH_ARGS="--config M" bash tools/var_bench.sh base head base head || exit 1
bash tools/var_bench.sh base head base head
