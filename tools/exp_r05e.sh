#!/bin/bash
# emit_big chunk pipelining: full GPU suite, then A/B at config M against the unpipelined kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh r05e || exit 1
BENCH_ARGS="--config M" bash tools/var_bench.sh base eb4np pp2 pp3 base eb4np pp3 pp2
