#!/bin/bash
# emit_big: record fields stored after their copy round (A/B against the previous build, var_ebold)
# + the full GPU suite + emit_big WRITE_SIZE at config M
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh r05d || exit 1
BENCH_ARGS="--config M" bash tools/var_bench.sh base ebold base ebold || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex emit_big -d gpurun_out/pmc_r05d_w -o run -f csv -- \
  python3 bench.py --config M --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie --no-oracle-check > /dev/null 2> gpurun_out/pmc_r05d_w.err || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_r05d_w
