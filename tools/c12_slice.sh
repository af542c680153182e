#!/bin/bash
# configs[4]'s per-GPU slice on one GPU: 3 key ranges x 1 Mi blocks (12.7 GB of L0 input), every
# output block oracle-checked range by range; the line reports peak host RSS and wall time
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py --config C --blocks 3145728 --ranges-per-gpu 3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r05_C12g_bench.json 2> gpurun_out/r05_C12g_bench.log
rc=$?; tail -5 gpurun_out/r05_C12g_bench.log; exit $rc
