#!/bin/bash
# GPU-box: parity tests -> full bench (cpu baseline + pcie) -> rocprof stats -> PMC traffic passes.
# usage: tools/round_gpu.sh TAG COMMIT [--no-pmc]   (the box has no .git: COMMIT stamps traffic.json)
set -o pipefail
TAG=$1; COMMIT=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 540 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
# the headline workload alone (the extras' kernels would mix into the per-kernel averages)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -f csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-pcie > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || { echo "rocprof failed"; exit 1; }
for cfg in M C; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$cfg -o run -f csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/benchprof_${TAG}_$cfg.json 2> gpurun_out/benchprof_${TAG}_$cfg.err || { echo "rocprof $cfg failed"; exit 1; }
done
head -6 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -d, -f1-4
if [ "$1" != "--no-pmc" ]; then
  bash tools/traffic.sh gpurun_out/traffic_$TAG.json "$COMMIT" U Z M C || exit 1
  cat gpurun_out/traffic_$TAG.json
fi
