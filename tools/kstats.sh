#!/bin/bash
# GPU-box: rocprofv3 kernel-trace stats of a short bench run -> per-kernel average (us)
# usage: tools/kstats.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$TAG -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ks_$TAG.json 2> gpurun_out/ks_$TAG.err || { echo "rocprof failed"; tail -5 gpurun_out/ks_$TAG.err; exit 1; }
python3 - "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/ks_{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows:
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "at::native" in r["Name"] or "rocclr" in r["Name"]:
        continue
    print(f'{name:28s} calls {r["Calls"]:>4s} avg_us {float(r["AverageNs"]) / 1e3:9.1f}')
PY
