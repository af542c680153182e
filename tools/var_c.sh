#!/bin/bash
# GPU box: config C per variant .so (plus "base" = the default build): bench value + rocprof per-kernel averages
#   tools/var_c.sh base v1 ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  so=lsm_amd/var_$v.so; [ "$v" = base ] && so=lsm_amd/liblsmblk.so
  export LSMBLK_SO_OVERRIDE=$PWD/$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vc_$v -o run -- python3 -u bench.py --config C \
    --no-extras --no-cpu-baseline --steps 10 > gpurun_out/vc_$v.json 2> gpurun_out/vc_$v.log || exit 1
  python3 - "$v" <<'PY' || exit 1
import csv, glob, json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/vc_{v}.json") if l.startswith("{")][-1])
f = glob.glob(f"gpurun_out/vc_{v}/**/*kernel_stats.csv", recursive=True)[0]
ks = {}
for r in csv.DictReader(open(f)):  # per step (warmup + timed steps; the oracle check adds a little)
    k = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
    ks[k] = ks.get(k, 0) + float(r["TotalDurationNs"]) / 1e6 / 13
top = sorted(ks.items(), key=lambda x: -x[1])[:12]
print(v, d["value"], d["ms_per_step"], d["stage_ms"], d["config"]["compaction_bit_exact"], {k: round(x, 3) for k, x in top})
PY
done
