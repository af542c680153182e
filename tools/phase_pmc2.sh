#!/bin/bash
# GPU-box: instruction / LDS-conflict PMC pass per ablation mask for one kernel.
# usage: tools/phase_pmc2.sh {encode|decode} KERNEL_REGEX MASK...
set -o pipefail
W=$1; KRE=$2; shift 2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for m in "$@"; do
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS \
    --kernel-include-regex "$KRE" -d gpurun_out/phase2_${W}/m$m -o run -f csv -- python3 tools/phase_probe.py $W $m \
    > /dev/null 2> gpurun_out/phase2_${W}_m$m.err || { echo "mask $m failed"; tail -3 gpurun_out/phase2_${W}_m$m.err; exit 1; }
  echo "== mask $m"
  python3 tools/pmc_summary.py gpurun_out/phase2_${W}/m$m
done
