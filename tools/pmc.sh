#!/bin/bash
# GPU-box helper: PMC counter passes (one rocprofv3 run per group) for one kernel.
# usage: tools/pmc.sh TAG KERNEL_REGEX [bench args...]
set -o pipefail
TAG=$1; KRE=$2; shift 2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d gpurun_out/pmc_$TAG/p$i -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> gpurun_out/pmc_${TAG}_p$i.err || { echo "pass $i failed"; tail -3 gpurun_out/pmc_${TAG}_p$i.err; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG
