#!/bin/bash
# GPU box: SQ instruction / wait counters of the compaction kernels (bench.py --config C, two passes)
# usage: tools/cpmc.sh TAG [REGEX] [CONFIG]
set -o pipefail
TAG=$1
RX=${2:-"merge_tile|mwrite|rot_next|rot_double|rot_f_|cand_rank|mflag|bounds"}
CFG=${3:-C}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d gpurun_out/cpmc_$TAG/p$i -o run -f csv \
    -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie --no-oracle-check \
    > /dev/null 2> gpurun_out/cpmc_${TAG}_$i.err || { echo "pass $i failed"; tail -3 gpurun_out/cpmc_${TAG}_$i.err; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/cpmc_$TAG/p$i
done
