#!/bin/bash
# GPU box: LDS-pipe counters (one rocprofv3 --pmc run per group) for the headline kernels.
# usage: tools/pmc_lds.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
KRE='emit_kernel|decode_lag_kernel|plan_walk_kernel'
i=0
for grp in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY TCP_PENDING_STALL_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  LSMBLK_SO_OVERRIDE=${SO:-$PWD/lsm_amd/liblsmblk.so} timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d gpurun_out/pmc_$TAG/p$i -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pcie --no-oracle-check "$@" > /dev/null 2> gpurun_out/pmc_${TAG}_p$i.err || { echo "pass $i failed"; tail -3 gpurun_out/pmc_${TAG}_p$i.err; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG
