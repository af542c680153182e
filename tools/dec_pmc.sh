#!/bin/bash
# GPU box: decode instruction / wait counters per ablation mask (two SQ passes each, phase_probe.py).
# usage: tools/dec_pmc.sh TAG MASK... (PROBE_TWO_PASS=1 / PROBE_LAG=N pass through)
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for m in "$@"; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "decode" -d gpurun_out/dpmc_$TAG/m${m}_$i -o run -f csv \
      -- python3 tools/phase_probe.py decode $m > /dev/null 2> gpurun_out/dpmc_${TAG}_m${m}_$i.err \
      || { echo "mask $m pass $i failed"; tail -3 gpurun_out/dpmc_${TAG}_m${m}_$i.err; exit 1; }
  done
  echo "== mask $m"
  python3 tools/pmc_summary.py gpurun_out/dpmc_$TAG/m${m}_1
  python3 tools/pmc_summary.py gpurun_out/dpmc_$TAG/m${m}_2
done
