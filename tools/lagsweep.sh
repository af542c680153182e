# GPU box: lagged-decode ablations at one lag (usage: tools/lagsweep.sh LAG MASK...)
L=$1; shift
for M in "$@"; do
  timeout -k 10 100 python3 -u bench.py --no-extras --no-cpu-baseline --no-oracle-check --no-pcie --steps 10 --ablate $M --ablate-only --decode-lag $L > gpurun_out/sw_${L}_$M.out 2>&1 || exit 1
  echo "lag $L mask $M $(tail -1 gpurun_out/sw_${L}_$M.out | cut -c1-80)"
done
