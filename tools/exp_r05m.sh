# A/B: session-start library (ab/liblsmblk_old.so) against the current one, U packed, alternating
set -e
cd $GRAFT_REPO_ROOT
A="--steps 20 --warmup 3 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check --encode-mode packed"
for r in 1 2; do
  LSMBLK_SO_OVERRIDE=$PWD/ab/liblsmblk_old.so timeout -k 10 300 python -u bench.py $A > gpurun_out/m_old$r.json 2> gpurun_out/m_old$r.log
  timeout -k 10 300 python -u bench.py $A > gpurun_out/m_new$r.json 2> gpurun_out/m_new$r.log
done
