set -e
cd $GRAFT_REPO_ROOT
A="--config M --steps 10 --warmup 3 --no-cpu-baseline --no-pcie --no-oracle-check"
timeout -k 10 300 python -u bench.py $A > gpurun_out/m_lag.json 2> gpurun_out/m_lag.log
timeout -k 10 300 python -u bench.py $A --decode-two-pass > gpurun_out/m_2p.json 2> gpurun_out/m_2p.log
