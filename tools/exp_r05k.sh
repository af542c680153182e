set -e
cd $GRAFT_REPO_ROOT
A="--steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check"
timeout -k 10 300 python -u bench.py $A --trace-fused --encode-mode slots > gpurun_out/k_trace.json 2> gpurun_out/k_trace.log
