set -e
cd $GRAFT_REPO_ROOT
A="--steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check"
timeout -k 10 300 python -u bench.py $A --trace-fused > gpurun_out/k_trace.json 2> gpurun_out/k_trace.log
timeout -k 10 300 python -u bench.py $A --trace-plan --encode-mode packed > gpurun_out/k_plantrace.json 2> gpurun_out/k_plantrace.log
