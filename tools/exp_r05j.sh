set -e
cd $GRAFT_REPO_ROOT
A="--steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check"
timeout -k 10 300 python -u bench.py $A --encode-mode slots > gpurun_out/j_slots.json 2> gpurun_out/j_slots.log
timeout -k 10 300 python -u bench.py $A --encode-mode slots --config Z > gpurun_out/j_slotsZ.json 2> gpurun_out/j_slotsZ.log
