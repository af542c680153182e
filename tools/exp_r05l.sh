set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/l_tests.log 2>&1
A="--steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check"
timeout -k 10 300 python -u bench.py $A --encode-mode slots > gpurun_out/l_slots.json 2> gpurun_out/l_slots.log
timeout -k 10 300 python -u bench.py $A --encode-mode packed > gpurun_out/l_packed.json 2> gpurun_out/l_packed.log
timeout -k 10 300 python -u bench.py $A --encode-mode slots --config Z > gpurun_out/l_slotsZ.json 2> gpurun_out/l_slotsZ.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check --trace-fused --encode-mode slots > gpurun_out/l_trace.json 2> gpurun_out/l_trace.log
