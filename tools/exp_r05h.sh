# round 5: fused walk + emit (per-segment slots) -- GPU parity tests, then U packed / slots / slots-unfused
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h_tests.log 2>&1
A="--steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-pcie"
timeout -k 10 400 python -u bench.py $A --encode-mode slots > gpurun_out/h_slots.json 2> gpurun_out/h_slots.log
timeout -k 10 300 python -u bench.py $A --no-oracle-check --encode-mode packed > gpurun_out/h_packed.json 2> gpurun_out/h_packed.log
timeout -k 10 300 python -u bench.py $A --no-oracle-check --encode-mode slots-unfused > gpurun_out/h_unfused.json 2> gpurun_out/h_unfused.log
