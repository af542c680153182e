# A/B: the plan walk's pipelined helper (default) against the unpipelined one and the session-start build
set -e
cd $GRAFT_REPO_ROOT
LSMBLK_PLAN_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/n_tests.log 2>&1
A="--steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-pcie --no-oracle-check"
for cfg in U Z M; do
  timeout -k 10 300 python -u bench.py $A --config $cfg --plan-pipe 1 > gpurun_out/n_${cfg}_pipe.json 2> gpurun_out/n_${cfg}_pipe.log
  timeout -k 10 300 python -u bench.py $A --config $cfg > gpurun_out/n_${cfg}_nopipe.json 2> gpurun_out/n_${cfg}_nopipe.log
  LSMBLK_SO_OVERRIDE=$PWD/ab/liblsmblk_old.so timeout -k 10 300 python -u bench.py $A --config $cfg > gpurun_out/n_${cfg}_old.json 2> gpurun_out/n_${cfg}_old.log
done
