set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --no-pcie --steps 10 --ablate 0 --ablate-lag > gpurun_out/e1_ablate_U.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --no-pcie --steps 10 --decode-two-pass > gpurun_out/e1_twopass_U.json 2>gpurun_out/e1_twopass_U.err && \
timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --no-pcie --steps 10 --ablate 65536 --ablate-only > gpurun_out/e1_plan_U.log 2>&1
echo done
