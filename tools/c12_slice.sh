set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 /usr/bin/time -v python3 -u bench.py --config C --blocks 3145728 --ranges-per-gpu 3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r05_C12g_bench.json 2> gpurun_out/r05_C12g_bench.log
rc=$?; tail -25 gpurun_out/r05_C12g_bench.log | grep -E "Maximum resident|Elapsed|oracle" ; exit $rc
