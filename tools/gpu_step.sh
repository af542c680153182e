#!/bin/bash
# GPU-box helper: run one named step with its own time limit, output under gpurun_out/.
# usage: tools/gpu_step.sh NAME SECONDS cmd...   (stops the chain on failure via the exit status)
NAME=$1; LIM=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 "$LIM" "$@" > "gpurun_out/$NAME.out" 2> "gpurun_out/$NAME.err"
rc=$?
echo "[$NAME] rc=$rc"
tail -3 "gpurun_out/$NAME.out"
[ $rc = 0 ] || tail -15 "gpurun_out/$NAME.err"
exit $rc
