#!/bin/bash
# occupancy sensitivity: the lagged decode at 16 / 12 waves per CU and emit at 12 (LDS padding)
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/var_bench.sh base dp16 dp12 ep12 base dp16 dp12 ep12
