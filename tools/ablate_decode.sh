#!/bin/bash
# time decode under ablation masks (outputs are wrong under a mask; timing only)
cd "$(dirname "$0")/.."
for m in 0 1 2 4 8 14 15; do
  LSMBLK_DEBUG_SKIP=$m timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('skip=$m', 'decode_ms', r['decode_ms'], 'encode_ms', r['encode_ms'])"
done
