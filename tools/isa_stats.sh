#!/bin/bash
# Resource usage (VGPRs, LDS, spills) of kernels from the gfx950 ISA of one source file.
# usage: tools/isa_stats.sh [SRC (default lsmblk_gpu.hip)] [NAME_SUBSTRING...]
SRC=lsmblk_gpu.hip
case "$1" in *.hip) SRC=$1; shift;; esac
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/include -DLSMBLK_DIAG_BUILD=0 --offload-device-only -S \
  -o /tmp/isa_stats.s /root/repo/lsm_amd/csrc/$SRC 2>/dev/null || exit 1
python3 - "$@" <<'PY'
import re, sys
s = open('/tmp/isa_stats.s').read()
md = s[s.index('amdhsa.kernels'):]
pat = sys.argv[1:] or ['decode', 'dec_count', 'emit_kernel', 'plan_walk']
for blk in md.split('  - .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if any(k in name for k in pat):
        g = lambda k: re.search(r'\.' + k + r':\s+(\d+)', blk).group(1)
        print(f"{name[:60]:60s} vgpr {g('vgpr_count'):>4s} sgpr {g('sgpr_count'):>4s} lds {g('group_segment_fixed_size'):>6s} "
              f"vspill {g('vgpr_spill_count')} scratch {g('private_segment_fixed_size')}")
PY
