"""Per-block table of a phase_pmc2.sh log: python3 tools/phase_table.py LOG [nblk]"""
import re
import sys

txt = open(sys.argv[1]).read()
nb = float(sys.argv[2]) if len(sys.argv) > 2 else 270600.0
parts = re.split(r'== mask (\d+)', txt)
keys = ['SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_ACTIVE_INST_LDS',
        'SQ_WAVE_CYCLES', 'SQ_WAIT_ANY']
print(sys.argv[1], 'per block')
print('mask', *[k[3:] for k in keys])
for i in range(1, len(parts), 2):
    d = {}
    for line in parts[i + 1].splitlines():
        mm = re.match(r'\s+(\S+)\s+([\d.e+]+)\s+\(n=', line)
        if mm:
            d[mm.group(1)] = float(mm.group(2))
    print(parts[i], *[round(d.get(k, 0) / nb, 1) for k in keys])
