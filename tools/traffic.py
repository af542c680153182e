"""Build profiles/traffic.json from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE / WRITE_SIZE are KiB,
and on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read
(MI355X_MICROARCH.md, "HBM").  The doubling is calibrated for 16-B/lane loads only: the
decode / emit / plan / staged count kernels stage with 16-B buffer loads.
usage: python tools/traffic.py PMC_DIR WORKLOAD BLOCKS OUT_JSON
"""
import csv, glob, json, os, sys
from collections import defaultdict

NAMES = {"decode_lag_kernel": "decode", "dec_count_kernel": "dec_count", "dec_count_staged_kernel": "dec_count", "dec_scan_kernel": "dec_scan", "decode_kernel": "decode_two_pass",
         "plan_adj_kernel": "plan_adj", "plan_walk_kernel": "plan_walk", "emit_kernel": "emit",
         "crc_kernel<false>": "crc32", "crc_kernel<true>": "crc32_count", "agg_tile_kernel": "agg_tile"}
root, workload, blocks, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = next((v for k, v in NAMES.items() if k in row["Kernel_Name"]), None)
        if name:
            per[(name, f, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
acc = defaultdict(lambda: defaultdict(list))
for (name, f, d), cs in per.items():
    for c, v in cs.items():
        acc[name][c].append(v)
res = {"workload": workload, "blocks": blocks, "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024",
       "fetch_kib": {}, "write_kib": {}, "bytes_per_launch": {}}
for name, cs in acc.items():
    fk = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) if cs["FETCH_SIZE"] else 0.0
    wk = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) if cs["WRITE_SIZE"] else 0.0
    res["fetch_kib"][name] = fk
    res["write_kib"][name] = wk
    res["bytes_per_launch"][name] = int((2 * fk + wk) * 1024)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
