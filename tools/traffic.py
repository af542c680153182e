"""Build profiles/traffic.json from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), one pair per
bench config (tools/traffic.sh).

HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE / WRITE_SIZE are KiB,
and on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read
(MI355X_MICROARCH.md, "HBM").  The doubling is calibrated for 16-B/lane loads: the decode /
emit / plan / count kernels stage with 16-B buffer loads; for the compaction kernels, whose
loads are narrower, the figure is an upper bound of the fabric bytes.

The file is stamped with the sha256 of the kernel sources it was measured at (lsm_amd/_build.py
src_sha); bench.py reports `traffic` only when that matches the sources it runs.
usage: python tools/traffic.py OUT_JSON COMMIT CFG=PMC_DIR [CFG=PMC_DIR ...]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lsm_amd._build import src_sha  # noqa: E402

# bench.py's roofline keys (its lsmblk_ctx_kernel_times slots) -> the kernels summed into them
SLOTS = {"decode": ["decode_lag_kernel"], "dec_count": ["dec_count_staged_kernel", "agg_tile_kernel"],
         "dec_scan": ["dec_scan_kernel"], "plan": ["plan_walk_kernel"], "emit": ["emit_kernel", "emit_big_kernel"],
         "decode_two_pass": ["decode_kernel"]}


def short(name):
    """Kernel function name without namespace, return type and argument list
    ("(anonymous namespace)::decode_lag_kernel((anonymous namespace)::DecodeArgs)" ->
    "decode_lag_kernel")."""
    n = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    n = n.split("::")[-1]
    return n.replace("void ", "").strip()


def one(root):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            per[(short(row["Kernel_Name"]), f, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    acc = defaultdict(lambda: defaultdict(list))
    for (name, f, d), cs in per.items():
        for c, v in cs.items():
            acc[name][c].append(v)
    kernels = {}
    for name, cs in acc.items():
        fk = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) if cs["FETCH_SIZE"] else 0.0
        wk = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) if cs["WRITE_SIZE"] else 0.0
        kernels[name] = {"dispatches": max(len(cs["FETCH_SIZE"]), len(cs["WRITE_SIZE"])), "fetch_kib": round(fk, 1),
                         "write_kib": round(wk, 1), "bytes_per_dispatch": int((2 * fk + wk) * 1024)}
    slots = {k: sum(kernels[n]["bytes_per_dispatch"] for n in v if n in kernels)
             for k, v in SLOTS.items() if any(n in kernels for n in v)}
    return {"kernels": kernels, "bytes_per_launch": slots}


def main():
    out, commit = sys.argv[1], sys.argv[2]
    res = {"src_sha256": src_sha(), "commit": commit, "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch",
           "configs": {}}
    for a in sys.argv[3:]:
        cfg, root = a.split("=", 1)
        res["configs"][cfg] = one(root)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({c: v["bytes_per_launch"] for c, v in res["configs"].items()}, indent=1))


if __name__ == "__main__":
    main()
