"""Print one step's kernel timeline from a rocprofv3 --kernel-trace CSV (config C analysis).
usage: python3 tools/ktrace.py gpurun_out/ktC/run_kernel_trace.csv [first-kernel-substring]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "decode_lag"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0 = idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
end = 0
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).replace("void ", "")
    name = name.split("(")[0]
    end = max(end, e)
    print(f"{s / 1000:9.1f} {e / 1000:9.1f} {(e - s) / 1000:8.1f}  q{r['Queue_Id']}  {name[:60]}")
print(f"step span {end / 1000:.1f} us")
