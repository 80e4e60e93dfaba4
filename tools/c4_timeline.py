"""One C4 step's kernels from a rocprofv3 kernel trace (csv): queue, start, end, duration.
    python tools/c4_timeline.py gpurun_out/c4trace_TAG/run_kernel_trace.csv"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
s, e = ad[-3] + 1, ad[-2] + 1
t0 = int(rows[s]["Start_Timestamp"])


def short(n):
    n = n.replace("specenh::", "")
    m = re.match(r"_ZN7specenh(?:12_GLOBAL__N_1)?(\d+)(\w+)", n)
    if m:
        n = m.group(2)[:int(m.group(1))] + n[m.end():][:40]
    return n[:70]


for r in rows[s:e]:
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    en = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{r['Queue_Id']:>3} {st:8.1f} {en:8.1f} {en - st:6.1f}  {short(r['Kernel_Name'])}")
