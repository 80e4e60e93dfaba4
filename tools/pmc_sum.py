"""Average per-launch PMC counters of one kernel family from tools/pmc_sq.sh output.
    python tools/pmc_sum.py DIR TAG [KERNEL_SUBSTRING]"""
import collections
import csv
import glob
import sys

d, tag = sys.argv[1], sys.argv[2]
sub = sys.argv[3] if len(sys.argv) > 3 else "conv_patch"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/{tag}_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    print(k)
    print("   ", {n: "%.3g" % (sum(v) / len(v)) for n, v in c.items()})
