"""Side-by-side per-kernel averages of two rocprofv3 kernel_stats CSVs.
    python tools/prof_cmp.py A.csv B.csv [min_total_pct]"""
import csv
import sys


def load(p):
    return {r["Name"]: r for r in csv.DictReader(open(p))}


a, b = load(sys.argv[1]), load(sys.argv[2])
mn = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
names = sorted(set(a) | set(b), key=lambda n: -float((b.get(n) or a.get(n))["TotalDurationNs"]))
print(f"{'avg A us':>9} {'avg B us':>9} {'calls A':>7} {'calls B':>7} {'%B':>6}  kernel")
for n in names:
    ra, rb = a.get(n), b.get(n)
    pb = float(rb["Percentage"]) if rb else 0.0
    pa = float(ra["Percentage"]) if ra else 0.0
    if max(pa, pb) < mn:
        continue
    fa = f"{float(ra['AverageNs'])/1e3:9.2f}" if ra else f"{'-':>9}"
    fb = f"{float(rb['AverageNs'])/1e3:9.2f}" if rb else f"{'-':>9}"
    ca = ra["Calls"] if ra else "-"
    cb = rb["Calls"] if rb else "-"
    print(f"{fa} {fb} {ca:>7} {cb:>7} {pb:6.2f}  {n[:110]}")
