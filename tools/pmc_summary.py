"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel name, the median over
dispatches of each counter (summed over the dimension instances of one dispatch).

    python tools/pmc_summary.py gpurun_out/pmc_conv/p*/p*_counter_collection.csv
"""
import collections
import csv
import statistics
import sys


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kern -> ctr -> disp -> v
    for path in sys.argv[1:]:
        for row in csv.DictReader(open(path)):
            k = row["Kernel_Name"]
            c = row["Counter_Name"]
            d = row["Dispatch_Id"]
            per[k][c][d] = per[k][c].get(d, 0.0) + float(row["Counter_Value"])
    for k, ctrs in per.items():
        print(k[:110])
        for c, disp in sorted(ctrs.items()):
            print(f"    {c:28s} {statistics.median(disp.values()):.4g}")


if __name__ == "__main__":
    main()
