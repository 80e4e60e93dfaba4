"""MFMA utilisation of each layer's own kernel from tools/pmc_mfma.sh output:
util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8
(rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs; MI355X_MICROARCH.md, PMC units).

    python tools/pmc_mfma_summary.py gpurun_out/pmc_mfma [out.json]
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

SIMDS = 256 * 4
KERNEL = {"l1": "conv_c1_kernel", "l2": "Li2ELi16ELb1", "l3": "Li4ELi32ELb1", "ct1": "Li4ELi64ELb0",
          "ct2": "Li2ELi64ELb0", "ct3": "Li1ELi32ELb0", "last": "conv_co1", "tail": "convt_conv_out"}


def main():
    src = sys.argv[1]
    res = {}
    for layer, sub in KERNEL.items():
        files = glob.glob(os.path.join(src, layer, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        name = None
        for f in files:
            for row in csv.DictReader(open(f)):
                if sub not in row["Kernel_Name"]:
                    continue
                name = row["Kernel_Name"]
                per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        if not per:
            continue
        med = {c: statistics.median(d[c] for d in per.values()) for c in next(iter(per.values()))}
        cyc = med["GRBM_GUI_ACTIVE"] / 8
        r = {"kernel": name, "kernel_cycles": cyc,
             "mfma_util": med["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc),
             "mfma_insts": med["SQ_INSTS_MFMA"], "valu_insts": med["SQ_INSTS_VALU"],
             "lds_insts": med["SQ_INSTS_LDS"],
             "lds_bank_conflict_frac": med["SQ_LDS_BANK_CONFLICT"] / max(med["SQ_LDS_IDX_ACTIVE"], 1),
             "counters": med}
        res[layer] = r
        print(f"{layer:5s} util {r['mfma_util']:.3f}  cycles {cyc:.3g}  mfma {r['mfma_insts']:.3g} "
              f"valu {r['valu_insts']:.3g} lds {r['lds_insts']:.3g} "
              f"conflict {r['lds_bank_conflict_frac']:.3f}  {name[:60]}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
