"""Fold the pmc_traffic.sh passes into profiles/pmc_traffic.json: per bench kernel the HBM
bytes of one launch (median over dispatches). FETCH_SIZE is doubled: on gfx950 it reports
half the bytes of 16-byte-per-lane streaming reads (MI355X_MICROARCH.md, HBM section);
WRITE_SIZE is exact for 16-byte stores. Both are KiB in rocprofv3's derived counters.

    python tools/pmc_layers.py gpurun_out/pmc_traffic profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

LAYERS = {"l1": "conv1+pool", "l2": "conv2+pool", "l3": "conv3+pool", "ct1": "convT1",
          "ct2": "convT2", "ct3": "convT3", "last": "conv_out", "tail": "convT3+conv_out",
          "stft_c2": "stft_c2"}
# the layer's own kernel (tools/conv_one.py adds a 1x1 tail conv after the convT layers)
KERNEL = {"l1": "conv_c1_kernel", "l2": "Li2ELi16ELb1", "l3": "Li4ELi32ELb1",
          "ct1": "Li4ELi64ELb0", "ct2": "Li2ELi64ELb0", "ct3": "Li1ELi32ELb0",
          "last": "conv_co1", "tail": "convt_conv_out", "stft_c2": "stft_team"}


def one(path, must="", skip=("cast", "flip", "Fill", "fill", "copy", "at::native", "rocclr")):
    per = collections.defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "specenh" not in k or must not in k or any(s in k for s in skip):
                continue
            d = row["Dispatch_Id"]
            per[k][d] = per[k].get(d, 0.0) + float(row["Counter_Value"])
            names[k] = k
    # the layer's own kernel: the one with the most dispatches x bytes
    best = max(per, key=lambda k: statistics.median(per[k].values()) * len(per[k]))
    return best, statistics.median(per[best].values())


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {}
    for tag, name in LAYERS.items():
        fk, fv = one(os.path.join(src, f"{tag}_FETCH_SIZE"), KERNEL[tag])
        wk, wv = one(os.path.join(src, f"{tag}_WRITE_SIZE"), KERNEL[tag])
        res[name] = {"kernel": fk, "fetch_bytes": 2 * fv * 1024, "write_bytes": wv * 1024,
                     "hbm_bytes": 2 * fv * 1024 + wv * 1024,
                     "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                               "FETCH x2 (gfx950 wide-read correction), KiB -> bytes"}
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k, v["kernel"][:70], f"{v['hbm_bytes']/1e9:.3f} GB")


if __name__ == "__main__":
    main()
