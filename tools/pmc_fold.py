"""Fold the rocprofv3 --pmc passes of tools/pmc_refresh.sh into one JSON keyed by target,
stage and exact kernel symbol (the file bench.py reads: profiles/pmc_r05.json).

    python tools/pmc_fold.py gpurun_out/pmc profiles/pmc_r05.json

Each pass directory <target>_<pass> holds rocprofv3's counter_collection.csv and the
manifest of tools/pmc_workload.py. The i-th dispatch whose kernel name contains "specenh"
(Dispatch_Id order) is the library's i-th launch on the host (specenh_launch_count), so the
manifest's index ranges say which dispatches belong to which stage; the count of such
dispatches must equal the manifest's total or the pass is rejected. Per stage and launch
position, counters are medians over the profiled repetitions.

Units and corrections (MI355X_MICROARCH.md, HBM / PMC sections):
  FETCH_SIZE, WRITE_SIZE  KiB; FETCH_SIZE is doubled (gfx950 reports half the bytes of wide
                          streaming reads); WRITE_SIZE exact for 16-byte stores
  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_*   quad-cycles (ratios only are reported)
  SQ_VALU_MFMA_BUSY_CYCLES  cycles; mfma_busy = it / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

SIMDS = 256 * 4


def demangled_match(symbol, csv_name):
    """True when rocprofv3's Kernel_Name (demangled where its demangler could) names the
    mangled ``symbol``: equal strings, or the demangled form starts with the symbol's
    qualified name (namespaces + kernel identifier parsed from the Itanium mangling)."""
    if symbol == csv_name:
        return True
    m = re.match(r"_ZN((?:\d+[A-Za-z_][A-Za-z0-9_]*)+)", symbol)
    if not m:
        return False
    parts, s = [], m.group(1)
    while s and s[0].isdigit():
        n = int(re.match(r"\d+", s).group())
        k = len(str(n))
        parts.append(s[k:k + n])
        s = s[k + n:]
    parts = [("(anonymous namespace)" if p == "_GLOBAL__N_1" else p) for p in parts]
    return "::".join(parts) in csv_name


def read_pass(d):
    man_path = os.path.join(d, "manifest.json")
    if not os.path.exists(man_path):
        return None, None
    man = json.load(open(man_path))
    per = collections.OrderedDict()
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "specenh" not in row["Kernel_Name"]:
                continue
            did = int(row["Dispatch_Id"])
            per.setdefault(did, collections.defaultdict(float))
            per[did][row["Counter_Name"]] += float(row["Counter_Value"])
            names[did] = row["Kernel_Name"]
    ids = sorted(per)
    if len(ids) != man["total_launches"]:
        raise SystemExit(f"{d}: {len(ids)} specenh dispatches in the CSV, manifest counts "
                         f"{man['total_launches']} launches: cannot attribute")
    return man, [(names[i], per[i]) for i in ids]


def fold(src):
    passes = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(src, "*_*"))):
        if os.path.isdir(d):
            passes[os.path.basename(d).rsplit("_", 1)[0]].append(d)
    out = {}
    for target, dirs in passes.items():
        stages = collections.OrderedDict()
        batch = None
        for d in dirs:
            man, disp = read_pass(d)
            if man is None:
                continue
            batch = man["batch"]
            # stage -> launch position -> list of counter dicts over reps
            acc = collections.defaultdict(lambda: collections.defaultdict(list))
            syms = {}
            for rep in man["reps"]:
                for st in rep:
                    syms[st["stage"]] = st["symbols"]
                    for k, i in enumerate(range(st["first"], st["end"])):
                        name, ctr = disp[i]
                        if not demangled_match(st["symbols"][k], name):
                            raise SystemExit(f"{d}: launch {i} is {name!r} in the CSV, the host "
                                             f"recorded {st['symbols'][k]!r}")
                        acc[st["stage"]][k].append((name, ctr))
            for stage, posd in acc.items():
                rec = stages.setdefault(stage, {"symbols": syms[stage], "kernels": []})
                while len(rec["kernels"]) < len(posd):
                    rec["kernels"].append({"symbol": syms[stage][len(rec["kernels"])],
                                           "csv_name": None, "counters": {}})
                for k, lst in posd.items():
                    kr = rec["kernels"][k]
                    kr["csv_name"] = lst[0][0]
                    for c in lst[0][1]:
                        kr["counters"][c] = statistics.median(x[1][c] for x in lst)
        for stage, rec in stages.items():
            tot_f = tot_w = 0.0
            have_f = have_w = True
            for kr in rec["kernels"]:
                c = kr["counters"]
                if "FETCH_SIZE" in c:
                    kr["fetch_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024
                    tot_f += kr["fetch_bytes"]
                else:
                    have_f = False
                if "WRITE_SIZE" in c:
                    kr["write_bytes"] = c["WRITE_SIZE"] * 1024
                    tot_w += kr["write_bytes"]
                else:
                    have_w = False
                if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    kr["hbm_bytes"] = kr["fetch_bytes"] + kr["write_bytes"]
                if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    cyc = c["GRBM_GUI_ACTIVE"] / 8
                    kr["kernel_cycles"] = cyc
                    kr["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
                if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
                    w = c["SQ_WAVE_CYCLES"]
                    kr["wait_frac"] = c.get("SQ_WAIT_ANY", 0) / w
                    kr["issue_stall_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / w
                    kr["active_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / w
                if "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"] > 0:
                    kr["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                if c.get("SQ_INSTS_MFMA"):
                    kr["valu_per_mfma"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"]
            if have_f:
                rec["fetch_bytes"] = tot_f
            if have_w:
                rec["write_bytes"] = tot_w
            if have_f and have_w:
                rec["hbm_bytes"] = tot_f + tot_w
            rec["batch"] = batch
            main_k = max(rec["kernels"], key=lambda k: k.get("hbm_bytes", 0) +
                         k.get("kernel_cycles", 0))
            rec["dominant"] = main_k["symbol"]
        out[target] = dict(stages)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]  # dst is updated in place
    res = fold(src)
    # targets not profiled in this run keep their earlier records; a re-profiled target is
    # replaced stage by stage (stages it no longer has are kept, their symbols say what ran)
    try:
        with open(dst) as fh:
            old = json.load(fh)
    except (OSError, ValueError):
        old = {}
    for target, stages in old.items():
        if target.startswith("_"):
            continue
        merged = dict(stages)
        merged.update(res.get(target, {}))
        res[target] = merged
    res["_source"] = ("rocprofv3 --pmc passes of tools/pmc_refresh.sh (FETCH_SIZE; WRITE_SIZE; "
                      "SQ waves/waits/MFMA busy + GRBM_GUI_ACTIVE; SQ instruction mix + LDS "
                      "conflicts), one pass each, folded by tools/pmc_fold.py; FETCH_SIZE x2, "
                      "KiB -> bytes")
    json.dump(res, open(dst, "w"), indent=1)
    for target, stages in res.items():
        if target.startswith("_"):
            continue
        for stage, rec in stages.items():
            for k in rec["kernels"]:
                print(f"{target:4s} {stage:18s} {k['symbol'][:58]:58s} "
                      f"hbm {k.get('hbm_bytes', float('nan')) / 1e6:9.1f} MB  "
                      f"mfma {k.get('mfma_busy', float('nan')):.3f}  "
                      f"wait {k.get('wait_frac', float('nan')):.2f}  "
                      f"ldsc {k.get('lds_bank_conflict_frac', float('nan')):.2f}")


if __name__ == "__main__":
    main()
