"""Summarise the round-4 variant PMC run (profiles/run_r04n.sh, in git history at cfe45c1): per interior-point kernel VARIANT (one-wave `<D, true, ...>` vs
two-wave `<D, false, ...>`, told apart by the template arguments of the kernel name), its average
duration (kernel trace) and per-dispatch PMC counters -- HBM bytes (gfx950: 2 x FETCH_SIZE +
WRITE_SIZE, KiB; MI355X_MICROARCH.md), the SQ cycle / wait / issue counters and the instruction
mix.  Writes profiles/<prefix>_<nenv>.json.

    python tools/pmc_ab_summary.py gpurun_out/r04n r04n_ab_onewave_twowave
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, prefix = sys.argv[1], sys.argv[2]


def variant(name):
    if "osc_setup_kernel" in name:
        return "setup"
    if "osc_ipm_kernel" not in name:
        return None
    args = name.split("osc_ipm_kernel<", 1)[1]
    return "ipm_one_wave" if ", true, " in args.split(">", 1)[1][:12] else "ipm_two_wave"


for nd in sorted(glob.glob(os.path.join(src, "*"))):
    if not os.path.isdir(nd):
        continue
    nenv = int(os.path.basename(nd))
    out = {"nenv": nenv, "algorithmic_bytes_per_launch": 7664 * nenv, "kernels": {}}
    f = glob.glob(os.path.join(nd, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if f:
        for row in csv.DictReader(open(f[0])):
            v = variant(row["Name"])
            if v:
                out["kernels"].setdefault(v, {})["avg_us"] = float(row["AverageNs"]) / 1e3
                out["kernels"][v]["calls"] = int(row["Calls"])
    acc = defaultdict(lambda: defaultdict(list))
    for sub in ("pmc_fetch", "pmc_write", "pmc_inst", "pmc_cyc"):
        for f in glob.glob(os.path.join(nd, sub, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                v = variant(row["Kernel_Name"])
                if v:
                    acc[v][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for v, cs in acc.items():
        avg = {c: sum(x) / len(x) for c, x in cs.items()}
        k = out["kernels"].setdefault(v, {})
        k["pmc_per_dispatch"] = avg
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            k["hbm_bytes"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            k["hbm_x_algorithmic"] = k["hbm_bytes"] / out["algorithmic_bytes_per_launch"]
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY"):
                if c in avg:
                    k[c + "_share"] = avg[c] / wc
    json.dump(out, open(os.path.join(REPO, "profiles", f"{prefix}_{nenv}.json"), "w"), indent=1)
    print(json.dumps({v: {kk: (round(x, 4) if isinstance(x, float) else x) for kk, x in d.items()
                          if kk != "pmc_per_dispatch"} for v, d in out["kernels"].items()}))
