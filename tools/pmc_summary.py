"""Summarise rocprofv3 outputs of the round-1 profiling run (profiles/run_r01.sh, in git history at cfe45c1): per-kernel average duration (kernel
trace) and per-dispatch PMC counters, HBM traffic per solve launch (gfx950 FETCH_SIZE doubled,
MI355X_MICROARCH.md §HBM) and executed FP64 work.  Writes profiles/pmc_traffic.json and
profiles/<prefix>_counters.json; copies the raw CSVs next to them."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "prof")
prefix = sys.argv[2] if len(sys.argv) > 2 else "r01_go2_4096"
nenv = int(sys.argv[3]) if len(sys.argv) > 3 else 4096   # Go2 envs per launch of the profiled run
# "cache" (bench.py's headline: the same batch every step) or "hbm" (bench.py --hbm-only: the batch
# rotated through > 256 MB of buffers, roofline.hbm_inputs)
inputs = sys.argv[4] if len(sys.argv) > 4 else "cache"
dst = os.path.join(REPO, "profiles", os.environ.get("OSC_PROFILE_SUBDIR", ""))


def short(name):
    for k in ("osc_setup_kernel", "osc_ipm_kernel"):
        if k in name:
            return k
    return None


def find(sub, pat):
    f = glob.glob(os.path.join(src, sub, "**", pat), recursive=True)
    return f[0] if f else None


out = {"prefix": prefix, "kernels": {}}
stats = find("trace", "*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(dst, f"{prefix}_kernel_stats.csv"))
    for row in csv.DictReader(open(stats)):
        k = short(row["Name"])
        if k:
            out["kernels"].setdefault(k, {})["avg_ns"] = float(row["AverageNs"])
            out["kernels"][k]["calls"] = int(row["Calls"])
counters = defaultdict(lambda: defaultdict(list))
for sub in ("pmc_fetch", "pmc_write", "pmc_inst", "pmc_cyc"):
    f = find(sub, "*counter_collection.csv")
    if not f:
        continue
    shutil.copy(f, os.path.join(dst, f"{prefix}_{sub}.csv"))
    for row in csv.DictReader(open(f)):
        k = short(row["Kernel_Name"])
        if k:
            counters[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in counters.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    out["kernels"].setdefault(k, {})["pmc_per_dispatch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["kernels"][k]["hbm_bytes"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
    if "SQ_INSTS_VALU_FMA_F64" in avg:
        f64 = (2 * avg["SQ_INSTS_VALU_FMA_F64"] + avg.get("SQ_INSTS_VALU_MUL_F64", 0) +
               avg.get("SQ_INSTS_VALU_ADD_F64", 0)) * 64
        out["kernels"][k]["executed_fp64_flop"] = f64
        ns = out["kernels"][k].get("avg_ns")
        if ns:
            out["kernels"][k]["executed_fp64_tflops"] = f64 / ns / 1e3
            out["kernels"][k]["fp64_peak_frac"] = f64 / ns / 1e3 / 78.6
    if "SQ_INSTS_VALU" in avg and "SQ_INSTS_VALU_FMA_F64" in avg:
        out["kernels"][k]["fp64_fma_share_of_valu"] = avg["SQ_INSTS_VALU_FMA_F64"] / avg["SQ_INSTS_VALU"]
json.dump(out, open(os.path.join(dst, f"{prefix}_counters.json"), "w"), indent=1)
hb = [v.get("hbm_bytes") for v in out["kernels"].values()]
if hb and all(h is not None for h in hb):
    # pmc_traffic.json is what bench.py's default (4,096-env) line reads; other sizes beside it
    tname = "pmc_traffic.json" if nenv == 4096 else f"pmc_traffic_{nenv}.json"
    if inputs == "hbm":
        tname = "pmc_traffic_hbm.json"
    json.dump({"robot": "unitree_go2", "nenv": nenv, "inputs": inputs, "bytes_per_launch": sum(hb),
               "per_kernel": {k: v.get("hbm_bytes") for k, v in out["kernels"].items()},
               "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per kernel (gfx950 "
                             "FETCH_SIZE halving for 16 B/lane reads; 8 B/lane reads uncalibrated)",
               "algorithmic_bytes_per_launch": 7664 * nenv,
               "source": [os.path.relpath(os.path.join(dst, f"{prefix}_pmc_{k}.csv"), REPO)
                          for k in ("fetch", "write")]},
              open(os.path.join(REPO, "profiles", tname), "w"), indent=1)
print(json.dumps(out, indent=1))
