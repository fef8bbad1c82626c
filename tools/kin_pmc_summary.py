"""Summarise the round-1 kinematics profiling run (profiles/run_r01_kin.sh, in git history at cfe45c1): per kinematics dispatch size (envs = grid / 16), the
average kernel duration (kernel trace) and HBM traffic per launch from FETCH_SIZE (doubled: gfx950
tallies 128-B requests at 64 B, MI355X_MICROARCH.md §HBM) and WRITE_SIZE (KB units).  Writes
profiles/r01_kin_counters.json and copies the raw CSVs."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "prof_kin")
dst = os.path.join(REPO, "profiles")
K = "osc_kinematics_kernel"
# kin_bench.py order: (robot, nenv) per grid; Go2 and WaLTER share grid sizes, so dispatches are
# split by order of appearance (the script runs go2 4096, go2 65536, walter 4096, walter 65536)
ORDER = [("unitree_go2", 4096), ("unitree_go2", 65536), ("walter_sr", 4096), ("walter_sr", 65536)]
ALG = {"unitree_go2": 7592, "walter_sr": 14152}


def dispatches(path, value_key=None):
    rows = [r for r in csv.DictReader(open(path)) if K in r["Kernel_Name"]]
    seq = []   # (grid, value) in dispatch order, grouped into runs of equal grid
    for r in rows:
        v = float(r[value_key]) if value_key else (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        seq.append((int(r.get("Grid_Size") or r["Grid_Size_X"]), v))
    groups, cur = [], None
    for g, v in seq:
        if cur is None or cur[0] != g:
            cur = [g, []]
            groups.append(cur)
        cur[1].append(v)
    return groups


def main():
    trace = os.path.join(src, "kin_trace", "run_kernel_trace.csv")
    fetch = os.path.join(src, "pmc_fetch", "run_counter_collection.csv")
    write = os.path.join(src, "pmc_write", "run_counter_collection.csv")
    tg = dispatches(trace)
    fg = dispatches(fetch, "Counter_Value")
    wg = dispatches(write, "Counter_Value")
    out = {"kernel": K, "source": ["profiles/r01_kin_kernel_stats.csv",
                                   "profiles/r01_kin_pmc_fetch.csv",
                                   "profiles/r01_kin_pmc_write.csv"],
           "correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024", "runs": []}
    for (robot, nenv), t, f, w in zip(ORDER, tg, fg, wg):
        avg_ns = sum(t[1][2:]) / max(len(t[1]) - 2, 1)      # skip warm-up dispatches
        fb = 2 * sum(f[1]) / len(f[1]) * 1024
        wb = sum(w[1]) / len(w[1]) * 1024
        alg = ALG[robot] * nenv
        out["runs"].append({"robot": robot, "nenv": nenv, "avg_ms": avg_ns / 1e6,
                            "alg_bytes": alg, "hbm_read_bytes": fb, "hbm_write_bytes": wb,
                            "traffic_over_alg": (fb + wb) / alg,
                            "alg_GBs": alg / avg_ns, "frac_of_8TBs": alg / avg_ns / 8000})
    with open(os.path.join(dst, "r01_kin_counters.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    shutil.copy(os.path.join(src, "kin_trace", "run_kernel_stats.csv"),
                os.path.join(dst, "r01_kin_kernel_stats.csv"))
    shutil.copy(fetch, os.path.join(dst, "r01_kin_pmc_fetch.csv"))
    shutil.copy(write, os.path.join(dst, "r01_kin_pmc_write.csv"))
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, "r01_go2_4096_front_end_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
