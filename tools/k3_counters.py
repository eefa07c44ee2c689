#!/usr/bin/env python3
"""Reduce the rocprofv3 CSVs of tools/gpujobs/r02b.sh (tools/prof_k3.py under
--kernel-trace and separate --pmc passes) to per-kernel means: K1
(k_quantize_pack<256,true,false,...>, local exponents) vs K3
(k_quantize_pack<256,true,true,...>, global exponents).  Writes
profiles/<tag>/k1_vs_k3_counters.json."""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"K1": "k_quantize_pack<256, true, false,", "K3": "k_quantize_pack<256, true, true,"}


def kname(name):
    for k, pat in KEYS.items():
        if pat in name:
            return k
    return None


def main(src, dst, full_grid=16384 * 256):
    out = {"source": os.path.relpath(src, ROOT), "kernels": {}}
    tr = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv"))))
    durs = defaultdict(list)
    for r in tr:
        k = kname(r["Kernel_Name"])
        if k and int(r.get("Grid_Size") or r["Grid_Size_X"]) == full_grid:
            durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    vals = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "pmc_counter_collection.csv")
        if not sub.startswith("pmc_") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k and int(r["Grid_Size"]) == full_grid:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                vals[k]["VGPR_Count"].append(float(r["VGPR_Count"]))
                vals[k]["SGPR_Count"].append(float(r["SGPR_Count"]))
    for k in KEYS:
        d = durs.get(k, [])
        e = {"launches_traced": len(d), "avg_duration_ns": statistics.mean(d) if d else None,
             "median_duration_ns": statistics.median(d) if d else None}
        for c, v in sorted(vals[k].items()):
            e[c] = statistics.median(v)
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes (2 x FETCH_SIZE x 1024)"] = 2 * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes (WRITE_SIZE x 1024)"] = 1024 * e["WRITE_SIZE"]
        if "SQ_WAVE_CYCLES" in e and e["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in e:
                    e[c + "_frac_of_wave_cycles"] = e[c] / e["SQ_WAVE_CYCLES"]
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            e["tcc_hit_rate"] = e["TCC_HIT_sum"] / max(1.0, e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        if "GRBM_GUI_ACTIVE" in e and d:
            e["effective_clock_GHz (GRBM_GUI_ACTIVE / 8 / duration)"] = e["GRBM_GUI_ACTIVE"] / 8 / statistics.mean(d)
        out["kernels"][k] = e
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "k1_vs_k3_counters.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r02b"),
         sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r02"))
