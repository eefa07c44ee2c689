#!/usr/bin/env python3
"""Summarise a profiles/run_profiles.sh run into committed evidence.

Reads gpurun_out/prof_<tag>/{kt,pmc_fetch,pmc_write} (rocprofv3 CSV) and writes
  profiles/<tag>/kernel_stats.csv     (rocprofv3 --kernel-trace --stats summary, sml kernels)
  profiles/<tag>/summary.json         (per-kernel avg duration, PMC bytes per launch)
  profiles/pmc_traffic.json           (what bench.py reports as roofline.traffic)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM / rocprofv3:
  FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (TCC slots);
  both are in KiB (x 1024); on gfx950 FETCH_SIZE reads exactly half of the
  bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
  WRITE_SIZE is exact for 16 B/lane streaming stores.
Only launches of the full bench workload (grid = the bench's grid) are used.
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(tag="r02", numel=64 * 1024 * 1024, packet_numel=256, timed_steps=2000):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)

    stats = rows(os.path.join(src, "kt", "kt_kernel_stats.csv"))
    trace = rows(os.path.join(src, "kt", "kt_kernel_trace.csv"))
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
        w.writeheader()
        for r in stats:
            if "sml::" in r["Name"] or "copyBuffer" in r["Name"]:
                w.writerow(r)

    # the headline's launches: the grid of the 256 MiB bucket (the most
    # launches: 2000 timed + warmup); other grids (the strong_1GiB reading's
    # 1 GiB job, 200 timed launches) are summarised apart in per_grid
    q = [r for r in trace if "k_quantize_pack" in r["Kernel_Name"]]
    gsz = lambda r: int(r.get("Grid_Size") or r["Grid_Size_X"])
    by_grid = {}
    for r in q:
        by_grid.setdefault(gsz(r), []).append(r)
    grid = max(by_grid, key=lambda g: len(by_grid[g]))
    per_grid = []
    for g, rs in sorted(by_grid.items()):
        rs = sorted(rs, key=lambda r: int(r["Start_Timestamp"]))
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs]
        per_grid.append({"grid_threads": g, "launches": len(d), "avg_duration_ns": statistics.mean(d),
                         "last_200_avg_duration_ns": statistics.mean(d[-200:])})
    full = by_grid[grid]
    full.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in full]
    timed = durs[-timed_steps:]   # the bench's timed window (the last K full-grid launches)

    def pmc(sub, counter):
        rr = rows(os.path.join(src, sub, "pmc_counter_collection.csv"))
        vals = [float(r["Counter_Value"]) for r in rr
                if "k_quantize_pack" in r["Kernel_Name"] and int(r["Grid_Size"]) == grid
                and r["Counter_Name"] == counter]
        return vals

    fetch = pmc("pmc_fetch", "FETCH_SIZE")
    write = pmc("pmc_write", "WRITE_SIZE")
    # round 3+: the default passes cycle 4 buckets (cold HBM) and res_* re-read
    # one bucket; round 2 had the default resident and cold_* cycling
    cycling = os.path.isdir(os.path.join(src, "res_fetch"))
    other = ("res_fetch", "res_write") if cycling else ("cold_fetch", "cold_write")
    other_b = None
    if os.path.isdir(os.path.join(src, other[0])) and os.path.isdir(os.path.join(src, other[1])):
        cf, cw = pmc(other[0], "FETCH_SIZE"), pmc(other[1], "WRITE_SIZE")
        if cf and cw:
            other_b = 2 * 1024 * statistics.mean(cf) + 1024 * statistics.mean(cw)
    B = -(-numel // packet_numel)
    alg_read, alg_write = 4 * numel, 4 * numel + B
    fetch_b = 2 * 1024 * statistics.mean(fetch)
    write_b = 1024 * statistics.mean(write)
    summary = {
        "tag": tag,
        "kernel": full[0]["Kernel_Name"],
        "grid_threads": grid,
        "launches": len(full),
        "avg_duration_ns": statistics.mean(durs),
        "median_duration_ns": statistics.median(durs),
        "timed_window_launches": len(timed),
        "timed_window_avg_duration_ns": statistics.mean(timed),
        "algorithmic_GBps_at_timed_window_avg": (alg_read + alg_write) / statistics.mean(timed),
        "algorithmic_bytes_per_launch": alg_read + alg_write,
        "algorithmic_GBps_at_avg": (alg_read + alg_write) / statistics.mean(durs),
        "pmc_fetch_size_kib_mean": statistics.mean(fetch),
        "pmc_write_size_kib_mean": statistics.mean(write),
        "hbm_read_bytes_per_launch (2 x FETCH_SIZE x 1024)": fetch_b,
        "hbm_write_bytes_per_launch (WRITE_SIZE x 1024)": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "traffic_over_algorithmic": (fetch_b + write_b) / (alg_read + alg_write),
        "default_steps": "4 distinct buckets cycled (cold HBM)" if cycling else "one resident bucket",
        "per_grid": per_grid,
    }
    key = "resident" if cycling else "cold"
    summary[f"{key}_hbm_bytes_per_launch"] = other_b
    summary[f"{key}_traffic_over_algorithmic"] = None if other_b is None else other_b / (alg_read + alg_write)
    if os.path.isdir(os.path.join(src, "fr_kt")):
        summary["frames"] = frames_summary(src, dst, numel, packet_numel)
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    main_key, other_key = ("quantize_pack_cold", "quantize_pack") if cycling else ("quantize_pack", "quantize_pack_cold")
    traffic = {"source": f"profiles/{tag}/summary.json",
               main_key: {"numel": numel, "packet_numel": packet_numel,
                          "hbm_bytes_per_launch": round(fetch_b + write_b)}}
    if other_b is not None:
        traffic[other_key] = {"numel": numel, "packet_numel": packet_numel, "hbm_bytes_per_launch": round(other_b)}
    slices = slice_traffic(src, packet_numel)
    if slices:
        traffic["quantize_pack_cold_slices"] = slices
        summary["slice_traffic"] = slices
        with open(os.path.join(dst, "summary.json"), "w") as f:
            json.dump(summary, f, indent=1)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(summary, indent=1))


def slice_traffic(src, packet_numel):
    """K1's HBM bytes per launch at configs[3]'s per-GPU FIFO slice sizes
    (run_profiles.sh: slice_<numel>_{fetch,write}, 4 buckets cycled), for the
    strong_1GiB reading's roofline.traffic at N = 1, 2 and 8."""
    out = []
    for d in sorted(os.listdir(src)) if os.path.isdir(src) else []:
        if not (d.startswith("slice_") and d.endswith("_fetch")):
            continue
        numel = int(d.split("_")[1])
        wdir = os.path.join(src, f"slice_{numel}_write")
        if not os.path.isdir(wdir):
            continue

        def vals(sub, counter):
            rr = rows(os.path.join(src, sub, "pmc_counter_collection.csv"))
            q = [r for r in rr if "k_quantize_pack" in r["Kernel_Name"] and r["Counter_Name"] == counter]
            if not q:
                return []
            grid = max(int(r["Grid_Size"]) for r in q)
            return [float(r["Counter_Value"]) for r in q if int(r["Grid_Size"]) == grid]

        f, w = vals(d, "FETCH_SIZE"), vals(f"slice_{numel}_write", "WRITE_SIZE")
        if not f or not w:
            continue
        B = -(-numel // packet_numel)
        hbm = 2 * 1024 * statistics.mean(f) + 1024 * statistics.mean(w)
        out.append({"numel": numel, "packet_numel": packet_numel, "buckets": 4,
                    "hbm_bytes_per_launch": round(hbm), "traffic_over_algorithmic": hbm / (8 * numel + B)})
    return out


def frames_summary(src, dst, numel, packet_numel, batch_max=64):
    """F3 kernels from tools/prof_frames.py: per-kernel average duration and
    PMC bytes per launch next to the algorithmic bytes (frames = B + b frames
    of 52 + 4P bytes).  FETCH_SIZE doubling applies to the wide payload reads."""
    stats = rows(os.path.join(src, "fr_kt", "kt_kernel_stats.csv"))
    with open(os.path.join(dst, "frames_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
        w.writeheader()
        for r in stats:
            if "sml::" in r["Name"]:
                w.writerow(r)
    B = -(-numel // packet_numel)
    fbytes = (B + min(B, batch_max)) * (52 + 4 * packet_numel)
    fbytes_i = B * (52 + 4 * packet_numel)   # INT32 slices: B frames, no extra batch
    alg = {"k_quantize_frames<%d, true, false, true, false>" % packet_numel: (4 * numel, fbytes),
           "k_quantize_frames<%d, true, false, true, true>" % packet_numel: (4 * numel, fbytes_i),
           "k_rx_apply": (fbytes, 4 * numel),
           "k_rx_claim": (None, None),   # k_rx_apply also retires the winners (the old commit pass)
           "k_rx_int32<": (fbytes_i, 4 * numel),
           "k_rx_int32_fixup": (None, None)}

    def pmc(sub, counter, key):
        rr = rows(os.path.join(src, sub, "pmc_counter_collection.csv"))
        v = [float(r["Counter_Value"]) * 1024 for r in rr if key in r["Kernel_Name"] and r["Counter_Name"] == counter]
        return statistics.median(v) if v else None

    out = {}
    for key, (ar, aw) in alg.items():
        st = [r for r in stats if key in r["Name"]]
        if not st:
            continue
        avg_ns = float(st[0]["AverageNs"])
        fetch, write = pmc("fr_fetch", "FETCH_SIZE", key), pmc("fr_write", "WRITE_SIZE", key)
        e = {"avg_duration_ns": avg_ns, "launches": int(st[0]["Calls"]),
             "hbm_read_bytes_per_launch (2 x FETCH_SIZE x 1024)": None if fetch is None else 2 * fetch,
             "hbm_write_bytes_per_launch (WRITE_SIZE x 1024)": write}
        if ar is not None:
            e["algorithmic_bytes_per_launch"] = ar + aw
            e["algorithmic_GBps_at_avg"] = (ar + aw) / avg_ns
        out[key] = e
    return out


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["r02"]))
