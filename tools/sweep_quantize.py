#!/usr/bin/env python3
"""Interleaved A/B sweep of launch geometry (grid cap, tiles per wave) for the bench
kernel (sml_quantize_pack, K1) on one GPU: every variant is timed in each
round, rounds repeat, medians reported (cdna_hip_programming.md §5.4 rule 24).
Also times a torch device copy of the same bytes as a practical ceiling."""
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main():
    N = int(os.environ.get("SWEEP_NUMEL", 64 * 1024 * 1024))
    P = int(os.environ.get("SWEEP_P", 256))
    rounds = int(os.environ.get("SWEEP_ROUNDS", 7))
    W = int(os.environ.get("SWEEP_W", 1))
    reps = 10
    dev = torch.device("cuda:0")
    x = torch.randn(N, device=dev)
    B = sw.num_blocks(N, P)
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    exps = torch.empty(B, dtype=torch.int8, device=dev)
    out = torch.empty_like(x)
    st = torch.cuda.current_stream()
    alg = 8 * N + B
    grids = [int(g) for g in os.environ.get("SWEEP_GRIDS", "0,4096,8192").split(",")]
    tpws = [int(t) for t in os.environ.get("SWEEP_TPW", "4,1").split(",")]
    variants = list(itertools.product(grids, tpws))
    res = {v: [] for v in variants}
    copy, ntcopy = [], []

    def t_of(fn):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e-3

    for _ in range(rounds):
        for g, tpw in variants:
            sw.set_grid_limit(g)
            sw.set_quantize_tile_slices(tpw)
            res[(g, tpw)].append(t_of(lambda: sw.quantize_pack(x, P, W, payload=payload, exps_out=exps, stream=st)))
        sw.set_grid_limit(0)
        sw.set_quantize_tile_slices(0)
        copy.append(t_of(lambda: out.copy_(x)))
        ntcopy.append(t_of(lambda: sw.stream_copy(x, out, stream=st)))
    rows = []
    for (g, tpw), ts in res.items():
        m = statistics.median(ts)
        rows.append({"grid_limit": g, "tile_slices": tpw, "median_us": round(m * 1e6, 2),
                     "min_us": round(min(ts) * 1e6, 2), "GBps": round(alg / m / 1e9, 1)})
    rows.sort(key=lambda r: r["median_us"])
    cm, nm = statistics.median(copy), statistics.median(ntcopy)
    print(json.dumps({"numel": N, "P": P, "W": W, "torch_copy_us": round(cm * 1e6, 2),
                      "torch_copy_GBps": round(8 * N / cm / 1e9, 1), "nt_tile_copy_us": round(nm * 1e6, 2),
                      "nt_tile_copy_GBps": round(8 * N / nm / 1e9, 1), "variants": rows}, indent=1))


if __name__ == "__main__":
    main()
