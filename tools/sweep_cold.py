#!/usr/bin/env python3
"""K1 launch-shape sweep on COLD HBM: the steps cycle 4 distinct 256 MiB
buckets + planes (2 GiB, past the 256 MiB Infinity Cache), so the shape
that wins on the resident bucket (round 1's sweeps) is re-checked where the
stream really comes from HBM.  Knobs: XCD run length, tiles per wave,
workgroup cap (grid-stride).  Interleaved rounds, medians."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(N=64 << 20, P=256, nbuf=4, rounds=7, reps=40):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    B = sw.num_blocks(N, P)
    xs = [torch.randn(N, device=dev, generator=g) for _ in range(nbuf)]
    pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
    exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
    st = torch.cuda.current_stream()
    arms = [("xcd64 tpw1", 64, 1, 0), ("xcd0 tpw1", 0, 1, 0), ("xcd32 tpw1", 32, 1, 0), ("xcd128 tpw1", 128, 1, 0),
            ("xcd256 tpw1", 256, 1, 0), ("xcd64 tpw2", 64, 2, 0), ("xcd64 grid8192", 64, 1, 8192),
            ("xcd64 grid4096", 64, 1, 4096), ("xcd64 grid2048", 64, 1, 2048)]
    times = {a[0]: [] for a in arms}
    i = [0]

    def step():
        k = i[0]
        i[0] = (k + 1) % nbuf
        sw.quantize_pack(xs[k], P, 1, payload=pls[k], exps_out=exs[k], stream=st)

    for _ in range(50):
        step()
    for _ in range(rounds):
        for name, xcd, tpw, grid in arms:
            sw.set_xcd_chunk(xcd)
            sw.set_tiles_per_wave(tpw)
            sw.set_grid_limit(grid)
            for _ in range(8):
                step()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                step()
            b.record(st)
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / reps * 1e3)
    sw.set_xcd_chunk(64)
    sw.set_tiles_per_wave(1)
    sw.set_grid_limit(0)
    alg = 8 * N + B
    out = {k: {"median_us": round(statistics.median(v), 2), "GBps": round(alg / statistics.median(v) / 1e3, 1)}
           for k, v in times.items()}
    print(json.dumps({"what": "K1, 4 cold 256 MiB buckets cycled, P=256, W=1", "res": out}, indent=1))


if __name__ == "__main__":
    main()
