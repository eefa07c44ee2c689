#!/usr/bin/env python3
"""Zero-copy (PCIe) quantize+pack: K1 reading a pinned host bucket and writing
pinned host planes, across launch geometries (grid cap, tiles per wave)."""
import itertools
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(N=64 * 1024 * 1024, P=256, reps=3, rounds=3):
    hx = torch.randn(N).pin_memory()
    B = sw.num_blocks(N, P)
    hp = torch.empty(B * P, dtype=torch.int32).pin_memory()
    he = torch.empty(B, dtype=torch.int8).pin_memory()
    st = torch.cuda.current_stream()
    res = {}
    for _ in range(rounds):
        for g, tpw in itertools.product([0, 1024, 2048, 4096], [4, 1]):
            sw.set_grid_limit(g)
            sw.set_quantize_tile_slices(tpw)
            sw.quantize_pack(hx, P, 1, payload=hp, exps_out=he, stream=st)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                sw.quantize_pack(hx, P, 1, payload=hp, exps_out=he, stream=st)
            torch.cuda.synchronize()
            res.setdefault(f"grid{g}_slices{tpw}", []).append(4 * N * reps / (time.perf_counter() - t0) / 1e9)
    sw.set_grid_limit(0)
    sw.set_quantize_tile_slices(0)
    print(json.dumps({k: round(statistics.median(v), 2) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
