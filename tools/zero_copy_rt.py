#!/usr/bin/env python3
"""Zero-copy (PCIe) rates of K1 and the fused round trip on pinned host
buffers, by bucket size and grid cap: fp32 GB/s each way (4N / t)."""
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


def main(P=256, W=8, reps=4, rounds=3):
    st = torch.cuda.current_stream()
    res = {}
    for N in (6_553_600, 64 * 1024 * 1024):
        hx = torch.randn(N).pin_memory()
        ho = torch.empty(N).pin_memory()
        B = sw.num_blocks(N, P)
        hp = torch.empty(B * P, dtype=torch.int32).pin_memory()
        he = torch.empty(B, dtype=torch.int8).pin_memory()
        fns = {"k1": lambda: sw.quantize_pack(hx, P, W, payload=hp, exps_out=he, stream=st),
               "roundtrip": lambda: sw.roundtrip_loopback(hx, P, W, out=ho, stream=st)}
        for _ in range(rounds):
            for (name, fn), g in itertools.product(fns.items(), [0, 256, 512, 1024, 2048]):
                sw.set_grid_limit(g)
                fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                torch.cuda.synchronize()
                res.setdefault(f"N{N}_{name}_grid{g}", []).append(4 * N * reps / (time.perf_counter() - t0) / 1e9)
        sw.set_grid_limit(0)
    print(json.dumps({k: round(statistics.median(v), 2) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
