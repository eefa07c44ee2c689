#!/usr/bin/env python3
"""K1 launch geometry on cold HBM at the N = 8 / 4 / 2 slice sizes of
configs[3] (128 / 256 / 512 MiB; 4 buckets + planes cycled per size): the
one-shot grid against grid-stride caps (sml_set_grid_limit) and XCD run
lengths (sml_set_xcd_chunk; 0 = plain block order), on the final kernels
(2-slice tiles, sc1 nt payload stores).  Interleaved rounds, medians; every
arm's planes equal the first arm's."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402

ARMS = [("one-shot xcd64", 0, 64), ("one-shot xcd32", 0, 32), ("one-shot xcd128", 0, 128),
        ("one-shot plain", 0, 0), ("cap2048 xcd64", 2048, 64), ("cap4096 xcd64", 4096, 64),
        ("cap8192 xcd64", 8192, 64)]


def main(rounds=7, nbuf=4, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    out = {}
    for mib in (128, 256, 512):
        N = mib << 18
        B = sw.num_blocks(N, P)
        xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
        pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
        i = [0]

        def k1():
            k = i[0] % nbuf
            i[0] += 1
            sw.quantize_pack(xs[k], P, 1, payload=pls[k], exps_out=exs[k], stream=st)
        ref = None
        for name, cap, xcd in ARMS:
            sw.set_grid_limit(cap)
            sw.set_xcd_chunk(xcd)
            sw.quantize_pack(xs[0], P, 1, payload=pls[0], exps_out=exs[0], stream=st)
            torch.cuda.synchronize()
            cur = (pls[0].clone(), exs[0].clone())
            if ref is None:
                ref = cur
            assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), name
        del ref, cur
        reps = max(10, int(30 * 256 / mib))
        t = {a[0]: [] for a in ARMS}
        for _ in range(30):
            k1()
        for _ in range(rounds):
            for name, cap, xcd in ARMS:
                sw.set_grid_limit(cap)
                sw.set_xcd_chunk(xcd)
                for _ in range(8):
                    k1()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    k1()
                b.record(st)
                torch.cuda.synchronize()
                t[name].append(a.elapsed_time(b) / reps * 1e3)
        sw.set_grid_limit(0)
        sw.set_xcd_chunk(64)
        alg = 8 * N + B
        out[f"{mib}MiB"] = {n: {"median_us": round(statistics.median(v), 2),
                                "GBps": round(alg / statistics.median(v) / 1e3, 1)} for n, v in t.items()}
        del xs, pls, exs
        torch.cuda.empty_cache()
        print(f"{mib} MiB done", file=sys.stderr, flush=True)
    print(json.dumps({"what": f"K1 grid cap x XCD run, {nbuf} cold buckets per size, {rounds} interleaved rounds, "
                      "medians", "res": out}, indent=1))


if __name__ == "__main__":
    main()
