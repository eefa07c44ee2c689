#!/usr/bin/env python3
"""A/B of K1's wave-tile size now that every tile size takes the same
non-temporal payload stores (round 4): 4-slice (1024-element) vs 2-slice
(512-element) tiles, XCD run lengths, on the bench's own workload —
bench_bucket gradient-like data, the steps cycling 4 distinct buckets +
planes — at the per-GPU slice sizes of the N = 8 / 4 / 2 / 1 (configs[3])
points and the headline's 256 MiB bucket; plus K3 / K2 at 256 MiB.
Interleaved rounds, medians; every arm's planes checked equal.
AB_KIND=stream: the same for K4 (dequantize) and the fused round trip
(sml_set_stream_tile_slices), outputs checked equal."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402
import bench  # noqa: E402


def main(rounds=9, nbuf=4):
    P = 256
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    sizes = [int(s) for s in os.environ.get("AB_SIZES_MIB", "128,256,512,1024").split(",")]
    arms = [("slices4 xcd64", 4, 64), ("slices2 xcd64", 2, 64), ("slices2 xcd32", 2, 32), ("slices2 xcd128", 2, 128)]
    res = {}
    for mib in sizes:
        N = mib << 18
        B = sw.num_blocks(N, P)
        xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
        pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
        kinds = ["K1"] + (["K3", "K2"] if mib == 256 else [])
        ref = None
        for name, sl, xcd in arms:
            sw.set_quantize_tile_slices(sl)
            sw.set_xcd_chunk(xcd)
            sw.quantize_pack(xs[0], P, 1, payload=pls[0], exps_out=exs[0], stream=st)
            torch.cuda.synchronize()
            cur = (pls[0].clone(), exs[0].clone())
            if ref is None:
                ref = cur
            assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), (mib, name)
        del ref, cur
        i = [0]

        def step(kind):
            k = i[0] % nbuf
            i[0] += 1
            if kind == "K1":
                sw.quantize_pack(xs[k], P, 1, payload=pls[k], exps_out=exs[k], stream=st)
            elif kind == "K3":
                sw.quantize_pack(xs[k], P, 2, global_exps=exs[k], payload=pls[k], stream=st)
            else:
                sw.exponents(xs[k], P, out=exs[k], stream=st)

        t = {(a[0], k): [] for a in arms for k in kinds}
        for _ in range(30):
            step("K1")
        reps = max(8, int(40 * 256 / mib))
        for _ in range(rounds):
            for name, sl, xcd in arms:
                sw.set_quantize_tile_slices(sl)
                sw.set_xcd_chunk(xcd)
                for kind in kinds:
                    for _ in range(8):
                        step(kind)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for _ in range(reps):
                        step(kind)
                    b.record(st)
                    torch.cuda.synchronize()
                    t[(name, kind)].append(a.elapsed_time(b) / reps * 1e3)
        alg = {"K1": 8 * N + B, "K3": 8 * N + B, "K2": 4 * N + B}
        for (name, kind), v in t.items():
            m = statistics.median(v)
            res.setdefault(f"{mib}MiB {kind}", {})[name] = {"median_us": round(m, 2),
                                                             "GBps": round(alg[kind] / m / 1e3, 1)}
        del xs, pls, exs
        torch.cuda.empty_cache()
    sw.set_quantize_tile_slices(0)
    sw.set_xcd_chunk(64)
    print(json.dumps({"what": "K1 (K3, K2 at 256 MiB) tile slices x XCD run, nt payload stores, bench_bucket data, "
                      f"{nbuf} buckets cycled, {rounds} interleaved rounds, medians", "res": res}, indent=1))


def main_stream(rounds=9, nbuf=4):
    P, W = 256, 1
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    sizes = [int(s) for s in os.environ.get("AB_SIZES_MIB", "128,256,512").split(",")]
    arms = [("slices4 xcd64", 4, 64), ("slices2 xcd64", 2, 64), ("slices2 xcd128", 2, 128)]
    res = {}
    for mib in sizes:
        N = mib << 18
        B = sw.num_blocks(N, P)
        xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
        pls, exs = [], []
        for x in xs:
            q, e = sw.quantize_pack(x, P, W)
            pls.append(q)
            exs.append(e)
        outs = [torch.empty(N, device=dev) for _ in range(nbuf)]
        ref = None
        for name, sl, xcd in arms:
            sw.set_stream_tile_slices(sl)
            sw.set_xcd_chunk(xcd)
            sw.dequantize(pls[0], exs[0], N, P, W, out=outs[0], stream=st)
            a = outs[0].clone()
            sw.roundtrip_loopback(xs[0], P, W, out=outs[0], stream=st)
            torch.cuda.synchronize()
            cur = (a, outs[0].clone())
            if ref is None:
                ref = cur
            assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), (mib, name)
            assert torch.equal(cur[0], cur[1]), (mib, name)
        del ref, cur, a
        i = [0]

        def step(kind):
            k = i[0] % nbuf
            i[0] += 1
            if kind == "K4":
                sw.dequantize(pls[k], exs[k], N, P, W, out=outs[k], stream=st)
            else:
                sw.roundtrip_loopback(xs[k], P, W, out=outs[k], stream=st)

        kinds = ("K4", "roundtrip")
        t = {(a_[0], k): [] for a_ in arms for k in kinds}
        reps = max(8, int(40 * 256 / mib))
        for _ in range(20):
            step("K4")
        for _ in range(rounds):
            for name, sl, xcd in arms:
                sw.set_stream_tile_slices(sl)
                sw.set_xcd_chunk(xcd)
                for kind in kinds:
                    for _ in range(8):
                        step(kind)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        step(kind)
                    e1.record(st)
                    torch.cuda.synchronize()
                    t[(name, kind)].append(e0.elapsed_time(e1) / reps * 1e3)
        alg = {"K4": 8 * N + B, "roundtrip": 8 * N}
        for (name, kind), v in t.items():
            m = statistics.median(v)
            res.setdefault(f"{mib}MiB {kind}", {})[name] = {"median_us": round(m, 2),
                                                             "GBps": round(alg[kind] / m / 1e3, 1)}
        del xs, pls, exs, outs
        torch.cuda.empty_cache()
    sw.set_stream_tile_slices(0)
    sw.set_xcd_chunk(64)
    print(json.dumps({"what": "K4 / fused round trip tile slices x XCD run, nt output stores, bench_bucket data, "
                      f"{nbuf} buckets cycled, {rounds} interleaved rounds, medians", "res": res}, indent=1))


if __name__ == "__main__":
    if os.environ.get("AB_KIND") == "stream":
        main_stream()
    else:
        main()
