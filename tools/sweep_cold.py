#!/usr/bin/env python3
"""K1 / K3 / K2 launch-shape sweep, resident and on COLD HBM.  Resident: one
256 MiB bucket re-read every step (the bench headline).  Cold: the steps
cycle 4 distinct 256 MiB buckets + planes (2 GiB, past the 256 MiB Infinity
Cache).  1 GiB: one configs[3]-sized job.  Knobs: slices per wave tile
(sml_set_quantize_tile_slices: 4 = round-1/2 tiles of 1024 elements, 1 =
256-element tiles) and XCD run length (sml_set_xcd_chunk, runs of C x 16 KiB
of input whatever the tile).  Interleaved rounds, medians; every arm's
planes are checked equal to the first arm's."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(N=64 << 20, nbuf=4, rounds=7, reps=30):
    P = int(os.environ.get("SWEEP_P", "256"))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    B = sw.num_blocks(N, P)
    xs = [torch.randn(N, device=dev, generator=g) for _ in range(nbuf)]
    pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
    exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
    NB = 4 * N
    xb = torch.randn(NB, device=dev, generator=g)
    BB = sw.num_blocks(NB, P)
    pb = torch.empty(BB * P, dtype=torch.int32, device=dev)
    eb = torch.empty(BB, dtype=torch.int8, device=dev)
    st = torch.cuda.current_stream()
    arms = [("slices4 xcd64", 4, 64), ("slices1 xcd64", 1, 64), ("slices2 xcd64", 2, 64),
            ("slices1 xcd32", 1, 32), ("slices1 xcd128", 1, 128)]
    kinds = ("K1 resident", "K1 cold", "K1 1GiB", "K3 cold", "K2 cold")
    times = {(a[0], k): [] for a in arms for k in kinds}
    i = [0]

    def k1(nb):
        k = i[0] % nb
        i[0] += 1
        sw.quantize_pack(xs[k], P, 1, payload=pls[k], exps_out=exs[k], stream=st)

    def k3(nb):
        k = i[0] % nb
        i[0] += 1
        sw.quantize_pack(xs[k], P, 2, global_exps=exs[k], payload=pls[k], stream=st)

    def k2(nb):
        k = i[0] % nb
        i[0] += 1
        sw.exponents(xs[k], P, out=exs[k], stream=st)

    def big(_):
        sw.quantize_pack(xb, P, 1, payload=pb, exps_out=eb, stream=st)

    fns = {"K1 resident": (k1, 1), "K1 cold": (k1, nbuf), "K1 1GiB": (big, 1), "K3 cold": (k3, nbuf),
           "K2 cold": (k2, nbuf)}
    ref = None
    for name, sl, xcd in arms:                       # equal planes for every shape
        sw.set_quantize_tile_slices(sl)
        sw.set_xcd_chunk(xcd)
        sw.quantize_pack(xs[0], P, 3, payload=pls[0], exps_out=exs[0], stream=st)
        torch.cuda.synchronize()
        cur = (pls[0].clone(), exs[0].clone())
        if ref is None:
            ref = cur
        assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), name
    for _ in range(50):
        k1(nbuf)
    for _ in range(rounds):
        for name, sl, xcd in arms:
            sw.set_quantize_tile_slices(sl)
            sw.set_xcd_chunk(xcd)
            for kind in kinds:
                fn, nb = fns[kind]
                r = reps if kind != "K1 1GiB" else max(4, reps // 4)
                for _ in range(6):
                    fn(nb)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(r):
                    fn(nb)
                b.record(st)
                torch.cuda.synchronize()
                times[(name, kind)].append(a.elapsed_time(b) / r * 1e3)
    sw.set_xcd_chunk(64)
    sw.set_quantize_tile_slices(0)
    alg = {"K1 resident": 8 * N + B, "K1 cold": 8 * N + B, "K1 1GiB": 8 * NB + BB, "K3 cold": 8 * N + B,
           "K2 cold": 4 * N + B}
    out = {}
    for (name, kind), v in times.items():
        m = statistics.median(v)
        out.setdefault(name, {})[kind] = {"median_us": round(m, 2), "GBps": round(alg[kind] / m / 1e3, 1)}
    print(json.dumps({"what": f"K1/K3/K2 tile slices x XCD run length, P={P}: resident 256 MiB, cold "
                      "(4 x 256 MiB cycled), one 1 GiB job", "res": out}, indent=1))


if __name__ == "__main__":
    main()
