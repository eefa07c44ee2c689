#!/usr/bin/env python3
"""Interleaved A/B of K1 (sml_quantize_pack) between library builds, on the
resident 256 MiB bucket and on cold HBM (steps cycling 4 distinct buckets +
planes, 2 GiB past the Infinity Cache).  Usage: ab_cold.py lib1.so lib2.so"""
import ctypes
import json
import statistics
import sys

import torch


def main(paths, N=64 * 1024 * 1024, P=256, nbuf=4, rounds=9, reps=40):
    dev = torch.device("cuda:0")
    B = (N + P - 1) // P
    xs = [torch.randn(N, device=dev) for _ in range(nbuf)]
    pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
    exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        libs.append(L)
    st = torch.cuda.current_stream()
    ref = None
    for p, L in zip(paths, libs):
        assert L.sml_quantize_pack(xs[0].data_ptr(), N, P, 1, None, pls[0].data_ptr(), exs[0].data_ptr(), 0, st.cuda_stream) == 0
        torch.cuda.synchronize()
        cur = (pls[0].clone(), exs[0].clone())
        ref = ref or cur
        assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), p
    res = {p: {"resident": [], "cold": []} for p in paths}
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            for kind, nb in (("resident", 1), ("cold", nbuf)):
                for i in range(10):
                    k = i % nb
                    L.sml_quantize_pack(xs[k].data_ptr(), N, P, 1, None, pls[k].data_ptr(), exs[k].data_ptr(), 0, st.cuda_stream)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for i in range(reps):
                    k = i % nb
                    L.sml_quantize_pack(xs[k].data_ptr(), N, P, 1, None, pls[k].data_ptr(), exs[k].data_ptr(), 0, st.cuda_stream)
                b.record(st)
                torch.cuda.synchronize()
                res[p][kind].append(a.elapsed_time(b) / reps * 1e3)
    alg = 8 * N + B
    print(json.dumps({p: {k: {"median_us": round(statistics.median(v), 2), "TBps": round(alg / statistics.median(v) / 1e6, 3)}
                          for k, v in r.items()} for p, r in res.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
