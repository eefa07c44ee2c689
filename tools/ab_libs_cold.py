#!/usr/bin/env python3
"""Interleaved A/B of K1 / K3 / K2 (sml_quantize_pack, sml_exponents) between
builds of the kernel library on the bench workload: bench_bucket data, the
steps cycling 4 distinct buckets + planes (cold HBM), at 256 and 128 MiB.
Same process, same buffers, alternating rounds, medians; every build's
planes checked equal.  Usage: ab_libs_cold.py lib1.so lib2.so ..."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402


def main(paths, rounds=9, nbuf=4, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    libs = []
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        L.sml_exponents.restype = ctypes.c_int
        L.sml_exponents.argtypes = [vp, u64, u32, vp, vp]
        L.sml_dequantize.restype = ctypes.c_int
        L.sml_dequantize.argtypes = [vp, vp, u64, u32, u16, vp, u32, vp]
        L.sml_roundtrip_loopback.restype = ctypes.c_int
        L.sml_roundtrip_loopback.argtypes = [vp, vp, u64, u32, u16, vp, vp, u32, vp]
        libs.append(L)
    res = {}
    for mib in (256, 128):
        N = mib << 18
        B = -(-N // P)
        xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
        pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nbuf)]
        outs = [torch.empty(N, device=dev) for _ in range(nbuf)]
        ref = None
        for p, L in zip(paths, libs):
            assert L.sml_quantize_pack(xs[0].data_ptr(), N, P, 1, None, pls[0].data_ptr(), exs[0].data_ptr(), 0,
                                       st.cuda_stream) == 0
            torch.cuda.synchronize()
            cur = (pls[0].clone(), exs[0].clone())
            if ref is None:
                ref = cur
            assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), p
        del ref, cur
        i = [0]

        def step(L, kind):
            k = i[0] % nbuf
            i[0] += 1
            if kind == "K1":
                L.sml_quantize_pack(xs[k].data_ptr(), N, P, 1, None, pls[k].data_ptr(), exs[k].data_ptr(), 0,
                                    st.cuda_stream)
            elif kind == "K3":
                L.sml_quantize_pack(xs[k].data_ptr(), N, P, 2, exs[k].data_ptr(), pls[k].data_ptr(), None, 0,
                                    st.cuda_stream)
            elif kind == "K2":
                L.sml_exponents(xs[k].data_ptr(), N, P, exs[k].data_ptr(), st.cuda_stream)
            elif kind == "K4":
                L.sml_dequantize(pls[k].data_ptr(), exs[k].data_ptr(), N, P, 1, outs[k].data_ptr(), 0,
                                 st.cuda_stream)
            else:
                L.sml_roundtrip_loopback(xs[k].data_ptr(), outs[k].data_ptr(), N, P, 1, None, None, 0,
                                         st.cuda_stream)

        kinds = tuple(os.environ.get("AB_KINDS", "K1,K3,K2").split(","))
        for k in range(nbuf):   # valid planes for K4
            libs[0].sml_quantize_pack(xs[k].data_ptr(), N, P, 1, None, pls[k].data_ptr(), exs[k].data_ptr(), 0,
                                      st.cuda_stream)
        if "K4" in kinds or "RT" in kinds:   # every build's K4 / round trip: the same bits
            ref = None
            for p, L in zip(paths, libs):
                L.sml_dequantize(pls[0].data_ptr(), exs[0].data_ptr(), N, P, 1, outs[0].data_ptr(), 0, st.cuda_stream)
                a4 = outs[0].clone()
                L.sml_roundtrip_loopback(xs[0].data_ptr(), outs[1].data_ptr(), N, P, 1, None, None, 0, st.cuda_stream)
                torch.cuda.synchronize()
                assert torch.equal(a4, outs[1]), p
                if ref is None:
                    ref = a4
                assert torch.equal(ref, a4), p
        t = {(p, k): [] for p in paths for k in kinds}
        reps = max(8, int(40 * 256 / mib))
        for _ in range(30):
            step(libs[0], "K1")
        for _ in range(rounds):
            for p, L in zip(paths, libs):
                for kind in kinds:
                    for _ in range(8):
                        step(L, kind)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for _ in range(reps):
                        step(L, kind)
                    b.record(st)
                    torch.cuda.synchronize()
                    t[(p, kind)].append(a.elapsed_time(b) / reps * 1e3)
        alg = {"K1": 8 * N + B, "K3": 8 * N + B, "K2": 4 * N + B, "K4": 8 * N + B, "RT": 8 * N}
        for (p, kind), v in t.items():
            m = statistics.median(v)
            res.setdefault(f"{mib}MiB {kind}", {})[os.path.basename(p)] = {
                "median_us": round(m, 2), "GBps": round(alg[kind] / m / 1e3, 1)}
        del xs, pls, exs, outs
        torch.cuda.empty_cache()
    print(json.dumps({"what": f"builds {[os.path.basename(p) for p in paths]}: K1 / K3 / K2, bench_bucket data, "
                      f"{nbuf} buckets cycled, {rounds} interleaved rounds, medians", "res": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
