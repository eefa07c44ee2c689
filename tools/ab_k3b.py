#!/usr/bin/env python3
"""Interleaved timing of K1 (fused exponents) and K3 (given global exponents =
K1's own plane, so no wrap path) across kernel-library builds and launch
shapes (tiles per wave 1 / 2), 256 MiB, P = 256, W = 1.  Usage:
ab_k3b.py lib.so [lib.so ...]   (first lib = reference for K3 payload equality)"""
import ctypes
import json
import statistics
import sys

import torch


def main(paths, N=64 * 1024 * 1024, P=256, rounds=9, reps=20):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = torch.randn(N, device=dev, generator=g)
    B = N // P
    exps = torch.empty(B, dtype=torch.int8, device=dev)
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    st = torch.cuda.current_stream()
    libs = {}
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        L.sml_dequantize.restype = ctypes.c_int
        L.sml_dequantize.argtypes = [vp, vp, u64, u32, u16, vp, u32, vp]
        L.sml_set_quantize_tile_slices.restype = u32
        L.sml_set_quantize_tile_slices.argtypes = [u32]
        libs[p] = L
    L0 = libs[paths[0]]
    assert L0.sml_quantize_pack(x.data_ptr(), N, P, 1, None, payload.data_ptr(), exps.data_ptr(), 0, st.cuda_stream) == 0
    torch.cuda.synchronize()
    ref = payload.clone()

    def k1(L):
        return L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, payload.data_ptr(), exps.data_ptr(), 0, st.cuda_stream)

    def k3(L):
        return L.sml_quantize_pack(x.data_ptr(), N, P, 1, exps.data_ptr(), payload.data_ptr(), None, 0, st.cuda_stream)

    out = torch.empty_like(x)

    def k4(L):
        return L.sml_dequantize(ref.data_ptr(), exps.data_ptr(), N, P, 1, out.data_ptr(), 0, st.cuda_stream)

    tpws = (4, 2) if "--slices2" in sys.argv else (4,)   # tile slices per wave
    arms = []
    for p in paths:
        for tpw in tpws:
            arms.append((f"{p.split('/')[-1]} K1 tpw{tpw}", libs[p], k1, tpw))
            arms.append((f"{p.split('/')[-1]} K3 tpw{tpw}", libs[p], k3, tpw))
        arms.append((f"{p.split('/')[-1]} K4", libs[p], k4, 1))
    eq = {}
    for name, L, fn, tpw in arms:
        L.sml_set_quantize_tile_slices(tpw)
        assert fn(L) == 0
        torch.cuda.synchronize()
        eq[name] = bool(torch.equal(payload, ref)) if fn is not k4 else None
    times = {a[0]: [] for a in arms}
    for _ in range(rounds):
        for name, L, fn, tpw in arms:
            L.sml_set_quantize_tile_slices(tpw)
            for _ in range(5):
                fn(L)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn(L)
            b.record(st)
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / reps * 1e3)
    alg = 8 * N + B
    print(json.dumps({k: {"median_us": round(statistics.median(v), 2), "GBps": round(alg / statistics.median(v) / 1e3, 1),
                          "payload_equal_ref": eq[k]} for k, v in times.items()}, indent=1))


if __name__ == "__main__":
    main([a for a in sys.argv[1:] if not a.startswith("--")])
