#!/usr/bin/env python3
"""Interleaved A/B of sml_quantize_pack between builds of the kernel library
(same process, same buffers, alternating rounds; cdna_hip_programming.md
§5.4 rule 24).  Usage: ab_libs.py lib1.so lib2.so ..."""
import ctypes
import json
import os
import statistics
import sys

import torch


def main(paths, N=64 * 1024 * 1024, P=256, rounds=9, reps=10):
    dev = torch.device("cuda:0")
    x = torch.randn(N, device=dev)
    B = (N + P - 1) // P
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    exps = torch.empty(B, dtype=torch.int8, device=dev)
    ref = None
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        libs.append(L)
    st = torch.cuda.current_stream()
    res = {p: [] for p in paths}
    cres = {p: [] for p in paths}
    dres = {p: [] for p in paths}
    rres = {p: [] for p in paths}
    out = torch.empty_like(x)
    for p, L in zip(paths, libs):  # correctness: identical bytes
        assert L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, payload.data_ptr(), exps.data_ptr(), 0, st.cuda_stream) == 0
        torch.cuda.synchronize()
        cur = (payload.clone(), exps.clone())
        if ref is None:
            ref = cur
        assert torch.equal(ref[0], cur[0]) and torch.equal(ref[1], cur[1]), p
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, payload.data_ptr(), exps.data_ptr(), 0, st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize()
            res[p].append(a.elapsed_time(b) / reps * 1e3)
            L.sml_dequantize.restype = ctypes.c_int
            L.sml_dequantize.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
            a.record(st)
            for _ in range(reps):
                L.sml_dequantize(payload.data_ptr(), exps.data_ptr(), N, P, 1, out.data_ptr(), 0, st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize()
            dres[p].append(a.elapsed_time(b) / reps * 1e3)
            L.sml_roundtrip_loopback.restype = ctypes.c_int
            L.sml_roundtrip_loopback.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint16, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_void_p]
            a.record(st)
            for _ in range(reps):
                L.sml_roundtrip_loopback(x.data_ptr(), out.data_ptr(), N, P, 1, None, None, 0, st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize()
            rres[p].append(a.elapsed_time(b) / reps * 1e3)
            if hasattr(L, "sml_stream_copy"):
                L.sml_stream_copy.restype = ctypes.c_int
                L.sml_stream_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
                a.record(st)
                for _ in range(reps):
                    L.sml_stream_copy(x.data_ptr(), out.data_ptr(), 4 * N, st.cuda_stream)
                b.record(st)
                torch.cuda.synchronize()
                cres[p].append(a.elapsed_time(b) / reps * 1e3)
    alg = 8 * N + B
    rep = {}
    for p, v in res.items():
        rep[p] = {"median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2),
                  "GBps": round(alg / statistics.median(v) / 1e3, 1)}
        rep[p]["dequant_GBps"] = round(alg / statistics.median(dres[p]) / 1e3, 1)
        rep[p]["roundtrip_GBps"] = round(8 * N / statistics.median(rres[p]) / 1e3, 1)
        if cres[p]:
            rep[p]["copy_probe_GBps"] = round(8 * N / statistics.median(cres[p]) / 1e3, 1)
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:], P=int(os.environ.get("AB_P", 256)))
