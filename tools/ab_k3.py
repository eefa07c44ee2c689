#!/usr/bin/env python3
"""Interleaved A/B of K3 (sml_quantize_pack with given global exponents, the
switch-sim / peer-to-peer quantize) between builds of the kernel library;
payloads must be identical.  Usage: ab_k3.py lib1.so lib2.so ..."""
import ctypes
import json
import statistics
import sys

import torch


def main(paths, N=64 * 1024 * 1024, P=256, rounds=9, reps=10):
    dev = torch.device("cuda:0")
    x = torch.randn(N, device=dev)
    B = N // P
    gexp = torch.randint(-3, 6, (B,), dtype=torch.int8, device=dev)
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        libs.append(L)
    st = torch.cuda.current_stream()

    def call(L):
        return L.sml_quantize_pack(x.data_ptr(), N, P, 2, gexp.data_ptr(), payload.data_ptr(), None, 0, st.cuda_stream)
    ref = None
    for p, L in zip(paths, libs):
        assert call(L) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = payload.clone()
        assert torch.equal(ref, payload), p
    times = {p: [] for p in paths}
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            for _ in range(3):
                call(L)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                call(L)
            b.record(st)
            torch.cuda.synchronize()
            times[p].append(a.elapsed_time(b) / reps * 1e3)
    alg = 8 * N + B
    print(json.dumps({p: {"median_us": round(statistics.median(v), 2),
                          "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in times.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
