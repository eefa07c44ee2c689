#!/usr/bin/env python3
"""Interleaved A/B of sml_switch_aggregate (K6) between builds of the kernel
library: W planes of the 256 MiB bucket -> fp32 out, same process, same
buffers, alternating rounds; outputs must be bit-identical.
Usage: ab_switch.py lib1.so lib2.so ..."""
import ctypes
import json
import statistics
import sys

import torch


def main(paths, N=64 * 1024 * 1024, P=256, rounds=7, reps=10):
    dev = torch.device("cuda:0")
    B = (N + P - 1) // P
    planes = [torch.randint(-2 ** 28, 2 ** 28, (B * P,), dtype=torch.int32, device=dev) for _ in range(8)]
    exps = torch.randint(-20, 5, (B,), dtype=torch.int8, device=dev)
    out = torch.empty(N, dtype=torch.float32, device=dev)
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_switch_aggregate.restype = ctypes.c_int
        L.sml_switch_aggregate.argtypes = [vp, vp, u16, u64, u32, vp, vp, vp, u32, vp]
        libs.append(L)
    st = torch.cuda.current_stream()
    pp = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in planes])
    ep = (ctypes.c_void_p * 8)(*([exps.data_ptr()] * 8))

    def call(L, W):
        return L.sml_switch_aggregate(ctypes.cast(pp, vp), ctypes.cast(ep, vp), W, N, P, None, None,
                                      out.data_ptr(), 0, st.cuda_stream)
    res = {}
    for W in (2, 4, 8):
        ref = None
        for p, L in zip(paths, libs):
            assert call(L, W) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(ref.view(torch.int32), out.view(torch.int32)), (p, W)
        times = {p: [] for p in paths}
        for _ in range(rounds):
            for p, L in zip(paths, libs):
                for _ in range(3):
                    call(L, W)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    call(L, W)
                b.record(st)
                torch.cuda.synchronize()
                times[p].append(a.elapsed_time(b) / reps * 1e3)
        alg = W * (4 * B * P + B) + 4 * N
        res[f"W{W}"] = {p: {"median_us": round(statistics.median(v), 2),
                            "GBps": round(alg / (statistics.median(v) * 1e-6) / 1e9, 1)} for p, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
