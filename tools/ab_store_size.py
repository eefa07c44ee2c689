#!/usr/bin/env python3
"""K1 payload store policy by bucket size: default-policy vs non-temporal
payload stores (two builds of the kernel library), one bucket re-read every
step at 256 MiB / 512 MiB / 1 GiB (the N = 1 headline, the N = 2 point of the
configs[3] curve, configs[3] on one GPU).  Interleaved rounds, medians;
planes checked equal.  Usage: ab_store_size.py default.so nt.so"""
import ctypes
import os
import json
import statistics
import sys

import torch


def main(paths, rounds=7):
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_quantize_pack.restype = ctypes.c_int
        L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
        libs.append(L)
    st = torch.cuda.current_stream()
    P = 256
    out = {}
    for mib in [int(v) for v in os.environ.get("AB_MIB", "256,512,1024").split(",")]:
        N = mib << 18
        B = N // P
        x = torch.randn(N, device="cuda")
        pl = torch.empty(B * P, dtype=torch.int32, device="cuda")
        ex = torch.empty(B, dtype=torch.int8, device="cuda")
        ref = None
        for L in libs:
            assert L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, pl.data_ptr(), ex.data_ptr(), 0, st.cuda_stream) == 0
            torch.cuda.synchronize()
            cur = pl.clone()
            ref = cur if ref is None else ref
            assert torch.equal(ref, cur)
        del ref, cur
        reps = max(10, 40 * 256 // mib)
        res = {p: [] for p in paths}
        for _ in range(rounds):
            for p, L in zip(paths, libs):
                for _ in range(5):
                    L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, pl.data_ptr(), ex.data_ptr(), 0, st.cuda_stream)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    L.sml_quantize_pack(x.data_ptr(), N, P, 1, None, pl.data_ptr(), ex.data_ptr(), 0, st.cuda_stream)
                b.record(st)
                torch.cuda.synchronize()
                res[p].append(a.elapsed_time(b) / reps * 1e3)
        alg = 8 * N + B
        out[f"{mib}MiB"] = {p.split("/")[-1]: {"median_us": round(statistics.median(v), 2),
                                                "TBps": round(alg / statistics.median(v) / 1e6, 3)}
                            for p, v in res.items()}
        del x, pl, ex
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
