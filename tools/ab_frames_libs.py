#!/usr/bin/env python3
"""Interleaved A/B of the frames transmit kernel (sml_quantize_pack_frames)
between builds of the kernel library, on cold HBM: bench_bucket data, the
calls cycling 4 distinct 256 MiB buckets and frame sets.  Same process,
alternating rounds, medians; every build's frames checked equal.
Usage: ab_frames_libs.py lib1.so lib2.so ..."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(paths, rounds=9, nbuf=4, reps=20, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        L.sml_quantize_pack_frames.restype = ctypes.c_int
        L.sml_quantize_pack_frames.argtypes = [vp, u64, u32, u16, vp, u32, ctypes.POINTER(sw.FrameParams), vp, u64,
                                               vp]
        libs.append(L)
    N = 64 << 20
    B = sw.num_blocks(N, P)
    fb = sw.frame_bytes(P)
    nfr = B + min(B, 64)
    fp = sw.frame_params(max_outstanding_pkts=64)
    xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
    frs = [torch.empty(nfr * fb, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    i = [0]

    def call(L):
        k = i[0] % nbuf
        i[0] += 1
        assert L.sml_quantize_pack_frames(xs[k].data_ptr(), N, P, 1, None, 64, ctypes.byref(fp), frs[k].data_ptr(), fb,
                                          st.cuda_stream) == 0

    ref = None
    for p, L in zip(paths, libs):
        i[0] = 0
        call(L)
        torch.cuda.synchronize()
        if ref is None:
            ref = frs[0].clone()
        assert torch.equal(ref, frs[0]), p
    del ref
    t = {p: [] for p in paths}
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            for _ in range(8):
                call(L)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                call(L)
            b.record(st)
            torch.cuda.synchronize()
            t[p].append(a.elapsed_time(b) / reps * 1e3)
    alg = 4 * N + nfr * fb
    res = {os.path.basename(p): {"median_us": round(statistics.median(v), 2),
                                 "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in t.items()}
    print(json.dumps({"what": f"frames tx, 256 MiB bucket, {nbuf} buckets + frame sets cycled, {rounds} interleaved "
                      "rounds, medians; bytes = 4N + frame bytes", "res": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
