#!/usr/bin/env python3
"""Interleaved A/B of the frames receive path (sml_rx_reset +
sml_dequantize_frames: claim + apply) between builds of the kernel library,
on cold HBM: 4 distinct frame sets of the 256 MiB bucket (bench_bucket data,
W = 1) and 4 rx slices cycled.  Every build's output equals the fused round
trip.  Usage: ab_rx_libs_cold.py lib1.so lib2.so ..."""
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
        L.sml_dequantize_frames.restype = ctypes.c_int
        L.sml_dequantize_frames.argtypes = [vp, u64, u64, u64, u32, u16, u32, u64, vp, vp, vp, vp, vp]
        L.sml_rx_reset.restype = ctypes.c_int
        L.sml_rx_reset.argtypes = [vp, u64, vp]
        libs.append(L)
    N = 64 << 20
    B = sw.num_blocks(N, P)
    fb = sw.frame_bytes(P)
    nfr = B + min(B, 64)
    fp = sw.frame_params(max_outstanding_pkts=64)
    xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
    frames = [sw.quantize_pack_frames(x, fp, P, 1, batch_max=64) for x in xs]
    refs = [sw.roundtrip_loopback(x, P, 1) for x in xs]
    del xs
    rxs = [sw.RxSlice(N, P, 64, device=dev) for _ in range(nbuf)]
    i = [0]

    def call(L):
        k = i[0] % nbuf
        i[0] += 1
        r = rxs[k]
        assert L.sml_rx_reset(r.state.data_ptr(), r.state.numel(), st.cuda_stream) == 0
        assert L.sml_dequantize_frames(frames[k].data_ptr(), nfr, fb, N, P, 1, 64, 0, r.exps.data_ptr(),
                                       r.state.data_ptr(), r.out.data_ptr(), r.counts.data_ptr(),
                                       st.cuda_stream) == 0

    for p, L in zip(paths, libs):
        i[0] = 0
        for k in range(nbuf):
            rxs[k].out.zero_()
            call(L)
        torch.cuda.synchronize()
        for k in range(nbuf):
            assert torch.equal(rxs[k].out.view(torch.int32), refs[k].view(torch.int32)), (p, k)
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
    # bench.py --extra's way, once per library (3 warm calls, 20 timed)
    once = {}
    for p, L in zip(paths, libs):
        for _ in range(3):
            call(L)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            call(L)
        b.record(st)
        torch.cuda.synchronize()
        once[os.path.basename(p)] = round(a.elapsed_time(b) / reps * 1e3, 2)
    alg = 4 * N + nfr * fb
    res = {os.path.basename(p): {"median_us": round(statistics.median(v), 2),
                                 "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in t.items()}
    print(json.dumps({"what": f"frames rx (reset + claim + apply) per 256 MiB call, {nbuf} frame sets cycled, "
                      f"{rounds} interleaved rounds, medians; bytes = 4N + frame bytes", "res": res,
                      "bench_style_us": once}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
