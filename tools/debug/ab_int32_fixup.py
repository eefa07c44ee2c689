#!/usr/bin/env python3
"""The marginal cost of the INT32 rx fix-up launch: sml_rx_reset +
sml_unpack_frames_int32 over 4 cycled 256 MiB-slice frame sets, interleaved
between two builds of the library — the product (`cur.so`: one-pass kernel +
one-workgroup fix-up) and a timing-only variant without the fix-up launch
(`nofix.so`, correct only when no copies race, as here).  Usage:
ab_int32_fixup.py cur.so nofix.so"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(paths, rounds=9, nbuf=4, reps=20, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    libs = []
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        L.sml_unpack_frames_int32.restype = ctypes.c_int
        L.sml_unpack_frames_int32.argtypes = [vp, u64, u64, u64, u32, u64, vp, vp, vp, vp]
        L.sml_rx_reset.restype = ctypes.c_int
        L.sml_rx_reset.argtypes = [vp, u64, vp]
        libs.append(L)
    N = 64 << 20
    B = sw.num_blocks(N, P)
    fb = sw.frame_bytes(P)
    fp = sw.frame_params(job_id=1)
    g = torch.Generator(device=dev)
    xs = []
    for b in range(nbuf):
        g.manual_seed(100 + b)
        xs.append(torch.randint(-2 ** 31, 2 ** 31 - 1, (N,), dtype=torch.int32, device=dev, generator=g))
    frames = [sw.pack_frames_int32(x, fp, P) for x in xs]
    rxs = [sw.RxSliceInt32(N, P, device=dev) for _ in range(nbuf)]
    i = [0]

    def call(L):
        k = i[0] % nbuf
        i[0] += 1
        r = rxs[k]
        assert L.sml_rx_reset(r.state.data_ptr(), r.state.numel(), st.cuda_stream) == 0
        assert L.sml_unpack_frames_int32(frames[k].data_ptr(), B, fb, N, P, 1, r.state.data_ptr(), r.out.data_ptr(),
                                         r.counts.data_ptr(), st.cuda_stream) == 0

    for p, L in zip(paths, libs):
        i[0] = 0
        for k in range(nbuf):
            rxs[k].out.zero_()
            call(L)
        torch.cuda.synchronize()
        for k in range(nbuf):
            assert torch.equal(rxs[k].out, xs[k]), (p, k)
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
    alg = 4 * N + B * fb
    res = {os.path.basename(p): {"median_us": round(statistics.median(v), 2),
                                 "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in t.items()}
    print(json.dumps({"what": f"INT32 rx (reset + one pass [+ fix-up]) per 256 MiB slice, {nbuf} frame sets cycled, "
                      f"{rounds} interleaved rounds, medians; bytes = 4N + frame bytes", "res": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
