#!/usr/bin/env python3
"""Interleaved A/B of sml_quantize_pack_frames between library builds."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch
import switchml_amd as sw


def main(paths, N=64 * 1024 * 1024, P=256, rounds=7, reps=10):
    x = torch.randn(N, device="cuda")
    B = sw.num_blocks(N, P)
    fb = 52 + 4 * P
    frames = torch.empty((B + 64) * fb, dtype=torch.uint8, device="cuda")
    fp = sw.frame_params(max_outstanding_pkts=64)
    st = torch.cuda.current_stream()
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_quantize_pack_frames.restype = ctypes.c_int
        L.sml_quantize_pack_frames.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16,
                                               ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(sw.FrameParams),
                                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        libs.append(L)
    ref = None
    for p, L in zip(paths, libs):
        assert L.sml_quantize_pack_frames(x.data_ptr(), N, P, 1, None, 64, ctypes.byref(fp), frames.data_ptr(), fb, st.cuda_stream) == 0
        torch.cuda.synchronize()
        cur = frames.clone()
        if ref is None:
            ref = cur
        if not os.environ.get("AB_NOCHECK"):
            assert torch.equal(ref, cur), p
    res = {p: [] for p in paths}
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                L.sml_quantize_pack_frames(x.data_ptr(), N, P, 1, None, 64, ctypes.byref(fp), frames.data_ptr(), fb, st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize()
            res[p].append(a.elapsed_time(b) / reps * 1e3)
    alg = 4 * N + (B + 64) * fb
    print(json.dumps({p: {"median_us": round(statistics.median(v), 2),
                          "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in res.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
