#!/usr/bin/env python3
"""Interleaved A/B of sml_dequantize_frames between library builds: frames
from the product library's quantize_pack_frames (256 MiB bucket, W = 1),
each build's receive side timed with the rx state reset inside the timed
region, output checked against the fused loopback round trip."""
import ctypes, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch
import switchml_amd as sw


def main(paths, N=64 * 1024 * 1024, P=256, bm=64, rounds=7, reps=10):
    x = torch.randn(N, device="cuda")
    B = sw.num_blocks(N, P)
    F = B + min(B, bm)
    fb = sw.frame_bytes(P)
    frames = sw.quantize_pack_frames(x, sw.frame_params(max_outstanding_pkts=bm), P, 1, batch_max=bm)
    if os.environ.get("AB_SHUFFLE"):
        # AB_SHUFFLE=w: frames permuted at random inside windows of w frames
        w = int(os.environ["AB_SHUFFLE"])
        g = torch.Generator().manual_seed(7)
        perm = torch.cat([i + torch.randperm(min(w, F - i), generator=g) for i in range(0, F, w)]).to("cuda")
        frames = frames.view(F, fb)[perm].reshape(-1).contiguous()
    ref = sw.roundtrip_loopback(x, P, 1)
    st = torch.cuda.current_stream()
    state = torch.zeros(F, dtype=torch.int64, device="cuda")
    exps = torch.zeros(B, dtype=torch.int8, device="cuda")
    out = torch.empty(N, device="cuda")
    vp, u64, u32, u16 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16
    libs = []
    for p in paths:
        L = ctypes.CDLL(p)
        L.sml_dequantize_frames.restype = ctypes.c_int
        L.sml_dequantize_frames.argtypes = [vp, u64, u64, u64, u32, u16, u32, u64, vp, vp, vp, vp, vp]
        libs.append(L)

    # AB_COUNTS=1: also pass the {accepted, discarded} counters
    counts = torch.zeros(2, dtype=torch.int64, device="cuda") if os.environ.get("AB_COUNTS") else None

    def run(L):
        state.zero_()
        rc = L.sml_dequantize_frames(frames.data_ptr(), F, fb, N, P, 1, bm, 0, exps.data_ptr(), state.data_ptr(),
                                     out.data_ptr(), None if counts is None else counts.data_ptr(), st.cuda_stream)
        assert rc == 0, rc

    for p, L in zip(paths, libs):
        out.zero_()
        run(L)
        torch.cuda.synchronize()
        if not os.environ.get("AB_NOCHECK"):
            assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), p
    res = {p: [] for p in paths}
    for _ in range(rounds):
        for p, L in zip(paths, libs):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                run(L)
            b.record(st)
            torch.cuda.synchronize()
            res[p].append(a.elapsed_time(b) / reps * 1e3)
    alg = 4 * N + F * fb
    print(json.dumps({p: {"median_us": round(statistics.median(v), 2),
                          "GBps": round(alg / statistics.median(v) / 1e3, 1)} for p, v in res.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
