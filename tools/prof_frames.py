#!/usr/bin/env python3
"""Frames tx + rx on the 256 MiB bucket, for rocprofv3 --kernel-trace --stats
and the PMC passes: quantize into DPDK frames (device), then the receive side
over the same frames (W = 1 loopback), `reps` times each, cycling `sets`
distinct frame sets and rx slices (4 = 1.1 GB of frames, past the 256 MiB
Infinity Cache: a receive stream's HBM-proper pattern, as bench.py's
`frames_*_4sets` fields; 1 = one re-read set).  Prints wall-clock rates."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(N=64 * 2 ** 20, P=256, bm=64, reps=20, sets=int(os.environ.get("FRAME_SETS", "4"))):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    x = torch.randn(N, device=dev, generator=g)
    B = sw.num_blocks(N, P)
    F = B + min(B, bm)
    fb = F * sw.frame_bytes(P)
    frames = [torch.empty(fb, dtype=torch.uint8, device=dev) for _ in range(sets)]
    fp = sw.frame_params(max_outstanding_pkts=bm)
    rxs = [sw.RxSlice(N, P, bm, device=dev) for _ in range(sets)]
    k = [0]

    def tx():
        sw.quantize_pack_frames(x, fp, P, 1, batch_max=bm, frames=frames[k[0] % sets])
        k[0] += 1

    def rx():
        r = rxs[k[0] % sets]
        r.reset()
        sw.dequantize_frames(frames[k[0] % sets], F, r)
        k[0] += 1

    res = {"frame_sets": sets}
    for name, fn in (("tx", tx), ("rx", rx)):
        k[0] = 0
        for _ in range(sets):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        res[name] = {"us": round(t * 1e6, 1), "GBps": round((4 * N + fb) / t / 1e9, 1)}
    ref = sw.roundtrip_loopback(x, P, 1)
    torch.cuda.synchronize()
    res["rx_equals_roundtrip"] = all(bool(torch.equal(ref.view(torch.int32), r.out.view(torch.int32))) for r in rxs)
    del frames, rxs, ref
    # INT32 slices: B frames, tx = k_quantize_frames<.., I32>, rx = k_rx_int32 + fix-up
    xi = x.view(torch.int32)
    fbi = B * sw.frame_bytes(P)
    iframes = [torch.empty(fbi, dtype=torch.uint8, device=dev) for _ in range(sets)]
    irxs = [sw.RxSliceInt32(N, P, device=dev) for _ in range(sets)]

    def itx():
        sw.pack_frames_int32(xi, fp, P, frames=iframes[k[0] % sets])
        k[0] += 1

    def irx():
        r = irxs[k[0] % sets]
        r.reset()
        sw.unpack_frames_int32(iframes[k[0] % sets], B, r)
        k[0] += 1

    for name, fn in (("int32_tx", itx), ("int32_rx", irx)):
        k[0] = 0
        for _ in range(sets):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        res[name] = {"us": round(t * 1e6, 1), "GBps": round((4 * N + fbi) / t / 1e9, 1)}
    res["int32_rx_exact"] = all(bool(torch.equal(r.out, xi)) for r in irxs)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
