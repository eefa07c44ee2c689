#!/usr/bin/env python3
"""Interleaved A/B of the XCD-aware workgroup order (sml_set_xcd_chunk) on
every streaming kernel of the path, one GPU: K1 quantize+pack, K4 dequantize,
the fused loopback round trip, the frames tx kernel and the tile copy probe.
Every (kernel, chunk) pair is timed in every round; medians reported.
Sizes via AB_SIZES (fp32 elements, comma list; default 256 MiB and 1 GiB)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def run(N, P, chunks, rounds, reps=10):
    dev = torch.device("cuda:0")
    x = torch.randn(N, device=dev)
    B = sw.num_blocks(N, P)
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    exps = torch.empty(B, dtype=torch.int8, device=dev)
    out = torch.empty_like(x)
    st = torch.cuda.current_stream()
    fp = sw.frame_params(max_outstanding_pkts=64)
    fbytes = (B + min(B, 64)) * sw.frame_bytes(P)
    frames = torch.empty(fbytes, dtype=torch.uint8, device=dev)
    kernels = {
        "quantize_pack": (8 * N + B, lambda: sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=st)),
        "dequantize": (8 * N + B, lambda: sw.dequantize(payload, exps, N, P, 1, out=out, stream=st)),
        "roundtrip": (8 * N, lambda: sw.roundtrip_loopback(x, P, 1, out=out, stream=st)),
        "frames_tx": (4 * N + fbytes, lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=64, frames=frames,
                                                                      stream=st)),
        "tile_copy": (8 * N, lambda: sw.stream_copy(x, out, stream=st)),
    }

    def t_of(fn):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e-3

    res = {(k, c): [] for k in kernels for c in chunks}
    for _ in range(rounds):
        for k, (_, fn) in kernels.items():
            for c in chunks:
                sw.set_xcd_chunk(c)
                res[(k, c)].append(t_of(fn))
    sw.set_xcd_chunk(64)
    rows = []
    for (k, c), ts in res.items():
        m = statistics.median(ts)
        rows.append({"kernel": k, "xcd_chunk": c, "median_us": round(m * 1e6, 2), "min_us": round(min(ts) * 1e6, 2),
                     "GBps": round(kernels[k][0] / m / 1e9, 1)})
    return {"numel": N, "P": P, "rounds": rounds, "reps": reps, "rows": rows}


def main():
    P = int(os.environ.get("AB_P", 256))
    rounds = int(os.environ.get("AB_ROUNDS", 7))
    chunks = [int(c) for c in os.environ.get("AB_CHUNKS", "0,16,32,64,128,256").split(",")]
    sizes = [int(s) for s in os.environ.get("AB_SIZES", f"{64 << 20},{256 << 20}").split(",")]
    out = [run(N, P, chunks, rounds) for N in sizes]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
