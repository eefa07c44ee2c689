#!/usr/bin/env python3
"""Frames tx (sml_quantize_pack_frames) on the 256 MiB bucket vs the frame
stride: packed 1076-byte frames (frame starts 4-B aligned) against padded
strides (64-B aligned frame starts, as in a DPDK mbuf pool whose data rooms
start 128 B into 2 KiB+ buffers).  Rates count useful bytes only:
4N fp32 read + (B + b) x 1076 frame bytes written.  Interleaved rounds."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(N=64 << 20, P=256, bm=64, rounds=7, reps=10):
    dev = torch.device("cuda:0")
    x = torch.randn(N, device=dev)
    B = sw.num_blocks(N, P)
    F = B + min(B, bm)
    fb = sw.frame_bytes(P)
    strides = [int(s) for s in os.environ.get("STRIDES", f"{fb},1088,1152,2048,2176").split(",")]
    bufs = {s: torch.empty(F * s + 64, dtype=torch.uint8, device=dev) for s in strides}
    fp = sw.frame_params(max_outstanding_pkts=bm)
    st = torch.cuda.current_stream()
    res = {s: [] for s in strides}
    for _ in range(rounds):
        for s in strides:
            fn = lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=bm, frames=bufs[s], stride=s, stream=st)
            fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            torch.cuda.synchronize()
            res[s].append(a.elapsed_time(b) / reps * 1e3)
    useful = 4 * N + F * fb
    print(json.dumps({str(s): {"median_us": round(statistics.median(v), 2),
                               "useful_GBps": round(useful / statistics.median(v) / 1e3, 1)} for s, v in res.items()},
                     indent=1))


if __name__ == "__main__":
    main()
