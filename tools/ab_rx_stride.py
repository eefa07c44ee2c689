#!/usr/bin/env python3
"""Frames tx and rx (sml_quantize_pack_frames / sml_rx_reset +
sml_dequantize_frames) on the 256 MiB bucket vs the frame stride: packed
1076-byte frames against 64-B aligned strides (a DPDK mbuf pool's data rooms
start 128 B into 2 KiB+ buffers).  Useful bytes only: 4N fp32 + (B + b) x 1076
frame bytes.  Interleaved rounds, medians; rx output checked against the
fused loopback round trip."""
import json
import os
import statistics
import sys

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
    strides = [fb, 1088, 1152, 2176]
    bufs = {s: torch.empty(F * s, dtype=torch.uint8, device=dev) for s in strides}
    fp = sw.frame_params(max_outstanding_pkts=bm)
    st = torch.cuda.current_stream()
    rx = sw.RxSlice(N, P, bm, device=dev)
    ref = sw.roundtrip_loopback(x, P, 1)
    for s in strides:
        sw.quantize_pack_frames(x, fp, P, 1, batch_max=bm, frames=bufs[s], stride=s, stream=st)
        rx.reset(stream=st)
        sw.dequantize_frames(bufs[s], F, rx, stride=s, stream=st)
        torch.cuda.synchronize()
        assert torch.equal(rx.out.view(torch.int32), ref.view(torch.int32)), s
    res = {s: {"tx": [], "rx": []} for s in strides}
    for _ in range(rounds):
        for s in strides:
            for kind in ("tx", "rx"):
                if kind == "tx":
                    fn = lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=bm, frames=bufs[s], stride=s, stream=st)
                else:
                    def fn():
                        rx.reset(stream=st)
                        sw.dequantize_frames(bufs[s], F, rx, stride=s, stream=st)
                fn()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                torch.cuda.synchronize()
                res[s][kind].append(a.elapsed_time(b) / reps * 1e3)
    useful = 4 * N + F * fb
    print(json.dumps({str(s): {k: {"median_us": round(statistics.median(v), 2),
                                   "GBps": round(useful / statistics.median(v) / 1e3, 1)} for k, v in r.items()}
                      for s, r in res.items()}, indent=1))


if __name__ == "__main__":
    main()
