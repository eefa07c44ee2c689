#!/usr/bin/env python3
"""A/B of the frames receive path's output store policy (round 4): the
apply pass (k_rx_apply) with non-temporal fp32 output stores (what outputs of
64 MiB and more now get, like K4's) vs default-policy stores, on cold HBM —
the calls cycle 4 distinct frame sets and outputs of the 256 MiB bucket
(4 x (282 MB frames + 268 MB out)).  Each call: the rx reset and
sml_dequantize_frames (claim + apply), as bench.py --extra times it.
Interleaved rounds, medians; outputs checked equal to the fused round trip."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402
import bench  # noqa: E402


def main(rounds=9, nbuf=4, reps=20):
    P, N = 256, 64 << 20
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    B = sw.num_blocks(N, P)
    fb = sw.frame_bytes(P)
    nframes = B + min(B, 64)
    fp = sw.frame_params(max_outstanding_pkts=64)
    xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
    frames = [sw.quantize_pack_frames(x, fp, P, 1, batch_max=64) for x in xs]
    rxs = [sw.RxSlice(N, P, 64, device=dev) for _ in range(nbuf)]
    refs = [sw.roundtrip_loopback(x, P, 1) for x in xs]
    del xs
    orig = sw.set_payload_nt_threshold(2 ** 64 - 1)
    arms = [("nt stores", 0), ("default stores", 2 ** 64 - 1)]
    i = [0]

    def call():
        k = i[0] % nbuf
        i[0] += 1
        rxs[k].reset(st)
        sw.dequantize_frames(frames[k], nframes, rxs[k], num_workers=1, stream=st)

    try:
        for name, thr in arms:
            sw.set_payload_nt_threshold(thr)
            for k in range(nbuf):
                call()
            torch.cuda.synchronize()
            for k in range(nbuf):
                assert torch.equal(rxs[k].out, refs[k]), (name, k)
        t = {a[0]: [] for a in arms}
        for _ in range(rounds):
            for name, thr in arms:
                sw.set_payload_nt_threshold(thr)
                for _ in range(8):
                    call()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    call()
                b.record(st)
                torch.cuda.synchronize()
                t[name].append(a.elapsed_time(b) / reps * 1e3)
    finally:
        sw.set_payload_nt_threshold(orig)
    alg = 4 * N + nframes * fb
    res = {n: {"median_us": round(statistics.median(v), 2), "GBps": round(alg / statistics.median(v) / 1e3, 1)}
           for n, v in t.items()}
    print(json.dumps({"what": "frames rx (reset + claim + apply) per 256 MiB call, 4 frame sets cycled, "
                      f"{rounds} interleaved rounds, medians; bytes = 4N + frame bytes", "res": res}, indent=1))


if __name__ == "__main__":
    main()
