#!/usr/bin/env python3
"""Why does bench.py --extra's frames_rx_device_4sets figure (~98 us per
256 MiB) sit above tools/ab_rx_libs_cold.py's (~92 us) on the same box?
Times the same rx call (reset + dequantize_frames over 4 cycled frame sets)
four ways, each the median of 7 (3 warm + 20 timed) runs:
  A  bench's code: Python wrappers, side stream, 4 frame sets of ONE bucket
  B  direct ctypes calls (the A/B tool's), side stream, same frames
  C  Python wrappers on the default stream
  D  Python wrappers, side stream, frame sets of 4 DISTINCT buckets."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(P=256, reps=20, runs=7):
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(dev)
    N = 64 << 20
    B = sw.num_blocks(N, P)
    fb = sw.frame_bytes(P)
    nfr = B + min(B, 64)
    fp = sw.frame_params(max_outstanding_pkts=64)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.randn(N, device=dev, generator=g)
    same = [sw.quantize_pack_frames(x, fp, P, 1, batch_max=64) for _ in range(4)]
    xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(4)]
    dist = [sw.quantize_pack_frames(xb, fp, P, 1, batch_max=64) for xb in xs]
    del xs
    rxs = [sw.RxSlice(N, P, 64, device=dev) for _ in range(4)]
    L = sw.lib()
    k = [0]

    def wrap(fsets, st):
        def f():
            r = rxs[k[0] % 4]
            r.reset(st)
            sw.dequantize_frames(fsets[k[0] % 4], nfr, r, num_workers=1, stream=st)
            k[0] += 1
        return f

    def raw(fsets, st):
        def f():
            r = rxs[k[0] % 4]
            L.sml_rx_reset(r.state.data_ptr(), r.state.numel(), st.cuda_stream)
            L.sml_dequantize_frames(fsets[k[0] % 4].data_ptr(), nfr, fb, N, P, 1, 64, 0, r.exps.data_ptr(),
                                    r.state.data_ptr(), r.out.data_ptr(), r.counts.data_ptr(), st.cuda_stream)
            k[0] += 1
        return f

    cur = torch.cuda.current_stream(dev)
    ways = {"A_bench_wrappers_side_same": (wrap(same, side), side),
            "B_ctypes_side_same": (raw(same, side), side),
            "C_wrappers_default_same": (wrap(same, cur), cur),
            "D_wrappers_side_distinct": (wrap(dist, side), side)}
    t = {w: [] for w in ways}
    for _ in range(runs):
        for w, (fn, st) in ways.items():
            with torch.cuda.stream(st):
                t[w].append(bench.time_launches(torch, fn, st, reps) * 1e6)
    alg = 4 * N + nfr * fb
    res = {w: {"median_us": round(statistics.median(v), 2), "GBps": round(alg / statistics.median(v) / 1e3, 1),
               "runs_us": [round(u, 1) for u in v]} for w, v in t.items()}
    print(json.dumps({"what": __doc__.splitlines()[0], "res": res}, indent=1))


if __name__ == "__main__":
    main()
