#!/usr/bin/env python3
"""Output store policy of the fused round trip when it runs IN PLACE (out is
the input bucket, as the reference's allreduce_benchmark and a framework's
in-place gradient all-reduce call it): non-temporal (threshold 0) vs
default-policy stores, on ONE re-reduced 256 MiB bucket (resident: what the
benchmark does job after job) and on 4 cycled buckets (cold), plus the
out-of-place cold case for reference.  Interleaved rounds, medians."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(rounds=9, nbuf=4, reps=30, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    N = 64 << 20
    xs = [bench.bench_bucket(torch, 4242 + b, 0, N, dev) for b in range(nbuf)]
    outs = [torch.empty(N, device=dev) for _ in range(nbuf)]
    i = [0]

    def call(nb, inplace):
        k = i[0] % nb
        i[0] += 1
        sw.roundtrip_loopback(xs[k], P, 1, out=xs[k] if inplace else outs[k], stream=st)
    cases = {"inplace resident": (1, True), "inplace cold": (nbuf, True), "out-of-place cold": (nbuf, False)}
    arms = [("nt", 0), ("default", 2 ** 64 - 1)]
    t = {(c, a): [] for c in cases for a, _ in arms}
    orig = sw.set_payload_nt_threshold(0)
    try:
        for _ in range(20):
            call(nbuf, False)
        for _ in range(rounds):
            for c, (nb, ip) in cases.items():
                for a, thr in arms:
                    sw.set_payload_nt_threshold(thr)
                    for _ in range(8):
                        call(nb, ip)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        call(nb, ip)
                    e1.record(st)
                    torch.cuda.synchronize()
                    t[(c, a)].append(e0.elapsed_time(e1) / reps * 1e3)
    finally:
        sw.set_payload_nt_threshold(orig)
    res = {}
    for (c, a), v in t.items():
        m = statistics.median(v)
        res.setdefault(c, {})[a] = {"median_us": round(m, 2), "GBps": round(8 * N / m / 1e3, 1)}
    print(json.dumps({"what": "fused round trip (W = 1), 256 MiB, output store policy, in place vs out of place, "
                      f"{rounds} interleaved rounds, medians", "res": res}, indent=1))


if __name__ == "__main__":
    main()
