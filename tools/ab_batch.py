#!/usr/bin/env python3
"""Kernel time of the fused round trip on a 256 MiB bucket: one
sml_roundtrip_loopback launch vs sml_roundtrip_loopback_batch with the
bucket as 1 slice and as T = 4 FIFO slices (HIP events, interleaved)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def fifo(n, T):
    out = []
    for t in range(T):
        q, r = divmod(n, T)
        m = q + (t < r)
        out.append((t * m if t < r else t * m + r, m))
    return out


def main(N=64 * 1024 * 1024, P=256, W=8, rounds=7, reps=20):
    x = torch.randn(N, device="cuda")
    o = torch.empty_like(x)
    st = torch.cuda.current_stream()
    arms = {
        "single": lambda: sw.roundtrip_loopback(x, P, W, out=o, stream=st),
        "batch_1slice": lambda: sw.roundtrip_loopback_batch([(x, o)], P, W, stream=st),
        "batch_T4": lambda: sw.roundtrip_loopback_batch([(x[a:a + m], o[a:a + m]) for a, m in fifo(N, 4)], P, W, stream=st),
        "batch_T4_unaligned": lambda: sw.roundtrip_loopback_batch([(x[a:a + m], o[a:a + m]) for a, m in fifo(N - 1, 4)], P, W, stream=st),
        "single_T4_launches": lambda: [sw.roundtrip_loopback(x[a:a + m], P, W, out=o[a:a + m], stream=st) for a, m in fifo(N, 4)],
    }
    res = {k: [] for k in arms}
    for _ in range(rounds):
        for k, fn in arms.items():
            for _ in range(3):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) / reps * 1e3)
    print(json.dumps({k: round(statistics.median(v), 2) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
