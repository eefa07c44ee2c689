#!/usr/bin/env python3
"""Zero-copy (PCIe) fused round trips over pinned host buffers: aggregate
fp32 GB/s each way by kernel size and number of concurrent streams (each
stream runs its own sequence of kernels on its own buffers)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(P=256, W=8, total=32 * 1024 * 1024, rounds=3):
    res = {}
    for n in (409_600, 1_638_400, 6_553_600, 26_214_400):
        for ns in (1, 2, 4, 8):
            per = max(1, total // (n * ns))                       # kernels per stream
            streams = [torch.cuda.Stream() for _ in range(ns)]
            bufs = [(torch.randn(n).pin_memory(), torch.empty(n).pin_memory()) for _ in range(ns)]

            def run():
                for _ in range(per):
                    for s, (x, o) in zip(streams, bufs):
                        sw.roundtrip_loopback(x, P, W, out=o, stream=s)
            run()
            torch.cuda.synchronize()
            v = []
            for _ in range(rounds):
                t0 = time.perf_counter()
                run()
                torch.cuda.synchronize()
                v.append(4 * n * ns * per / (time.perf_counter() - t0) / 1e9)
            res[f"n{n}_streams{ns}"] = round(statistics.median(v), 2)
            del bufs
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
