#!/usr/bin/env python3
"""configs[4] through the CollNet plugin (bench.plugin_buckets: ResNet-50
buckets, loopback W = 8, T = 4, fused, batched dispatch), alternating the
batch worker's zero-copy coalescing window ([backend.hip] coalesce_us):
0 (off) against 20 / 50 us.  Medians over rounds, per placement."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402

BASE = ("[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\nmax_outstanding_packets = 256\n"
        "[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\ncoalesce_us = %d\n")


def main(rounds=5):
    os.environ["SWITCHML_COLLNET_LOOPBACK"] = "1"
    dev = torch.device("cuda:0")
    arms = [int(a) for a in os.environ.get("AB_COALESCE", "0,20,50").split(",")]
    res = {a: {"device": [], "pinned_host": []} for a in arms}
    agree = True
    for _ in range(rounds):
        for a in arms:
            r = bench.plugin_buckets(torch, dev, iters=10, ini=BASE % a)
            agree = agree and r["placements_agree"]
            for k in ("device", "pinned_host"):
                res[a][k].append(r[k]["ms_per_iteration"])
    out = {f"coalesce_us={a}": {k: {"median_ms": round(statistics.median(v), 4), "all_ms": v} for k, v in r.items()}
           for a, r in res.items()}
    out["placements_agree"] = agree
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
