#!/usr/bin/env python3
"""Per-burst latency of the per-packet paths: one
sml_exchange_burst launch + stream sync against one sml_burst_server_submit,
for 1 and 64 packets, packets in HBM and in pinned host memory.  Each burst
is a full exchange (post of q, pre of q + b into the same buffer) over a
fixed set of slots; median of `reps` bursts after a warm-up.

Usage: python tools/burst_latency.py [OUT.json]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))


def main():
    import numpy as np
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda", 0)
    P, W, b = 256, 2, 64
    n = 4096 * P                         # B = 4096 blocks, far more than the bursts touch
    x = torch.randn(n, device=dev)
    out = torch.zeros(n, device=dev)
    recv = torch.zeros(n // P, dtype=torch.int8, device=dev)
    res = {}
    stream = torch.cuda.current_stream(dev)
    for place in ("device", "pinned"):
        if place == "device":
            ring = torch.zeros(b * P, dtype=torch.int32, device=dev)
            ex = torch.zeros(b * 2, dtype=torch.uint8, device=dev)
        else:
            ring = torch.zeros(b * P, dtype=torch.int32).pin_memory()
            ex = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
        for count in (1, 16, 64):
            ids = list(range(b, b + count))          # received packets q >= b: post + pre of q + b
            bt = sw.packet_burst(x, out, P, W, b, recv, ids, [ring.data_ptr() + (q % b) * P * 4 for q in ids],
                                 [ex.data_ptr() + (q % b) * 2 for q in ids], flags=sw.FLAG_PROCESS_PACKET)
            for name in ("launch", "server"):
                srv = sw.BurstServer(P) if name == "server" else None

                def one():
                    if srv is None:
                        sw.exchange_burst(bt, stream)
                        stream.synchronize()
                    else:
                        srv.submit(sw.BURST_EXCHANGE, bt)
                for _ in range(50):
                    one()
                ts = []
                for _ in range(400):
                    t0 = time.perf_counter()
                    one()
                    ts.append(time.perf_counter() - t0)
                if srv is not None:
                    srv.close()
                res[f"{place}_{count}pkt_{name}_us"] = round(float(np.median(ts)) * 1e6, 2)
                print(place, count, name, res[f"{place}_{count}pkt_{name}_us"], flush=True)
    s = json.dumps(res, indent=1)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
