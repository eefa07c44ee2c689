#!/usr/bin/env python3
"""The batched fused round trip (sml_roundtrip_loopback_batch: one launch
over several slices — the client's batched dispatch) on 2- vs 4-slice wave
tiles (sml_set_stream_tile_slices), on cold HBM: a 256 MiB job split into
its 4 FIFO slices (the allreduce_benchmark T = 4 shape) and 4 ResNet-50-sized
25 MiB buckets (configs[4]), 4 jobs of each cycled.  Interleaved rounds,
medians; outputs equal across tile sizes and to the single-slice kernel."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(rounds=9, nbuf=4, reps=20, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    shapes = {"256MiB as 4 FIFO slices": [sw.fifo_slice(64 << 20, 4, r) for r in range(4)],
              "4 x 25 MiB buckets": None}
    res = {}
    for name, sl in shapes.items():
        if sl is None:
            sizes = [6_553_600] * 3 + [5_896_232]
            offs = [sum(sizes[:i]) for i in range(4)]
            sl = list(zip(offs, sizes))
        total = sum(n for _, n in sl)
        jobs = []
        for b in range(nbuf):
            x = bench.bench_bucket(torch, 4242 + b, 0, total, dev)
            out = torch.empty_like(x)
            jobs.append([(x[o:o + n], out[o:o + n]) for o, n in sl])
        i = [0]

        def call():
            k = i[0] % nbuf
            i[0] += 1
            sw.roundtrip_loopback_batch(jobs[k], P, 1, stream=st)
        ref = None
        for arm in (4, 0):
            sw.set_stream_tile_slices(arm)
            for k in range(nbuf):
                i[0] = k
                call()
            torch.cuda.synchronize()
            cur = [torch.cat([o for _, o in j]).clone() for j in jobs]
            if ref is None:
                ref = cur
                single = torch.empty_like(ref[0])
                for (x, _), (o, n) in zip(jobs[0], sl):
                    sw.roundtrip_loopback(x, P, 1, out=single[o:o + n])
                torch.cuda.synchronize()
                assert torch.equal(single.view(torch.int32), ref[0].view(torch.int32))
            assert all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(ref, cur)), arm
        del ref, cur
        t = {4: [], 0: []}
        for _ in range(rounds):
            for arm in (4, 0):
                sw.set_stream_tile_slices(arm)
                for _ in range(8):
                    call()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    call()
                b.record(st)
                torch.cuda.synchronize()
                t[arm].append(a.elapsed_time(b) / reps * 1e3)
        sw.set_stream_tile_slices(0)
        res[name] = {("4 slices" if arm == 4 else "2 slices (default)"): {
            "median_us": round(statistics.median(v), 2), "GBps": round(8 * total / statistics.median(v) / 1e3, 1)}
            for arm, v in t.items()}
        del jobs
        torch.cuda.empty_cache()
    print(json.dumps({"what": f"batched fused round trip, W = 1, {nbuf} jobs cycled, {rounds} interleaved rounds, "
                      "medians; bytes = 8N", "res": res}, indent=1))


if __name__ == "__main__":
    main()
