#!/usr/bin/env python3
"""The batched fused round trip (sml_roundtrip_loopback_batch: one launch
over several slices — the client's batched dispatch) between library builds
(e.g. -DSML_BATCH_SLICES=2 vs 4), on cold HBM: a 256 MiB job split into its
4 FIFO slices (the allreduce_benchmark T = 4 shape) and 4 ResNet-50-sized
25 MiB buckets (configs[4]), 4 jobs of each cycled.  Interleaved rounds,
medians; every build's outputs equal the single-slice kernel's.
Usage: ab_batch_slices.py lib1.so lib2.so ..."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import bench  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(paths, rounds=9, nbuf=4, reps=20, P=256):
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    libs = []
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        L.sml_roundtrip_loopback_batch.restype = ctypes.c_int
        L.sml_roundtrip_loopback_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.c_uint16, ctypes.c_uint32, ctypes.c_void_p]
        libs.append(L)
    sizes25 = [6_553_600] * 3 + [5_896_232]
    shapes = {"256MiB as 4 FIFO slices": [sw.fifo_slice(64 << 20, 4, r) for r in range(4)],
              "4 x 25 MiB buckets": [(sum(sizes25[:i]), sizes25[i]) for i in range(4)]}
    res = {}
    for name, sl in shapes.items():
        total = sum(n for _, n in sl)
        xs, outs, arrs = [], [], []
        for b in range(nbuf):
            x = bench.bench_bucket(torch, 4242 + b, 0, total, dev)
            out = torch.empty_like(x)
            arr = (sw.Slice * len(sl))()
            for i, (o, n) in enumerate(sl):
                arr[i] = sw.Slice(x.data_ptr() + 4 * o, out.data_ptr() + 4 * o, n)
            xs.append(x)
            outs.append(out)
            arrs.append(arr)
        ref = torch.empty_like(xs[0])
        for o, n in sl:
            sw.roundtrip_loopback(xs[0][o:o + n], P, 1, out=ref[o:o + n])
        i = [0]

        def call(L):
            k = i[0] % nbuf
            i[0] += 1
            assert L.sml_roundtrip_loopback_batch(arrs[k], len(sl), P, 1, 0, st.cuda_stream) == 0
        for p, L in zip(paths, libs):
            outs[0].zero_()
            i[0] = 0
            call(L)
            torch.cuda.synchronize()
            assert torch.equal(outs[0].view(torch.int32), ref.view(torch.int32)), (p, name)
        t = {p: [] for p in paths}
        for _ in range(rounds):
            for p, L in zip(paths, libs):
                for _ in range(8):
                    call(L)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    call(L)
                b.record(st)
                torch.cuda.synchronize()
                t[p].append(a.elapsed_time(b) / reps * 1e3)
        res[name] = {os.path.basename(p): {"median_us": round(statistics.median(v), 2),
                                           "GBps": round(8 * total / statistics.median(v) / 1e3, 1)}
                     for p, v in t.items()}
        del xs, outs, arrs, ref
        torch.cuda.empty_cache()
    print(json.dumps({"what": f"batched fused round trip, W = 1, {nbuf} jobs cycled, {rounds} interleaved rounds, "
                      "medians; bytes = 8N", "res": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
