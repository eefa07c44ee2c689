#!/usr/bin/env python3
"""configs[4] on one GPU: ResNet-50-sized gradient buckets streamed through
the SwitchML pre/post-processor, device-resident and host-inclusive.

ResNet-50 has 25,557,032 fp32 parameters; PyTorch DDP's default 25 MiB
buckets cut them into 3 x 6,553,600 + 5,896,232 elements (SURVEY §8 D3 cfg5;
not in the reference, so the sizes are parity-unpinned).  Per "iteration"
every bucket goes through quantize -> loopback (x W) -> dequantize, the
dummy-backend all-reduce, in three placements:

  device      buckets in HBM, fused round-trip kernel per bucket
  staged      buckets in pinned host memory (what ProcessGroupSML /
              the NCCL plugin hand SwitchML, ProcessGroupSML.cpp:113-163):
              H2D copy, fused round trip, D2H copy, one stream
  zero_copy   buckets in pinned host memory, the fused kernel reads and
              writes them directly over PCIe

Reported: ms per iteration (all buckets) and elements/s (the unit of the
reference's own headline figure, docs/img/benchmark.png) per GPU.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402  (torch first: it owns the process's HIP runtime)
import switchml_amd as sw  # noqa: E402

RESNET50 = 25_557_032
BUCKET = 25 * 1024 * 1024 // 4


def buckets():
    sizes, left = [], RESNET50
    while left > 0:
        sizes.append(min(BUCKET, left))
        left -= sizes[-1]
    return sizes


def main(iters=20, W=8, P=256):
    dev = torch.device("cuda:0")
    sizes = buckets()
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    dbufs = [torch.randn(n, device=dev, generator=gen) * 1e-3 for n in sizes]
    douts = [torch.empty_like(b) for b in dbufs]
    hbufs = [b.cpu().pin_memory() for b in dbufs]
    houts = [torch.empty_like(b).pin_memory() for b in hbufs]
    st = torch.cuda.current_stream()

    def device():
        for b, o in zip(dbufs, douts):
            sw.roundtrip_loopback(b, P, W, out=o, stream=st)

    def staged():
        for h, ho, d, o in zip(hbufs, houts, dbufs, douts):
            d.copy_(h, non_blocking=True)
            sw.roundtrip_loopback(d, P, W, out=o, stream=st)
            ho.copy_(o, non_blocking=True)

    def zero_copy():
        for h, ho in zip(hbufs, houts):
            sw.roundtrip_loopback(h, P, W, out=ho, stream=st)

    res = {"buckets": sizes, "params": RESNET50, "num_workers": W, "packet_numel": P}
    for name, fn in (("device", device), ("staged", staged), ("zero_copy", zero_copy)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = statistics.median(ts)
        res[name] = {"ms_per_iteration": round(t * 1e3, 4), "elements_per_s": round(RESNET50 / t, 1)}
    # same bits in every placement
    device()
    zero_copy()
    torch.cuda.synchronize()
    res["placements_agree"] = all(torch.equal(o.cpu(), ho) for o, ho in zip(douts, houts))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
