#!/usr/bin/env python3
"""The INT32 rx fix-up with conflicts to resolve: a 256 MiB INT32
slice (B = 262 144 frames of P = 256), received in order, with K pkt_ids
whose claim was planted beforehand as a LATER frame's tag (what a later copy
that won the race to the claim atomic leaves) — so the real frames displace
them, mark them dirty and the fix-up must rewrite K blocks.  Three modes, 10
calls each, in this order: "clean" (no planted claims), "list" (K planted:
the fix-up walks its dirty list), "scan" (K planted and the list marked full:
the fix-up's fallback scan of all B state words).  Run under
`rocprofv3 --kernel-trace --stats`: the k_rx_int32_fixup launches come in
that order (10 + 10 + 10), so their durations split by mode; the script also
prints the per-call event time and checks every output against the input.
Usage: int32_fixup_conflicts.py [K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import switchml_amd as sw  # noqa: E402


def claim_tag(call, f):
    """k_rx_int32's claim tag (sml_frames.hip rx_int32_tag) as a signed int64."""
    t = ((0xFFFFFFFF - call) << 32) | ((0x7FFFFFFF - f) << 1)
    return int(np.array(t, dtype=np.uint64).view(np.int64))


def main(K=1000, reps=10):
    dev = torch.device("cuda", 0)
    P, n = 256, 64 << 20
    B = sw.num_blocks(n, P)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = torch.randint(-2 ** 31, 2 ** 31, (n,), dtype=torch.int64, device=dev, generator=g).to(torch.int32)
    fp = sw.frame_params(job_id=3)
    frames = sw.pack_frames_int32(x, fp, P)
    rx = sw.RxSliceInt32(n, P, device=dev)
    stolen = torch.from_numpy(np.sort(np.random.default_rng(1).choice(B, K, replace=False))).to(dev)
    tags = torch.tensor([claim_tag(0, B + int(k)) for k in stolen.tolist()], dtype=torch.int64, device=dev)
    out = {"numel": n, "packet_numel": P, "B": B, "K": K}
    for mode in ("clean", "list", "scan"):
        ts = []
        for _ in range(reps):
            rx.reset()
            rx.out.fill_(-1)
            if mode != "clean":
                rx.state[stolen] = tags
            if mode == "scan":
                rx.state[B + 3] = B
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            sw.unpack_frames_int32(frames, B, rx, job_id=3)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
            assert torch.equal(rx.out, x), mode
            assert rx.conflicts == (0 if mode == "clean" else K), (mode, rx.conflicts)
        out[mode] = {"call_us_median": round(float(np.median(ts)), 2), "call_us": [round(t, 2) for t in ts]}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:2]))
