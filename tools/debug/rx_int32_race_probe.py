#!/usr/bin/env python3
"""How often does a later copy of a pkt_id claim it before an earlier copy in
the one-pass INT32 rx (k_rx_int32)?  Streams of the slice's frames plus
altered copies at random distances (tests/test_frames_int32.py's
altered_copies_stream), under several grid limits and XCD chunkings; prints
the slice's conflict total (copies resolved by the fix-up) and whether the
output equals the sequential first-copy-wins loop."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_frames_int32 import altered_copies_stream, int32_data, python_rx  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    P, n = 256, 8 * 1024 * 1024
    fp = sw.frame_params(job_id=5)
    x = int32_data(1, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    out = []
    for gap in (16, 256, 4096):
        s = altered_copies_stream(O.build_frames_i32(x, fp, P=P), B, fb, seed=gap, pairs=8000, max_gap=gap)
        nfr = s.size // fb
        seen = np.zeros(B, dtype=np.uint8)
        ref = np.zeros(n, dtype=np.int32)
        python_rx(s, fb, n, P, 5, seen, ref)
        sd = torch.from_numpy(s).to(dev)
        for lim, xcd in ((0, 64), (0, 0), (8, 0), (64, 0), (256, 64)):
            old_lim, old_xcd = sw.set_grid_limit(lim), sw.set_xcd_chunk(xcd)
            try:
                rx = sw.RxSliceInt32(n, P, device=dev)
                rx.reset()
                sw.unpack_frames_int32(sd, nfr, rx, job_id=5)
                torch.cuda.synchronize()
                ok = bool(np.array_equal(rx.out.cpu().numpy(), ref))
                out.append({"max_gap": gap, "grid_limit": lim, "xcd_chunk": xcd, "conflicts": rx.conflicts,
                            "equal": ok})
                print(out[-1], flush=True)
            finally:
                sw.set_grid_limit(old_lim)
                sw.set_xcd_chunk(old_xcd)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
