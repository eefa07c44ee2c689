"""Prints the first payload bytes of an INT32 frame set, GPU vs oracle (debug)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402
from oracle import oracle as O  # noqa: E402

for n, P in ((1, 64), (300, 256), (8, 64)):
    x = np.arange(1, n + 1, dtype=np.int32) * 0x01020304
    fp = sw.frame_params(job_id=9)
    ref = O.build_frames_i32(x, fp, P=P)
    got = sw.pack_frames_int32(torch.from_numpy(x).cuda(), fp, P).cpu().numpy()
    torch.cuda.synchronize()
    print(n, P, "got", got[44:84].tolist())
    print(n, P, "ref", ref[44:84].tolist())
    bad = np.nonzero(got != ref)[0]
    print("bad bytes", bad[:40].tolist(), "count", bad.size)
