#!/usr/bin/env python3
"""The in-node switch's multicast on one GPU: W shards of S words gathered
by W sequential sml_copy_words launches (the old Gather) against one
sml_copy_segments launch.  One GPU has no xGMI links, so this checks only
that the single launch streams at the copy rate; across GPUs it is what
lets the W peers' links run at once."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]
import ctypes  # noqa: E402
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(W=8, S=8 << 20, rounds=9, reps=10):
    src = torch.randint(0, 1 << 30, (W * S,), dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    L = sw.lib()
    L.sml_copy_words.restype = ctypes.c_int
    L.sml_copy_words.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    pairs = [(src[w * S:(w + 1) * S], dst[w * S:(w + 1) * S]) for w in range(W)]

    def seq():
        for s, d in pairs:
            assert L.sml_copy_words(s.data_ptr(), d.data_ptr(), S, st.cuda_stream) == 0

    def one():
        sw.copy_segments(pairs, stream=st)

    res = {"sequential_copy_words": [], "copy_segments": []}
    for _ in range(rounds):
        for name, fn in (("sequential_copy_words", seq), ("copy_segments", one)):
            fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(b) / reps * 1e3)
    assert torch.equal(src, dst)
    nbytes = 2 * 4 * W * S
    print(json.dumps({"what": f"{W} shards of {S} words: gather by {W} launches vs one", **{
        k: {"median_us": round(statistics.median(v), 2), "GBps": round(nbytes / statistics.median(v) / 1e3, 1)}
        for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
