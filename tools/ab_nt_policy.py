#!/usr/bin/env python3
"""Output store policy of K1, K4 (dequantize) and the fused round trip by
bucket size, in one process with the product library: default-policy vs
non-temporal output stores (sml_set_payload_nt_threshold never / always),
one bucket re-read every step at 256 MiB / 512 MiB / 1 GiB.  Interleaved
rounds, medians; outputs checked equal across policies."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402

NEVER, ALWAYS = 2 ** 64 - 1, 0


def main(rounds=7):
    P, W = 256, 1
    st = torch.cuda.current_stream()
    out = {}
    for mib in (256, 512, 1024):
        N = mib << 18
        x = torch.randn(N, device="cuda")
        pl, ex = sw.quantize_pack(x, P, W)
        y = torch.empty_like(x)
        fns = {"K1": lambda: sw.quantize_pack(x, P, W, payload=pl, exps_out=ex, stream=st),
               "K4": lambda: sw.dequantize(pl, ex, N, P, W, out=y, stream=st),
               "roundtrip": lambda: sw.roundtrip_loopback(x, P, W, out=y, stream=st)}
        ref = {}
        for pol in (NEVER, ALWAYS):
            sw.set_payload_nt_threshold(pol)
            for k, fn in fns.items():
                fn()
                torch.cuda.synchronize()
                cur = (pl if k == "K1" else y).clone()
                if k in ref:
                    assert torch.equal(ref[k], cur), (mib, k)
                else:
                    ref[k] = cur
        del ref, cur
        reps = max(8, 40 * 256 // mib)
        res = {(k, p): [] for k in fns for p in ("default", "nt")}
        for _ in range(rounds):
            for k, fn in fns.items():
                for pname, pol in (("default", NEVER), ("nt", ALWAYS)):
                    sw.set_payload_nt_threshold(pol)
                    for _ in range(4):
                        fn()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for _ in range(reps):
                        fn()
                    b.record(st)
                    torch.cuda.synchronize()
                    res[(k, pname)].append(a.elapsed_time(b) / reps * 1e3)
        alg = 8 * N + N // P
        out[f"{mib}MiB"] = {f"{k} {p}": {"median_us": round(statistics.median(v), 2),
                                         "TBps": round(alg / statistics.median(v) / 1e6, 3)} for (k, p), v in res.items()}
        del x, pl, ex, y
        torch.cuda.empty_cache()
    sw.set_payload_nt_threshold((256 << 20) + 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
