#!/usr/bin/env python3
"""K1 on cold HBM: payload store policy and tile size, interleaved in one
process (round 3: the headline now cycles 4 distinct buckets).

Variants (library knobs, bytes identical for all — tested):
  thr=default  default-policy payload stores for planes up to 256 MiB
               (sml_set_payload_nt_threshold default), non-temporal above
  thr=0        non-temporal payload stores at every size
  tiles=4/2    sml_set_quantize_tile_slices
For each bucket size: `cycle` = steps cycling 4 distinct buckets + planes
(the bench's headline pattern), `resident` = one bucket re-read every step.
Medians of interleaved rounds of HIP-event-timed launch runs.
Usage: python tools/ab_cold_policy.py OUT.json"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]
import switchml_amd as sw  # noqa: E402

VARIANTS = [("thr=default,tiles=4", None, 4), ("thr=0,tiles=4", 0, 4),
            ("thr=default,tiles=2", None, 2), ("thr=0,tiles=2", 0, 2)]


def main_k4(rounds=7):
    """K4 (dequantize) and the fused round trip under the same two policies
    (their fp32 output plane follows the same threshold)."""
    default_thr = sw.set_payload_nt_threshold(1 << 62)
    sw.set_payload_nt_threshold(default_thr)
    st = torch.cuda.current_stream()
    P = 256
    res = {}
    for mib in (64, 128, 256):
        N = mib << 18
        B = N // P
        nb = 4 if mib >= 256 else 8
        xs = [torch.randn(N, device="cuda") for _ in range(nb)]
        pls, exs = [], []
        for x in xs:
            pl, ex = sw.quantize_pack(x, P, 1, stream=st)
            pls.append(pl)
            exs.append(ex)
        outs = [torch.empty_like(x) for x in xs]
        kern = {"k4": lambda i: sw.dequantize(pls[i], exs[i], N, P, 1, out=outs[i], stream=st),
                "roundtrip": lambda i: sw.roundtrip_loopback(xs[i], P, 1, out=outs[i], stream=st)}
        times = {}
        reps = max(40, 160 * 64 // mib)
        for _ in range(rounds):
            for name, thr in (("thr=default", default_thr), ("thr=0", 0)):
                sw.set_payload_nt_threshold(thr)
                for kn, fn in kern.items():
                    for pat in ("cycle", "resident"):
                        k = nb if pat == "cycle" else 1
                        for i in range(2 * k):
                            fn(i % k)
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record(st)
                        for i in range(reps):
                            fn(i % k)
                        b.record(st)
                        torch.cuda.synchronize()
                        times.setdefault(f"{kn} {name} {pat}", []).append(a.elapsed_time(b) / reps * 1e3)
        res[f"{mib}MiB"] = {k: {"median_us": round(statistics.median(v), 2),
                                "TBps": round(8 * N / statistics.median(v) / 1e6, 3)} for k, v in times.items()}
        del xs, pls, exs, outs
        torch.cuda.empty_cache()
    sw.set_payload_nt_threshold(default_thr)
    return res


def main(out_path=None, rounds=7):
    sw.lib()
    if os.environ.get("AB_ONLY_K4"):
        print(json.dumps(main_k4(rounds), indent=1))
        return
    default_thr = sw.set_payload_nt_threshold(1 << 62)
    sw.set_payload_nt_threshold(default_thr)
    st = torch.cuda.current_stream()
    P = 256
    res = {}
    for mib in (64, 128, 256):
        N = mib << 18
        B = N // P
        nb = 4 if mib >= 256 else 8       # every pattern's working set well past the 256 MiB MALL
        xs = [torch.randn(N, device="cuda") for _ in range(nb)]
        pls = [torch.empty(B * P, dtype=torch.int32, device="cuda") for _ in range(nb)]
        exs = [torch.empty(B, dtype=torch.int8, device="cuda") for _ in range(nb)]
        ref = None
        for name, thr, tiles in VARIANTS:          # same bytes under every variant
            sw.set_payload_nt_threshold(default_thr if thr is None else thr)
            sw.set_quantize_tile_slices(tiles)
            sw.quantize_pack(xs[0], P, 1, payload=pls[0], exps_out=exs[0], stream=st)
            torch.cuda.synchronize()
            cur = pls[0].clone()
            ref = cur if ref is None else ref
            assert torch.equal(ref, cur), name
        del ref, cur
        times = {(n, pat): [] for n, _, _ in VARIANTS for pat in ("cycle", "resident")}
        reps = max(40, 160 * 64 // mib)
        for _ in range(rounds):
            for name, thr, tiles in VARIANTS:
                sw.set_payload_nt_threshold(default_thr if thr is None else thr)
                sw.set_quantize_tile_slices(tiles)
                for pat in ("cycle", "resident"):
                    k = nb if pat == "cycle" else 1
                    for i in range(2 * k):
                        sw.quantize_pack(xs[i % k], P, 1, payload=pls[i % k], exps_out=exs[i % k], stream=st)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for i in range(reps):
                        sw.quantize_pack(xs[i % k], P, 1, payload=pls[i % k], exps_out=exs[i % k], stream=st)
                    b.record(st)
                    torch.cuda.synchronize()
                    times[(name, pat)].append(a.elapsed_time(b) / reps * 1e3)
        alg = 8 * N + B
        res[f"{mib}MiB"] = {f"{n} {pat}": {"median_us": round(statistics.median(v), 2),
                                           "TBps": round(alg / statistics.median(v) / 1e6, 3)}
                            for (n, pat), v in times.items()}
        del xs, pls, exs
        torch.cuda.empty_cache()
    sw.set_payload_nt_threshold(default_thr)
    sw.set_quantize_tile_slices(0)
    s = json.dumps({"default_nt_threshold_bytes": default_thr, "results": res,
                    "k4_and_roundtrip": main_k4(rounds)}, indent=1)
    print(s)
    if out_path:
        with open(out_path, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main(*(sys.argv[1:2]))
