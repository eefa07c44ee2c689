#!/usr/bin/env python3
"""K1 vs K3 under rocprofv3 (name K3's gap with counters).

Launches, on one resident 256 MiB bucket (P = 256, W = 1):
  K1  sml_quantize_pack fused (local exponents, writes exps)      x reps
  K3  sml_quantize_pack with global exponents (K1's exps plane)   x reps
  K3b K3 reading a global-exponent plane that is NOT resident in L2
      (a second plane, alternated) — whether the exponent reads miss
interleaved, so clocks are shared.  Run it under rocprofv3 --kernel-trace
--stats and separate --pmc passes (tools/gpujobs/*.sh); tools/k3_counters.py
reduces the CSVs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]

import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402


def main(reps=int(os.environ.get("K3_REPS", "40")), N=64 << 20, P=256):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.randn(N, device=dev, generator=g)
    B = sw.num_blocks(N, P)
    pl = torch.empty(B * P, dtype=torch.int32, device=dev)
    e1 = torch.empty(B, dtype=torch.int8, device=dev)
    e2 = torch.empty(B, dtype=torch.int8, device=dev)
    st = torch.cuda.current_stream()
    sw.quantize_pack(x, P, 1, payload=pl, exps_out=e1, stream=st)
    e2.copy_(e1)
    for _ in range(20):   # clock settle
        sw.quantize_pack(x, P, 1, payload=pl, exps_out=e1, stream=st)
    for i in range(reps):
        sw.quantize_pack(x, P, 1, payload=pl, exps_out=e1, stream=st)                     # K1
        sw.quantize_pack(x, P, 1, global_exps=e1 if i % 2 == 0 else e2, payload=pl, stream=st)  # K3
    torch.cuda.synchronize()
    print("prof_k3 done", reps)


if __name__ == "__main__":
    main()
