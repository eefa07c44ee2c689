#!/usr/bin/env python3
"""Per-launch time of K1 vs the number of back-to-back launches (1..50) and
the XCD order, one GPU — why an event-timed run of 50 launches and a 10-launch
A/B disagree.  Rounds interleave every configuration; medians reported."""
import json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
import torch  # noqa: E402
import switchml_amd as sw  # noqa: E402

N, P = 64 << 20, 256
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev); gen.manual_seed(42)
x = torch.randn(N, device=dev, generator=gen)
B = sw.num_blocks(N, P)
payload = torch.empty(B * P, dtype=torch.int32, device=dev)
exps = torch.empty(B, dtype=torch.int8, device=dev)
st = torch.cuda.current_stream()
fn = lambda: sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=st)
res = {}
for r in range(int(os.environ.get("ROUNDS", 5))):
    for chunk in (0, 64):
        sw.set_xcd_chunk(chunk)
        for reps in (1, 2, 5, 10, 20, 50):
            for warm in (0, 1, 10):
                for _ in range(warm):
                    fn()
                if os.environ.get("SYNC_BEFORE", "0") == "1":
                    torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                torch.cuda.synchronize()
                res.setdefault(f"chunk{chunk} warm{warm} reps{reps}", []).append(a.elapsed_time(b) / reps * 1e3)
                time.sleep(0.002)
out = {k: round(statistics.median(v), 2) for k, v in res.items()}
print(json.dumps(out, indent=1))
