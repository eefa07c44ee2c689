"""Debug: Context::AllReduce of a 5 GiB device tensor vs per-slice round
trips (tests/test_large_gpu.py::test_client_allreduce_past_4GiB), with the
input checked before/after and the mismatch located per FIFO slice."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
sys.path.insert(0, ROOT)
import torch
import switchml_amd as sw
from switchml_amd import client as C

N = 5 * 2 ** 28 + 333
P = 256
mode = sys.argv[1] if len(sys.argv) > 1 else "fused"
n = int(sys.argv[2]) if len(sys.argv) > 2 else N
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(20240)
x = torch.randn(n, device=dev, generator=g) * 3.0
x0 = x.clone()
out = torch.empty_like(x)
T, Wc = 4, 2
C.start(C.make_config(num_workers=Wc, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                      mode=mode, bandwidth=0))
try:
    C.allreduce(x, out)
finally:
    C.stop()
torch.cuda.synchronize()
print("x unchanged:", torch.equal(x, x0))
ref = torch.empty_like(x)
for t in range(T):
    q, r = divmod(n, T)
    m = q + (t < r)
    off = t * m if t < r else t * m + r
    sw.roundtrip_loopback(x0[off:off + m], P, Wc, out=ref[off:off + m])
    torch.cuda.synchronize()
    eq = torch.equal(out[off:off + m].view(torch.int32), ref[off:off + m].view(torch.int32))
    ne = (out[off:off + m].view(torch.int32) != ref[off:off + m].view(torch.int32)).nonzero()
    print(f"slice {t} off {off} m {m}: equal {eq} mismatches {ne.numel()} first {ne[:3].flatten().tolist()} "
          f"x {x0[off:off+3].tolist()} out {out[off:off+3].tolist()} ref {ref[off:off+3].tolist()}", flush=True)
