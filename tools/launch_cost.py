#!/usr/bin/env python3
"""Host cost of one Python/ctypes launch of sml_quantize_pack (tiny input,
1000 launches, no sync inside the loop): shows the bench's eager launch path
cannot starve the GPU (8.5 us per launch on the MI355X box vs a 75 us kernel)."""
import sys, time, os
sys.path.insert(0, "p4app-switchml_amd")
import torch, switchml_amd as sw
dev = torch.device("cuda:0")
x = torch.randn(4096, device=dev)
B = sw.num_blocks(4096, 256)
p = torch.empty(B*256, dtype=torch.int32, device=dev); e = torch.empty(B, dtype=torch.int8, device=dev)
st = torch.cuda.current_stream()
for _ in range(100): sw.quantize_pack(x, 256, 1, payload=p, exps_out=e, stream=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(1000): sw.quantize_pack(x, 256, 1, payload=p, exps_out=e, stream=torch.cuda.current_stream())
t1 = time.perf_counter()
torch.cuda.synchronize()
print("host us per python launch:", (t1 - t0) * 1e3, "(of 1000 calls, /1000 -> us)", (t1-t0)/1000*1e6)
