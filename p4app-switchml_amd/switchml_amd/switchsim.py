"""Switch-sim mode: W real workers (one process per GPU) with RCCL over xGMI
standing in for the Tofino switch.

The switch's per-slot arithmetic (dev_root/p4):
  * exponents: signed int8 max over workers   (p4/exponents.p4:48-54, types.p4:119)
  * payload:   bit<32> wrapping sum over workers (p4/processor.p4:48-54)
and the result is multicast back to every worker.  Here that is one
all_reduce(MAX) on the int8 exponent plane and one all_reduce(SUM) on the
int32 payload plane (RCCL's int32 sum wraps like bit<32>).  The switch
parses big-endian words; RCCL cannot add big-endian words, so the payload
plane is produced in host order for the exchange (SML_FLAG_PAYLOAD_LE) — the
values summed are identical (tests check the BE wire words separately).

The reference pipelines this per packet with a one-batch exponent
look-ahead (ppp.cc:115-156, dummy_worker_thread.cc:106-163); with planes the
look-ahead becomes two exchange steps:

   K2 exponents --all_reduce MAX--> global exps --K3 quantize (x scale(W, e))-->
   LE payload --all_reduce SUM--> K4 dequantize -> out  (= sum over workers)

The exchange functions are plain torch.distributed calls and work on any
backend/device ("nccl" = RCCL on ROCm for GPU tensors; "gloo" for CPU tests).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from . import FLAG_PAYLOAD_LE, dequantize, exponents, num_blocks, quantize_pack


def exchange_exponents(exps: torch.Tensor, group=None) -> torch.Tensor:
    """The switch's signed int8 max of the per-packet exponents, in place."""
    if exps.dtype != torch.int8:
        raise TypeError("exponent plane must be int8")
    dist.all_reduce(exps, op=dist.ReduceOp.MAX, group=group)
    return exps


def exchange_payload(payload_le: torch.Tensor, group=None) -> torch.Tensor:
    """The switch's wrapping int32 sum of host-order payload words, in place."""
    if payload_le.dtype != torch.int32:
        raise TypeError("payload plane must be int32")
    dist.all_reduce(payload_le, op=dist.ReduceOp.SUM, group=group)
    return payload_le


class SwitchSimAllReduce:
    """Reusable planes for repeated switch-sim all-reduces of one bucket size
    (the GPU analogue of a worker's packet ring; allocate once, reuse)."""

    def __init__(self, numel: int, packet_numel: int = 256, device=None, group=None):
        self.numel = numel
        self.P = packet_numel
        self.group = group
        self.W = dist.get_world_size(group)
        self.B = num_blocks(numel, packet_numel)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.exps = torch.empty(self.B, dtype=torch.int8, device=dev)
        self.payload = torch.empty(self.B * packet_numel, dtype=torch.int32, device=dev)
        # diagnostics: a dict here makes the next call record host times at
        # its phase boundaries (each after a stream sync) — bench.py's breakdown
        self.phases = None

    def _mark(self, name: str, x: torch.Tensor):
        if self.phases is not None:
            torch.cuda.current_stream(x.device).synchronize()
            self.phases[name] = time.perf_counter()

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """All-reduce (SUM) of a FLOAT32 bucket (quantized, as the exponent
        quantizer PPP does) or an INT32 bucket (the INT32 PPP only reorders
        bytes, ppp.cc:158-190, 262-298: htonl, the switch's wrapping sum,
        ntohl — the same words as a wrapping sum in host order)."""
        if x.numel() != self.numel:
            raise ValueError("bucket size changed; build a new SwitchSimAllReduce")
        if x.dtype not in (torch.float32, torch.int32):
            raise TypeError("FLOAT32 or INT32 buckets only (common.h:51-55)")
        if out is None:
            out = torch.empty_like(x)
        if out.dtype != x.dtype:
            raise TypeError("out must have the bucket's dtype")
        if x.dtype == torch.int32:
            plane = self.payload[:self.numel]
            plane.copy_(x)
            exchange_payload(plane, self.group)                              # switch: int32 sum
            out.copy_(plane)
            return out
        self._mark("start", x)
        exponents(x, self.P, out=self.exps)                                  # K2
        self._mark("k2", x)
        exchange_exponents(self.exps, self.group)                            # switch: int8 max
        self._mark("exps_max", x)
        quantize_pack(x, self.P, self.W, global_exps=self.exps, payload=self.payload,
                      flags=FLAG_PAYLOAD_LE)                                 # K3, LE words
        self._mark("k3", x)
        exchange_payload(self.payload, self.group)                           # switch: int32 sum
        self._mark("payload_sum", x)
        dequantize(self.payload, self.exps, self.numel, self.P, self.W, out=out,
                   flags=FLAG_PAYLOAD_LE)                                    # K4
        self._mark("k4", x)
        return out


def allreduce(x: torch.Tensor, packet_numel: int = 256, out=None, group=None) -> torch.Tensor:
    """One-shot switch-sim all-reduce (SUM) of a GPU fp32 bucket."""
    return SwitchSimAllReduce(x.numel(), packet_numel, x.device, group)(x, out)
