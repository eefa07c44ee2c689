"""Peer-to-peer switch: W workers (one process per GPU) aggregate through
each other's HBM over xGMI instead of through a ring all-reduce.

The Tofino switch gives every worker the slot-wise wrapping sum of the W
workers' payload words and the signed int8 max of their exponents
(p4/processor.p4:48-54, p4/exponents.p4:48-54).  Here each worker keeps its
BE payload plane (the wire words of its packets) in its own HBM, maps every
peer's plane once (hipIpc handles, sml_ipc_*), and per all-reduce:

  K2 exponents --all_reduce MAX (B bytes)--> global exps
  K3 quantize with the global exps -> own BE payload plane        | barrier
  K6 on this rank's shard of blocks: read the W peers' planes over xGMI,
     wrapping sum + fused dequantize -> fp32 shard of `out`       | barrier
  all_gather of the fp32 shards -> every rank holds the whole bucket

So the payload exchange is one-shot over all point-to-point links at once:
each rank pulls (W-1)/W of its shard's payload from the peers in parallel
(every xGMI link busy), instead of the ring's 2(W-1) dependent steps.  The
result is bit-identical to SwitchSimAllReduce (and to the oracle switch).

Shards: block ranges of S = ceil(B / W) blocks, rank r owns blocks
[r*S, min((r+1)*S, B)); `out` is padded to W*S*P elements internally so the
all-gather moves equal shards.

Every wait is bounded (the round-4 hang): the host waits for
the device at each hand-off by polling an event against `sync_timeout`
(a named TimeoutError, never an unbounded stream synchronize); the rendezvous
collectives carry the process group's timeout; and a rank whose peer mapping
fails says so to its peers in the same collective that publishes the
mappings, so every rank raises together instead of one of them waiting in
the next barrier for a peer that has already given up.
"""
from __future__ import annotations

import ctypes
import os
import time

import torch
import torch.distributed as dist

from . import (FLAG_PEER_PLANES, _check, bswap_i32, exponents, lib, num_blocks, quantize_pack,
               release_to_peers, switch_aggregate)


def shard_blocks(num_blocks: int, world: int, rank: int) -> tuple[int, int]:
    """(first block, block count) of `rank`'s shard: S = ceil(B / W) blocks
    per rank, the last shards shorter or empty."""
    S = -(-num_blocks // world)
    blk0 = min(rank * S, num_blocks)
    return blk0, max(0, min(S, num_blocks - blk0))


def _handle_of(t: torch.Tensor):
    L = lib()
    buf = (ctypes.c_uint8 * L.sml_ipc_handle_bytes())()
    off = ctypes.c_uint64()
    _check("sml_ipc_get_handle", L.sml_ipc_get_handle(ctypes.c_void_p(t.data_ptr()), buf, ctypes.byref(off)))
    return bytes(buf), off.value


class _PeerPlane:
    """A peer's int32 plane mapped into this process (a raw device pointer)."""

    def __init__(self, handle: bytes, offset: int):
        L = lib()
        buf = (ctypes.c_uint8 * len(handle)).from_buffer_copy(handle)
        base = ctypes.c_void_p()
        _check("sml_ipc_open_handle", L.sml_ipc_open_handle(buf, ctypes.byref(base)))
        self.base = base.value
        self.ptr = base.value + offset

    def close(self):
        if self.base:
            _check("sml_ipc_close_handle", lib().sml_ipc_close_handle(ctypes.c_void_p(self.base)))
            self.base = None


class _Ptr:
    """Duck-typed int32 plane for switch_aggregate: a raw device pointer."""
    dtype = torch.int32
    is_cuda = True

    def __init__(self, ptr: int, numel: int, device):
        self._ptr, self._n, self.device = ptr, numel, device

    def data_ptr(self):
        return self._ptr

    def numel(self):
        return self._n

    def is_contiguous(self):
        return True

    def is_pinned(self):
        return False


def wait_device(stream: torch.cuda.Stream, what: str, timeout_s: float) -> None:
    """Wait until the work queued on `stream` so far has finished, or raise
    TimeoutError naming `what` after timeout_s (a device that never finishes
    is reported, not waited on forever)."""
    ev = torch.cuda.Event()
    ev.record(stream)
    t0 = time.monotonic()
    # spin like a stream synchronize for the first 100 ms (the hand-offs this
    # guards take micro- to milliseconds: a sleep's wake-up latency would be
    # timed into every all-reduce), then back off
    spin_until = t0 + 0.1
    while not ev.query():
        now = time.monotonic()
        if now - t0 > timeout_s:
            raise TimeoutError(f"p2p switch: device work before '{what}' not finished after {timeout_s:g} s")
        if now > spin_until:
            time.sleep(1e-3)


def _sync_timeout_default() -> float:
    return float(os.environ.get("SML_P2P_SYNC_TIMEOUT_S", "120"))


class PeerSwitchAllReduce:
    """Reusable planes + peer mappings for repeated all-reduces of one bucket
    size.  Needs one GPU per rank (or ranks sharing one GPU, for tests) and a
    process group whose backend can all_reduce int8 and all_gather fp32
    tensors on the device ("nccl" = RCCL); with "gloo" those two small /
    final collectives go through host memory (CPU tests of the plumbing).
    sync_timeout: seconds any host wait for this rank's device work may take
    (default SML_P2P_SYNC_TIMEOUT_S or 120)."""

    def __init__(self, numel: int, packet_numel: int = 256, device=None, group=None,
                 sync_timeout: float | None = None):
        self.numel, self.P, self.group = numel, packet_numel, group
        self.sync_timeout = _sync_timeout_default() if sync_timeout is None else float(sync_timeout)
        self.peers = {}
        self.W = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.B = num_blocks(numel, packet_numel)
        self.S = -(-self.B // self.W)
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.host_collectives = dist.get_backend(group) == "gloo"
        self.exps = torch.empty(self.B, dtype=torch.int8, device=self.dev)
        self.payload = torch.empty(self.B * packet_numel, dtype=torch.int32, device=self.dev)
        self.out_pad = torch.empty(self.W * self.S * packet_numel, dtype=torch.float32, device=self.dev)
        self.phases = None      # diagnostics: see SwitchSimAllReduce.phases
        wait_device(torch.cuda.current_stream(self.dev), "publish planes", self.sync_timeout)
        # publish this rank's plane; a rank that cannot export still takes
        # part in the collective (with its error), so no peer waits on it
        try:
            mine = ("ok",) + _handle_of(self.payload)
        except Exception as e:  # noqa: BLE001 - reported to every rank below
            mine = ("error", repr(e)[:300], 0)
        allh = [None] * self.W
        dist.all_gather_object(allh, mine, group=group)
        err = None
        bad = [(w, h[1]) for w, h in enumerate(allh) if h[0] != "ok"]
        if bad:
            err = f"rank(s) could not export their plane: {bad}"
        else:
            try:
                for w, (_, h, off) in enumerate(allh):
                    if w != self.rank:
                        self.peers[w] = _PeerPlane(h, off)
            except Exception as e:  # noqa: BLE001
                err = f"rank {self.rank} could not map a peer plane: {e!r}"[:300]
        # agree on the outcome before anyone uses (or gives up on) the mappings
        verdicts = [None] * self.W
        dist.all_gather_object(verdicts, err, group=group)
        errs = [v for v in verdicts if v]
        if errs:
            self._unmap()
            raise RuntimeError("PeerSwitchAllReduce setup failed: " + "; ".join(errs))

    def _plane(self, w: int, blk0: int, nblk: int):
        if w == self.rank:
            return self.payload[blk0 * self.P:(blk0 + nblk) * self.P]
        return _Ptr(self.peers[w].ptr + blk0 * self.P * 4, nblk * self.P, self.dev)

    def _barrier(self, release: bool = True):
        """Hand-off to the peers: release this GPU's writes to
        system scope (L2 written back), wait for them, meet the peers; the
        kernels that then read peer planes acquire (FLAG_PEER_PLANES)."""
        if release:
            release_to_peers(device=self.dev)
        wait_device(torch.cuda.current_stream(self.dev), "barrier", self.sync_timeout)
        dist.barrier(group=self.group)

    def _mark(self, name: str):
        if self.phases is not None:
            wait_device(torch.cuda.current_stream(self.dev), name, self.sync_timeout)
            self.phases[name] = time.perf_counter()

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """All-reduce (SUM) of a FLOAT32 bucket (quantized, as the exponent
        quantizer PPP does) or an INT32 bucket (byte order only: ppp.cc:158-190,
        262-298; no exponents, no extra batch)."""
        if self.peers is None:
            raise RuntimeError("PeerSwitchAllReduce is closed")
        if x.numel() != self.numel:
            raise ValueError("bucket size changed; build a new PeerSwitchAllReduce")
        if x.dtype not in (torch.float32, torch.int32):
            raise TypeError("FLOAT32 or INT32 buckets only (common.h:51-55)")
        if out is None:
            out = torch.empty_like(x)
        if out.dtype != x.dtype:
            raise TypeError("out must have the bucket's dtype")
        P, S = self.P, self.S
        is_int = x.dtype == torch.int32
        self._mark("start")
        if is_int:
            bswap_i32(x, out=self.payload[:self.numel])                         # INT32 PPP: wire words
        else:
            exponents(x, P, out=self.exps)                                      # K2
            if self.host_collectives:
                e = self.exps.cpu()
                dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.group)
                self.exps.copy_(e)
            else:
                dist.all_reduce(self.exps, op=dist.ReduceOp.MAX, group=self.group)  # switch: int8 max
            quantize_pack(x, P, self.W, global_exps=self.exps, payload=self.payload)  # K3, BE wire words
        self._barrier()                                                         # every plane written
        self._mark("k2_max_k3")
        blk0, nblk = shard_blocks(self.B, self.W, self.rank)
        # gather straight into `out` when the shards tile it exactly
        pad = self.out_pad.view(torch.int32) if is_int else self.out_pad
        dst = out if out.numel() == self.W * S * P and out.is_contiguous() else pad
        shard = dst[self.rank * S * P:(self.rank + 1) * S * P]
        if nblk:
            n_el = min(nblk * P, self.numel - blk0 * P)
            planes = [self._plane(w, blk0, nblk) for w in range(self.W)]
            if is_int:
                # the switch's wrapping sum of the BE words, then ntohl
                switch_aggregate(planes, None, nblk * P, P, payload_out=shard[:nblk * P], flags=FLAG_PEER_PLANES)
                bswap_i32(shard[:n_el], out=shard[:n_el])
            else:
                ex = self.exps[blk0:blk0 + nblk]
                switch_aggregate(planes, [ex] * self.W, n_el, P, out=shard[:n_el],
                                 flags=FLAG_PEER_PLANES)                        # K6 over xGMI
        self._barrier(release=False)                                            # peers done reading
        self._mark("k6")
        if self.host_collectives:
            parts = [torch.empty(S * P, dtype=dst.dtype) for _ in range(self.W)]
            dist.all_gather(parts, shard.cpu(), group=self.group)
            dst.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(dst, shard, group=self.group)
        if dst is not out:
            out.copy_(dst[:self.numel])
        self._mark("gather")
        return out

    def _unmap(self) -> list:
        """Close every peer mapping; return the errors (each is attempted)."""
        errs = []
        for w, p in self.peers.items():
            try:
                p.close()
            except Exception as e:  # noqa: BLE001
                errs.append(f"peer {w}: {e!r}"[:200])
        self.peers = {}
        return errs

    def close(self):
        """Unmap the peers' planes; collective (every rank calls it), so no
        rank frees its own plane while a peer still has it mapped: this
        rank's reads of the peers' planes are done before its mappings go,
        and the closing barrier holds every plane until all peers have
        unmapped it.  Idempotent."""
        if self.peers is None:
            return
        wait_device(torch.cuda.current_stream(self.dev), "close", self.sync_timeout)
        errs = self._unmap()
        self.peers = None
        dist.barrier(group=self.group)
        if errs:
            raise RuntimeError("PeerSwitchAllReduce.close: " + "; ".join(errs))
