"""switchml_amd — Python front end of the MI355X-native SwitchML end-host
pre/post-processor (libswitchml_hip.so, C-ABI in include/switchml_hip.h).

Thin ctypes layer over the C-ABI for tests, bench and the torch.distributed
switch simulation.  Tensors are torch CUDA (HIP) tensors; every call is
enqueued on torch's current stream unless a stream is given.  There is no CPU
fallback: if the HIP library is missing or the tensor is not on the GPU, the
call raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libswitchml_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "switchml_hip.h")

SML_OK = 0
SML_ERR_INVALID_ARG = 1
SML_ERR_UNSUPPORTED = 2
SML_ERR_ALIGNMENT = 3
SML_ERR_HIP = 4

FLAG_PAYLOAD_LE = 0x1
FLAG_ROUND_RNE = 0x2
FLAG_PEER_PLANES = 0x4   # inputs written by other GPUs: acquire first (sml_release_to_peers on the writer)
FLAG_PROCESS_PACKET = 0x8   # sml_exchange_burst: the dummy backend's ProcessPacket (x W) on each packet first

PACKET_NUMELS = (64, 128, 256, 512, 1024)

_lib = None


class FrameParams(ctypes.Structure):
    """sml_frame_params (include/switchml_hip.h): addresses in network byte order."""
    _fields_ = [("dst_mac", ctypes.c_uint8 * 6), ("src_mac", ctypes.c_uint8 * 6),
                ("src_ip_be", ctypes.c_uint32), ("dst_ip_be", ctypes.c_uint32),
                ("src_port_be", ctypes.c_uint16), ("dst_port_be", ctypes.c_uint16),
                ("job_id", ctypes.c_uint64), ("pool_index_start", ctypes.c_uint32),
                ("pool_index_shift", ctypes.c_uint32), ("max_outstanding_pkts", ctypes.c_uint32)]


def frame_params(dst_mac=b"\x02\x00\x00\x00\x00\x01", src_mac=b"\x02\x00\x00\x00\x00\x02",
                 src_ip="10.0.0.1", dst_ip="10.0.0.253", src_port=4000, dst_port=48879, job_id=0,
                 pool_index_start=0, pool_index_shift=0, max_outstanding_pkts=64) -> FrameParams:
    import socket
    import struct
    fp = FrameParams()
    fp.dst_mac[:] = list(dst_mac)
    fp.src_mac[:] = list(src_mac)
    fp.src_ip_be = struct.unpack("<I", socket.inet_aton(src_ip))[0]
    fp.dst_ip_be = struct.unpack("<I", socket.inet_aton(dst_ip))[0]
    fp.src_port_be = socket.htons(src_port)
    fp.dst_port_be = socket.htons(dst_port)
    fp.job_id = job_id
    fp.pool_index_start = pool_index_start
    fp.pool_index_shift = pool_index_shift
    fp.max_outstanding_pkts = max_outstanding_pkts
    return fp


MAX_BURST = 64


class PacketBurst(ctypes.Structure):
    """sml_packet_burst (include/switchml_hip.h): up to MAX_BURST per-packet
    calls of one job slice in one launch."""
    _fields_ = [("in_", ctypes.c_void_p), ("out", ctypes.c_void_p), ("numel", ctypes.c_uint64),
                ("packet_numel", ctypes.c_uint32), ("num_workers", ctypes.c_uint16), ("data_type", ctypes.c_uint16),
                ("batch_num_ltus", ctypes.c_uint64), ("recv_exps", ctypes.c_void_p), ("count", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("pkt_ids", ctypes.c_uint64 * MAX_BURST),
                ("entries", ctypes.c_void_p * MAX_BURST), ("extras", ctypes.c_void_p * MAX_BURST)]


class SwitchMLError(RuntimeError):
    def __init__(self, fn: str, status: int):
        L = lib()
        msg = L.sml_status_string(status).decode()
        err = L.sml_last_error().decode()
        super().__init__(f"{fn} failed: {msg}" + (f" ({err})" if err else ""))
        self.status = status


def lib():
    """Load libswitchml_hip.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found — build it with `make -C p4app-switchml_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    u64, u32, u16, i32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int, ctypes.c_void_p
    L.sml_abi_version.restype = i32
    L.sml_status_string.restype = ctypes.c_char_p
    L.sml_status_string.argtypes = [i32]
    L.sml_last_error.restype = ctypes.c_char_p
    L.sml_num_blocks.restype = u64
    L.sml_num_blocks.argtypes = [u64, u32]
    L.sml_scale_lut.restype = i32
    L.sml_scale_lut.argtypes = [u16, vp]
    L.sml_scale_lut_device.restype = i32
    L.sml_scale_lut_device.argtypes = [u16, vp, vp]
    L.sml_exponents.restype = i32
    L.sml_exponents.argtypes = [vp, u64, u32, vp, vp]
    L.sml_quantize_pack.restype = i32
    L.sml_quantize_pack.argtypes = [vp, u64, u32, u16, vp, vp, vp, u32, vp]
    L.sml_dequantize.restype = i32
    L.sml_dequantize.argtypes = [vp, vp, u64, u32, u16, vp, u32, vp]
    L.sml_bswap_i32.restype = i32
    L.sml_bswap_i32.argtypes = [vp, vp, u64, vp]
    L.sml_loopback_aggregate.restype = i32
    L.sml_loopback_aggregate.argtypes = [vp, u64, u16, u32, vp]
    L.sml_roundtrip_loopback.restype = i32
    L.sml_roundtrip_loopback.argtypes = [vp, vp, u64, u32, u16, vp, vp, u32, vp]
    L.sml_roundtrip_loopback_batch.restype = i32
    L.sml_roundtrip_loopback_batch.argtypes = [vp, u32, u32, u16, u32, vp]
    L.sml_set_grid_limit.restype = u32
    L.sml_set_grid_limit.argtypes = [u32]
    L.sml_stream_copy.restype = i32
    L.sml_stream_copy.argtypes = [vp, vp, u64, vp]
    L.sml_rdma_imm.restype = i32
    L.sml_rdma_imm.argtypes = [vp, u64, u32, vp, vp]
    L.sml_rdma_imm_int32.restype = i32
    L.sml_rdma_imm_int32.argtypes = [u64, vp, vp]
    L.sml_debug_stall.restype = i32
    L.sml_debug_stall.argtypes = [u32, vp]
    L.sml_frame_bytes.restype = u64
    L.sml_frame_bytes.argtypes = [u32]
    L.sml_rx_state_words.restype = u64
    L.sml_rx_state_words.argtypes = [u64, u32, u32, i32]
    L.sml_quantize_pack_frames.restype = i32
    L.sml_quantize_pack_frames.argtypes = [vp, u64, u32, u16, vp, u32, ctypes.POINTER(FrameParams), vp, u64, vp]
    L.sml_set_quantize_tile_slices.restype = u32
    L.sml_set_quantize_tile_slices.argtypes = [u32]
    L.sml_set_stream_tile_slices.restype = u32
    L.sml_set_stream_tile_slices.argtypes = [u32]
    L.sml_set_payload_nt_threshold.restype = u64
    L.sml_set_payload_nt_threshold.argtypes = [u64]
    L.sml_set_xcd_chunk.restype = u32
    L.sml_set_xcd_chunk.argtypes = [u32]
    L.sml_dequantize_frames.restype = i32
    L.sml_dequantize_frames.argtypes = [vp, u64, u64, u64, u32, u16, u32, u64, vp, vp, vp, vp, vp]
    L.sml_rx_reset.restype = i32
    L.sml_rx_reset.argtypes = [vp, u64, vp]
    L.sml_pack_frames_int32.restype = i32
    L.sml_pack_frames_int32.argtypes = [vp, u64, u32, ctypes.POINTER(FrameParams), vp, u64, vp]
    L.sml_unpack_frames_int32.restype = i32
    L.sml_unpack_frames_int32.argtypes = [vp, u64, u64, u64, u32, u64, vp, vp, vp, vp]
    L.sml_switch_aggregate.restype = i32
    L.sml_switch_aggregate.argtypes = [vp, vp, u16, u64, u32, vp, vp, vp, u32, vp]
    L.sml_copy_segments.restype = i32
    L.sml_copy_segments.argtypes = [vp, vp, vp, u32, u32, vp]
    L.sml_switch_exps.restype = i32
    L.sml_switch_exps.argtypes = [vp, u16, u64, vp, u32, vp]
    L.sml_release_to_peers.restype = i32
    L.sml_release_to_peers.argtypes = [vp]
    L.sml_preprocess_burst.restype = i32
    L.sml_preprocess_burst.argtypes = [ctypes.POINTER(PacketBurst), vp]
    L.sml_postprocess_burst.restype = i32
    L.sml_postprocess_burst.argtypes = [ctypes.POINTER(PacketBurst), vp]
    L.sml_exchange_burst.restype = i32
    L.sml_exchange_burst.argtypes = [ctypes.POINTER(PacketBurst), vp]
    L.sml_burst_server_create.restype = i32
    L.sml_burst_server_create.argtypes = [u32, u32, u32, ctypes.POINTER(vp)]
    L.sml_burst_server_submit.restype = i32
    L.sml_burst_server_submit.argtypes = [vp, u32, ctypes.POINTER(PacketBurst)]
    L.sml_burst_server_destroy.restype = i32
    L.sml_burst_server_destroy.argtypes = [vp]
    L.sml_burst_server_stop.restype = i32
    L.sml_burst_server_stop.argtypes = [vp]
    L.sml_burst_server_start.restype = i32
    L.sml_burst_server_start.argtypes = [vp]
    L.sml_burst_server_inject_unanswered.restype = i32
    L.sml_burst_server_inject_unanswered.argtypes = [vp, u32, ctypes.POINTER(PacketBurst)]
    L.sml_ipc_handle_bytes.restype = u32
    L.sml_ipc_get_handle.restype = i32
    L.sml_ipc_get_handle.argtypes = [vp, vp, ctypes.POINTER(u64)]
    L.sml_ipc_open_handle.restype = i32
    L.sml_ipc_open_handle.argtypes = [vp, ctypes.POINTER(vp)]
    L.sml_ipc_close_handle.restype = i32
    L.sml_ipc_close_handle.argtypes = [vp]
    _lib = L
    return L


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the C-ABI header declares (for the export test)."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sml_[a-z0-9_]+)\s*\(", src)))


def _check(fn: str, status: int):
    if status != SML_OK:
        raise SwitchMLError(fn, status)


def num_blocks(numel: int, packet_numel: int = 256) -> int:
    return int(lib().sml_num_blocks(numel, packet_numel))


def fifo_slice(numel: int, num_slices: int, t: int) -> tuple[int, int]:
    """(offset, numel) of slice t of a job split num_slices ways — the FIFO
    scheduler's rule (client_lib/src/schedulers/fifo_scheduler.cc:93-109):
    the first numel % num_slices slices get one extra element.  Used for the
    multi-GPU sharding mode (slice g -> GPU g, as worker thread g would get it)."""
    if num_slices <= 0 or not 0 <= t < num_slices:
        raise ValueError("need 0 <= t < num_slices")
    n = numel // num_slices
    rem = numel % num_slices
    if t < rem:
        n += 1
        return t * n, n
    return t * n + rem, n


def shard_quantize_pack(job, rank: int, world: int, packet_numel: int = 256, num_workers: int = 1,
                        flags: int = 0, stream=None):
    """Sharding mode: K1 over this rank's FIFO slice of `job` (a 1-D fp32
    device tensor holding the whole job).  Returns (offset, payload, exps);
    blocks restart at the slice start, exactly as for worker thread `rank`
    of `world` (ppp.cc:54-62 per slice)."""
    off, n = fifo_slice(job.numel(), world, rank)
    payload, exps = quantize_pack(job[off:off + n], packet_numel, num_workers, flags=flags, stream=stream)
    return off, payload, exps


def set_grid_limit(max_workgroups: int) -> int:
    return int(lib().sml_set_grid_limit(max_workgroups))


def set_payload_nt_threshold(nbytes: int) -> int:
    """Payload planes (and K4 / round-trip outputs) of at least `nbytes`
    bytes take non-temporal stores (default 64 MiB, a quarter of the Infinity
    Cache; 2**64-1 = never, 0 = always); returns the previous threshold."""
    return int(lib().sml_set_payload_nt_threshold(nbytes))


def set_quantize_tile_slices(slices: int) -> int:
    """Slices of 256 elements per K1/K2/K3 wave tile: 4, 2 or 1 for every
    kernel (never below P/256), or 0 = the default, 2 slices for every kernel
    (never below P/256); returns the previous setting."""
    return int(lib().sml_set_quantize_tile_slices(slices))


def set_stream_tile_slices(slices: int) -> int:
    """Slices of 256 elements per K4 / fused round-trip wave tile: 4 or 2,
    or 0 = the default; returns the previous setting."""
    return int(lib().sml_set_stream_tile_slices(slices))


def set_xcd_chunk(chunk: int) -> int:
    """Workgroups per contiguous run on one XCD (0 = plain order); returns the previous value."""
    return int(lib().sml_set_xcd_chunk(chunk))


# ------------------------------------------------------------- torch glue --

def _torch():
    import torch
    return torch


def _stream(stream, like=None):
    """The HIP stream to launch on: the given one, else torch's current
    stream of `like`'s device (else of the current device)."""
    torch = _torch()
    if stream is None:
        dev = like.device if like is not None and getattr(like, "is_cuda", False) else None
        stream = torch.cuda.current_stream(dev)
    return ctypes.c_void_p(stream.cuda_stream)


def _dev(t, dtype, name):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not (t.is_cuda or t.is_pinned()):
        raise TypeError(f"{name} must be a CUDA (HIP) tensor or pinned host memory (read by the "
                        "kernel over PCIe) — the HIP path has no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def scale_lut(num_workers: int):
    import numpy as np
    out = np.empty(256, dtype=np.float32)
    _check("sml_scale_lut", lib().sml_scale_lut(num_workers, out.ctypes.data))
    return out


def scale_lut_device(num_workers: int, device="cuda", stream=None):
    torch = _torch()
    out = torch.empty(256, dtype=torch.float32, device=device)
    _check("sml_scale_lut_device", lib().sml_scale_lut_device(num_workers, _dev(out, torch.float32, "lut"), _stream(stream, out)))
    return out


def exponents(x, packet_numel: int = 256, out=None, stream=None):
    torch = _torch()
    B = num_blocks(x.numel(), packet_numel)
    if out is None:
        out = torch.empty(B, dtype=torch.int8, device=x.device)
    _check("sml_exponents", lib().sml_exponents(_dev(x, torch.float32, "x"), x.numel(), packet_numel,
                                                _dev(out, torch.int8, "exps"), _stream(stream, x)))
    return out


def quantize_pack(x, packet_numel: int = 256, num_workers: int = 1, global_exps=None,
                  payload=None, exps_out=None, want_exps: bool = True, flags: int = 0, stream=None):
    """Returns (payload int32[B*P] (BE words unless FLAG_PAYLOAD_LE), exps int8[B] or None)."""
    torch = _torch()
    B = num_blocks(x.numel(), packet_numel)
    if payload is None:
        payload = torch.empty(B * packet_numel, dtype=torch.int32, device=x.device)
    if global_exps is None and want_exps and exps_out is None:
        exps_out = torch.empty(B, dtype=torch.int8, device=x.device)
    g = None if global_exps is None else _dev(global_exps, torch.int8, "global_exps")
    e = None if exps_out is None else _dev(exps_out, torch.int8, "exps_out")
    _check("sml_quantize_pack", lib().sml_quantize_pack(
        _dev(x, torch.float32, "x"), x.numel(), packet_numel, num_workers, g,
        _dev(payload, torch.int32, "payload"), e, flags, _stream(stream, x)))
    return payload, (global_exps if global_exps is not None else exps_out)


def quantize_pack_launcher(x, packet_numel: int, num_workers: int, payload, exps_out=None, global_exps=None,
                           flags: int = 0, stream=None):
    """A zero-argument callable that launches sml_quantize_pack on these
    tensors: every argument checked and converted once, so a loop over the
    same bucket (a training step's gradient bucket, the bench's steps) pays
    one C call per launch instead of the wrapper's tensor checks.  The
    tensors must stay alive while the callable is used."""
    torch = _torch()
    B = num_blocks(x.numel(), packet_numel)
    if payload.numel() != B * packet_numel:
        raise ValueError(f"payload must hold B*P = {B * packet_numel} words")
    if exps_out is not None and exps_out.numel() != B:
        raise ValueError(f"exps_out must hold B = {B} bytes")
    args = (_dev(x, torch.float32, "x"), x.numel(), packet_numel, num_workers,
            None if global_exps is None else _dev(global_exps, torch.int8, "global_exps"),
            _dev(payload, torch.int32, "payload"),
            None if exps_out is None else _dev(exps_out, torch.int8, "exps_out"), flags, _stream(stream, x))
    fn = lib().sml_quantize_pack

    def launch():
        s = fn(*args)
        if s != SML_OK:
            raise SwitchMLError("sml_quantize_pack", s)
    return launch


def dequantize(payload, exps, numel: int, packet_numel: int = 256, num_workers: int = 1,
               out=None, flags: int = 0, stream=None):
    torch = _torch()
    if out is None:
        out = torch.empty(numel, dtype=torch.float32, device=payload.device)
    _check("sml_dequantize", lib().sml_dequantize(
        _dev(payload, torch.int32, "payload"), _dev(exps, torch.int8, "exps"), numel, packet_numel,
        num_workers, _dev(out, torch.float32, "out"), flags, _stream(stream, payload)))
    return out


def bswap_i32(x, out=None, stream=None):
    torch = _torch()
    if out is None:
        out = torch.empty_like(x)
    _check("sml_bswap_i32", lib().sml_bswap_i32(_dev(x, torch.int32, "x"), _dev(out, torch.int32, "out"),
                                                x.numel(), _stream(stream, x)))
    return out


def loopback_aggregate(payload, num_workers: int, flags: int = 0, stream=None):
    torch = _torch()
    _check("sml_loopback_aggregate", lib().sml_loopback_aggregate(
        _dev(payload, torch.int32, "payload"), payload.numel(), num_workers, flags, _stream(stream, payload)))
    return payload


def roundtrip_loopback(x, packet_numel: int = 256, num_workers: int = 1, out=None,
                       payload=None, exps_out=None, flags: int = 0, stream=None):
    torch = _torch()
    if out is None:
        out = torch.empty_like(x)
    p = None if payload is None else _dev(payload, torch.int32, "payload")
    e = None if exps_out is None else _dev(exps_out, torch.int8, "exps_out")
    _check("sml_roundtrip_loopback", lib().sml_roundtrip_loopback(
        _dev(x, torch.float32, "x"), _dev(out, torch.float32, "out"), x.numel(), packet_numel,
        num_workers, p, e, flags, _stream(stream, x)))
    return out


class Slice(ctypes.Structure):
    """sml_slice: one job slice of a batched round trip."""
    _fields_ = [("in_", ctypes.c_void_p), ("out", ctypes.c_void_p), ("numel", ctypes.c_uint64)]


MAX_BATCH_SLICES = 64


def roundtrip_loopback_batch(slices, packet_numel: int = 256, num_workers: int = 1, flags: int = 0, stream=None):
    """The fused round trip over several slices in one launch
    (sml_roundtrip_loopback_batch): `slices` is a list of (x, out) fp32
    device (or pinned host) tensors; slice i gets exactly
    roundtrip_loopback(x_i, out=out_i) — its blocks start at its own first
    element."""
    torch = _torch()
    arr = (Slice * max(1, len(slices)))()
    for i, (x, o) in enumerate(slices):
        if x.numel() != o.numel():
            raise ValueError("slice in/out sizes differ")
        arr[i] = Slice(_dev(x, torch.float32, "x").value, _dev(o, torch.float32, "out").value, x.numel())
    st = _stream(stream, slices[0][0]) if slices else None
    _check("sml_roundtrip_loopback_batch", lib().sml_roundtrip_loopback_batch(
        arr, len(slices), packet_numel, num_workers, flags, st))


MAX_SWITCH_WORKERS = 16


def switch_aggregate(payloads, exps=None, numel: int | None = None, packet_numel: int = 256,
                     payload_out=None, exps_out=None, out=None, flags: int = 0, stream=None):
    """K6: the switch's per-slot aggregation over W worker planes, fused with
    the dequantize (p4/processor.p4:48-54 wrapping bit<32> sum,
    p4/exponents.p4:48-54 signed int8 max, then PostprocessSingle with
    scale(W, e_max), ppp.cc:197-251).  `payloads`: W int32 planes of B*P
    words (BE unless FLAG_PAYLOAD_LE); `exps`: W int8 planes of B bytes.
    Writes whichever of payload_out / exps_out / out is given; with none
    given, returns a new fp32 bucket `out` of `numel` elements."""
    torch = _torch()
    W = len(payloads)
    if W == 0 or W > MAX_SWITCH_WORKERS:
        raise ValueError(f"1 <= workers <= {MAX_SWITCH_WORKERS}, got {W}")
    n_words = payloads[0].numel()
    if any(p.numel() != n_words for p in payloads):
        raise ValueError("payload planes differ in size")
    if numel is None:
        numel = n_words
    B = num_blocks(numel, packet_numel)
    if B * packet_numel != n_words:
        raise ValueError(f"payload planes hold {n_words} words, B*P = {B * packet_numel}")
    if exps is not None:
        if len(exps) != W or any(e.numel() != B for e in exps):
            raise ValueError("need one exponent plane of B bytes per payload plane")
    if payload_out is None and exps_out is None and out is None:
        out = torch.empty(numel, dtype=torch.float32, device=payloads[0].device)
    # planes are int32 tensors, or (peer-to-peer switch) mapped peer planes
    # exposing data_ptr()/numel() only
    pp = (ctypes.c_void_p * W)(*[_dev(p, torch.int32, "payloads[w]").value if isinstance(p, torch.Tensor)
                                 else p.data_ptr() for p in payloads])
    ep = None if exps is None else (ctypes.c_void_p * W)(*[_dev(e, torch.int8, "exps[w]").value for e in exps])
    _check("sml_switch_aggregate", lib().sml_switch_aggregate(
        ctypes.cast(pp, ctypes.c_void_p), None if ep is None else ctypes.cast(ep, ctypes.c_void_p), W, numel,
        packet_numel,
        None if payload_out is None else _dev(payload_out, torch.int32, "payload_out"),
        None if exps_out is None else _dev(exps_out, torch.int8, "exps_out"),
        None if out is None else _dev(out, torch.float32, "out"), flags, _stream(stream, payloads[0])))
    return out


def copy_segments(pairs, flags: int = 0, stream=None):
    """sml_copy_segments: every (src, dst) pair of 32-bit tensors (same
    numel; CUDA or pinned host) copied in ONE launch, the tiles dealt
    round-robin over the pairs (the in-node switch's multicast).
    flags = FLAG_PEER_PLANES when sources were written by other GPUs."""
    torch = _torch()
    k = len(pairs)
    if k > MAX_SWITCH_WORKERS:
        raise ValueError(f"at most {MAX_SWITCH_WORKERS} segments")
    srcs = (ctypes.c_void_p * max(1, k))()
    dsts = (ctypes.c_void_p * max(1, k))()
    words = (ctypes.c_uint64 * max(1, k))()
    for i, (s, d) in enumerate(pairs):
        if s.numel() != d.numel() or s.element_size() != 4 or d.element_size() != 4:
            raise ValueError("segments are pairs of equal-size 32-bit tensors")
        srcs[i] = _dev(s, s.dtype, "src").value
        dsts[i] = _dev(d, d.dtype, "dst").value
        words[i] = s.numel()
    _check("sml_copy_segments", lib().sml_copy_segments(
        ctypes.cast(srcs, ctypes.c_void_p), ctypes.cast(dsts, ctypes.c_void_p), ctypes.cast(words, ctypes.c_void_p),
        k, flags, _stream(stream, pairs[0][0] if pairs else None)))


def packet_burst(x, out, packet_numel: int, num_workers: int, batch_num_ltus: int, recv_exps, pkt_ids,
                 entries, extras, flags: int = 0) -> PacketBurst:
    """A PacketBurst over slice `x` (fp32 or int32 CUDA tensor) and output
    `out`; entries / extras are device-addressable addresses (ints)."""
    torch = _torch()
    if len(pkt_ids) > MAX_BURST:
        raise ValueError(f"at most {MAX_BURST} packets per burst")
    b = PacketBurst()
    b.in_ = x.data_ptr()
    b.out = out.data_ptr() if out is not None else None
    b.numel = x.numel()
    b.packet_numel = packet_numel
    b.num_workers = num_workers
    b.data_type = 1 if x.dtype == torch.int32 else 0
    b.batch_num_ltus = batch_num_ltus
    b.recv_exps = recv_exps.data_ptr() if recv_exps is not None else None
    b.count = len(pkt_ids)
    b.flags = flags
    for i, (q, e, x_) in enumerate(zip(pkt_ids, entries, extras)):
        b.pkt_ids[i], b.entries[i], b.extras[i] = q, e, x_
    return b


def preprocess_burst(burst: PacketBurst, stream=None, like=None):
    """sml_preprocess_burst: PreprocessSingle for every packet of the burst."""
    _check("sml_preprocess_burst", lib().sml_preprocess_burst(ctypes.byref(burst), _stream(stream, like)))


def postprocess_burst(burst: PacketBurst, stream=None, like=None):
    """sml_postprocess_burst: PostprocessSingle for every packet of the burst."""
    _check("sml_postprocess_burst", lib().sml_postprocess_burst(ctypes.byref(burst), _stream(stream, like)))


def exchange_burst(burst: PacketBurst, stream=None, like=None):
    """sml_exchange_burst: for every received packet q, PostprocessSingle(q)
    then PreprocessSingle(q + b) into the same buffer (the DPDK receive loop's
    post + ReusePacket) in one launch; FLAG_PROCESS_PACKET applies the dummy
    backend's ProcessPacket (x W) first."""
    _check("sml_exchange_burst", lib().sml_exchange_burst(ctypes.byref(burst), _stream(stream, like)))


BURST_PRE, BURST_POST, BURST_EXCHANGE = 0, 1, 2


class BurstServer:
    """sml_burst_server_*: a persistent workgroup that runs bursts submitted
    through a doorbell in host memory (for packet buffers in pinned host
    memory).  submit() returns with the burst complete; close() stops it."""

    def __init__(self, packet_numel: int, flags: int = 0, idle_ms: int = 100):
        self._h = ctypes.c_void_p()
        _check("sml_burst_server_create", lib().sml_burst_server_create(packet_numel, flags, idle_ms,
                                                                        ctypes.byref(self._h)))

    def submit(self, op: int, burst: PacketBurst):
        _check("sml_burst_server_submit", lib().sml_burst_server_submit(self._h, op, ctypes.byref(burst)))

    def stop(self):
        """Leave the loop now (the next submit restarts it)."""
        _check("sml_burst_server_stop", lib().sml_burst_server_stop(self._h))

    def start(self):
        """Start the loop now instead of on the next submit."""
        _check("sml_burst_server_start", lib().sml_burst_server_start(self._h))

    def inject_unanswered(self, op: int, burst: PacketBurst):
        """Test fault injection: ring the doorbell for `burst` with the server
        stopped (what a failed submit leaves behind)."""
        _check("sml_burst_server_inject_unanswered",
               lib().sml_burst_server_inject_unanswered(self._h, op, ctypes.byref(burst)))

    def close(self):
        if self._h:
            h, self._h = self._h, None
            _check("sml_burst_server_destroy", lib().sml_burst_server_destroy(h))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().sml_burst_server_destroy(self._h)
            self._h = None


def release_to_peers(stream=None, device=None):
    """sml_release_to_peers: system-scope release on every XCD after the work
    on `stream` (the writer's half of a hand-off to other GPUs)."""
    if stream is None:
        stream = _torch().cuda.current_stream(device)
    _check("sml_release_to_peers", lib().sml_release_to_peers(_stream(stream)))


def stream_copy(src, dst, stream=None):
    """Measurement probe: non-temporal tile copy (src/dst same byte size)."""
    nbytes = src.numel() * src.element_size()
    _check("sml_stream_copy", lib().sml_stream_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                                    nbytes, _stream(stream, src)))
    return dst


def frame_bytes(packet_numel: int = 256) -> int:
    return int(lib().sml_frame_bytes(packet_numel))


def quantize_pack_frames(x, params: FrameParams, packet_numel: int = 256, num_workers: int = 1,
                         batch_max: int = 64, global_exps=None, frames=None, stride: int | None = None,
                         stream=None):
    """Fused quantize + pack straight into DPDK frames (B + b frames of
    `stride` bytes, uint8).  `frames` may be a device tensor or pinned host
    memory (the NIC's buffers)."""
    torch = _torch()
    B = num_blocks(x.numel(), packet_numel)
    b = min(B, batch_max)
    stride = stride or frame_bytes(packet_numel)
    if frames is None:
        frames = torch.empty((B + b) * stride, dtype=torch.uint8, device=x.device)
    g = None if global_exps is None else _dev(global_exps, torch.int8, "global_exps")
    _check("sml_quantize_pack_frames", lib().sml_quantize_pack_frames(
        _dev(x, torch.float32, "x"), x.numel(), packet_numel, num_workers, g, batch_max,
        ctypes.byref(params), _dev(frames, torch.uint8, "frames"), stride, _stream(stream, x)))
    return frames


class RxSlice:
    """Receive-side state of one job slice for dequantize_frames: the
    received exponents, the rx bitmap (DpdkWorkerThread's rte_bitmap,
    dpdk_worker_thread.cc:316-342) and {accepted, discarded} counters."""

    def __init__(self, numel: int, packet_numel: int = 256, batch_max: int = 64, device="cuda",
                 out=None):
        torch = _torch()
        self.numel, self.packet_numel, self.batch_max = numel, packet_numel, batch_max
        B = num_blocks(numel, packet_numel)
        self.exps = torch.zeros(B, dtype=torch.int8, device=device)
        self.state = torch.zeros(int(lib().sml_rx_state_words(numel, packet_numel, batch_max, 0)),
                                 dtype=torch.int64, device=device)
        self.counts = torch.zeros(2, dtype=torch.int64, device=device)
        self.out = out if out is not None else torch.zeros(numel, dtype=torch.float32, device=device)

    def reset(self, stream=None):
        """rte_bitmap_reset for a new job slice: zero the rx state (one async
        memset, sml_rx_reset)."""
        torch = _torch()
        _check("sml_rx_reset", lib().sml_rx_reset(_dev(self.state, torch.int64, "state"), self.state.numel(),
                                                  _stream(stream, self.state)))


def dequantize_frames(frames, num_frames: int, rx: RxSlice, num_workers: int = 1, job_id: int = 0,
                      stride: int | None = None, stream=None):
    """PostprocessSingle over received DPDK frames (any order; duplicates and
    other jobs' frames discarded), writing rx.out / rx.exps / rx.counts."""
    torch = _torch()
    stride = stride or frame_bytes(rx.packet_numel)
    _check("sml_dequantize_frames", lib().sml_dequantize_frames(
        _dev(frames, torch.uint8, "frames"), num_frames, stride, rx.numel, rx.packet_numel, num_workers,
        rx.batch_max, job_id, _dev(rx.exps, torch.int8, "exps"), _dev(rx.state, torch.int64, "state"),
        _dev(rx.out, torch.float32, "out"), _dev(rx.counts, torch.int64, "counts"), _stream(stream, rx.out)))
    return rx.out


def pack_frames_int32(x, params: FrameParams, packet_numel: int = 256, frames=None, stride: int | None = None,
                      stream=None):
    """An INT32 job slice straight into DPDK frames: B frames (no extra
    batch), frame p = BuildPacket's headers + htonl of block p's words."""
    torch = _torch()
    B = num_blocks(x.numel(), packet_numel)
    stride = stride or frame_bytes(packet_numel)
    if frames is None:
        frames = torch.empty(B * stride, dtype=torch.uint8, device=x.device)
    _check("sml_pack_frames_int32", lib().sml_pack_frames_int32(
        _dev(x, torch.int32, "x"), x.numel(), packet_numel, ctypes.byref(params),
        _dev(frames, torch.uint8, "frames"), stride, _stream(stream, x)))
    return frames


class RxSliceInt32:
    """Receive-side state of one INT32 job slice for unpack_frames_int32: the
    rx bitmap over its B pkt_ids plus the slice's call sequence, the running
    call's conflict count, the slice's conflict total and the fix-up's dirty
    list (uint64[2B + 6], sml_rx_state_words), {accepted, discarded}
    counters, the output."""

    def __init__(self, numel: int, packet_numel: int = 256, device="cuda", out=None):
        torch = _torch()
        self.numel, self.packet_numel = numel, packet_numel
        self.nblocks = num_blocks(numel, packet_numel)
        self.state = torch.zeros(int(lib().sml_rx_state_words(numel, packet_numel, 1, 1)), dtype=torch.int64,
                                 device=device)
        self.counts = torch.zeros(2, dtype=torch.int64, device=device)
        self.out = out if out is not None else torch.zeros(numel, dtype=torch.int32, device=device)

    @property
    def conflicts(self) -> int:
        """Copies of a pkt_id that claimed it ahead of an earlier copy and were
        resolved by the fix-up, over the slice so far (reads the device)."""
        return int(self.state[self.nblocks + 1].item())

    def reset(self, stream=None):
        """rte_bitmap_reset for a new job slice (sml_rx_reset)."""
        torch = _torch()
        _check("sml_rx_reset", lib().sml_rx_reset(_dev(self.state, torch.int64, "state"), self.state.numel(),
                                                  _stream(stream, self.state)))


def unpack_frames_int32(frames, num_frames: int, rx: RxSliceInt32, job_id: int = 0, stride: int | None = None,
                        stream=None):
    """PostprocessSingle's INT32 branch over received DPDK frames (any order;
    duplicates, other jobs' frames and pkt_id >= B discarded): ntohl into rx.out."""
    torch = _torch()
    stride = stride or frame_bytes(rx.packet_numel)
    _check("sml_unpack_frames_int32", lib().sml_unpack_frames_int32(
        _dev(frames, torch.uint8, "frames"), num_frames, stride, rx.numel, rx.packet_numel, job_id,
        _dev(rx.state, torch.int64, "state"), _dev(rx.out, torch.int32, "out"),
        _dev(rx.counts, torch.int64, "counts"), _stream(stream, rx.out)))
    return rx.out


def debug_stall(microseconds: int, stream=None):
    """Fault injection for tests: keep `stream` busy for `microseconds` of
    device wall-clock time (<= 60 s), then end (sml_debug_stall)."""
    _check("sml_debug_stall", lib().sml_debug_stall(int(microseconds), _stream(stream)))


def rdma_imm(exps, batch_max: int = 64, stream=None, num_blocks_int32: int | None = None, device=None):
    """RDMA immediates of one slice's B + b messages (uint32 in host order, as
    int32 tensor): (msg_id & 0xFFFF) | exponent << 16.  exps=None with
    num_blocks_int32=B: an INT32 slice's B messages, msg_id & 0xFFFF."""
    torch = _torch()
    if exps is None:
        B = int(num_blocks_int32)
        out = torch.empty(B, dtype=torch.int32, device=device or "cuda")
        _check("sml_rdma_imm_int32", lib().sml_rdma_imm_int32(B, _dev(out, torch.int32, "imm"),
                                                             _stream(stream, out)))
        return out
    B = exps.numel()
    out = torch.empty(B + min(B, batch_max), dtype=torch.int32, device=exps.device)
    _check("sml_rdma_imm", lib().sml_rdma_imm(_dev(exps, torch.int8, "exps"), B, batch_max,
                                             _dev(out, torch.int32, "imm"), _stream(stream, exps)))
    return out
