"""ctypes + numpy front end of the CPU restatement in sml_oracle.c.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / reported CPU baseline.  The
product path (p4app-switchml_amd/) never imports this module.

Parity status: "parity unpinned" at the bit level — the reference client_lib
is not buildable here (client_lib/src/common.h:31 needs glog, absent from the
image).  Pinned by the reference's own 1 % known-answer checks
(examples/hello_world/main.cc:58-74, benchmarks/allreduce_benchmark/main.cc:331-399)
and by hand-derived vectors (tests/golden/).

Besides the C library this module holds a second, independent numpy
restatement (``np_*``) so the C code is cross-checked by a different
implementation of the same reading of ppp.cc.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsml_oracle.so")
_lib = None

HALF_AWAY = 0
RNE_VCL = 1
MODE_ROUNDTRIP = 0
MODE_PREPROCESS = 1


def build() -> str:
    """Compile libsml_oracle.so with the committed Makefile."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, u32, u16, i32, vp = (ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16,
                                  ctypes.c_int, ctypes.c_void_p)
        L.orc_num_blocks.restype = u64
        L.orc_num_blocks.argtypes = [u64, u64]
        L.orc_scale.restype = ctypes.c_float
        L.orc_scale.argtypes = [u16, ctypes.c_int8]
        L.orc_scale_lut.argtypes = [u16, vp]
        L.orc_exponents.argtypes = [vp, u64, u64, vp]
        L.orc_quantize.argtypes = [vp, u64, u64, u16, vp, i32, vp]
        L.orc_dequantize.argtypes = [vp, vp, u64, u64, u16, vp]
        L.orc_bswap32.argtypes = [vp, vp, u64]
        L.orc_loopback_aggregate.argtypes = [vp, u64, u16]
        L.orc_switch_exps.argtypes = [vp, i32, u64, vp]
        L.orc_switch_payload.argtypes = [vp, i32, u64, vp]
        L.orc_slice.argtypes = [u64, i32, i32, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.orc_dummy_allreduce.restype = i32
        L.orc_dummy_allreduce.argtypes = [vp, vp, u64, u64, u32, i32, u16, i32, i32]
        L.orc_dummy_allreduce_ex.restype = i32
        L.orc_dummy_allreduce_ex.argtypes = [vp, vp, u64, u64, u32, i32, u16, i32, i32, i32]
        L.orc_quantize_vcl.argtypes = [vp, u64, u64, u16, vp, vp]
        L.orc_dummy_packet_stream.restype = i32
        L.orc_dummy_packet_stream.argtypes = [vp, u64, u64, u32, u16, vp, vp, vp]
        L.orc_build_frames.restype = i32
        L.orc_build_frames.argtypes = [vp, u64, u64, u16, vp, u32, vp, vp, u64]
        L.orc_dequantize_frames.argtypes = [vp, u64, u64, u64, u64, u16, u32, u64, vp, vp, vp, vp]
        L.orc_build_frames_i32.restype = i32
        L.orc_build_frames_i32.argtypes = [vp, u64, u64, vp, vp, u64]
        L.orc_unpack_frames_i32.argtypes = [vp, u64, u64, u64, u64, u64, vp, vp, vp]
        L.orc_pkt_id_to_pool_index.restype = ctypes.c_uint16
        L.orc_pkt_id_to_pool_index.argtypes = [u64, u32, u32, u32]
        L.orc_glibc_rand.argtypes = [u32, u64, vp]
        L.orc_ref_random_floats.argtypes = [u32, u64, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


# ---------------------------------------------------------------- C oracle --

def num_blocks(numel: int, P: int) -> int:
    return int(lib().orc_num_blocks(numel, P))


def scale_lut(num_workers: int) -> np.ndarray:
    out = np.empty(256, dtype=np.float32)
    lib().orc_scale_lut(num_workers, _p(out))
    return out


def exponents(x: np.ndarray, P: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(num_blocks(x.size, P), dtype=np.int8)
    lib().orc_exponents(_p(x), x.size, P, _p(out))
    return out


def quantize(x: np.ndarray, P: int, num_workers: int = 1, global_exps: np.ndarray | None = None,
             rounding: int = HALF_AWAY) -> np.ndarray:
    """Payload plane [B*P] of big-endian int32 words, returned as uint32 (raw bytes)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    B = num_blocks(x.size, P)
    out = np.empty(B * P, dtype=np.uint32)
    ge = None if global_exps is None else np.ascontiguousarray(global_exps, dtype=np.int8)
    lib().orc_quantize(_p(x), x.size, P, num_workers, None if ge is None else _p(ge), rounding, _p(out))
    return out


def quantize_vcl(x: np.ndarray, P: int, num_workers: int = 1):
    """(payload_be uint32[B*P], exps int8[B]) of the VCL=1 build's vector loops (SSE2)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    B = num_blocks(x.size, P)
    out = np.empty(B * P, dtype=np.uint32)
    exps = np.empty(B, dtype=np.int8)
    lib().orc_quantize_vcl(_p(x), x.size, P, num_workers, _p(out), _p(exps))
    return out, exps


def dequantize(payload_be: np.ndarray, exps: np.ndarray, numel: int, P: int, num_workers: int = 1) -> np.ndarray:
    payload_be = np.ascontiguousarray(payload_be, dtype=np.uint32)
    exps = np.ascontiguousarray(exps, dtype=np.int8)
    out = np.empty(numel, dtype=np.float32)
    lib().orc_dequantize(_p(payload_be), _p(exps), numel, P, num_workers, _p(out))
    return out


def bswap32(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a).view(np.uint32)
    out = np.empty_like(a)
    lib().orc_bswap32(_p(a), _p(out), a.size)
    return out


def loopback_aggregate(payload_be: np.ndarray, num_workers: int) -> np.ndarray:
    out = np.array(payload_be, dtype=np.uint32, copy=True)
    lib().orc_loopback_aggregate(_p(out), out.size, num_workers)
    return out


def switch_exps(exps_per_worker) -> np.ndarray:
    arrs = [np.ascontiguousarray(e, dtype=np.int8) for e in exps_per_worker]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    out = np.empty(arrs[0].size, dtype=np.int8)
    lib().orc_switch_exps(ctypes.cast(ptrs, ctypes.c_void_p), len(arrs), out.size, _p(out))
    return out


def switch_payload(payload_per_worker) -> np.ndarray:
    arrs = [np.ascontiguousarray(e, dtype=np.uint32) for e in payload_per_worker]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    out = np.empty(arrs[0].size, dtype=np.uint32)
    lib().orc_switch_payload(ctypes.cast(ptrs, ctypes.c_void_p), len(arrs), out.size, _p(out))
    return out


def slice_geometry(numel: int, num_slices: int, t: int):
    off, n = ctypes.c_uint64(), ctypes.c_uint64()
    lib().orc_slice(numel, num_slices, t, ctypes.byref(off), ctypes.byref(n))
    return int(off.value), int(n.value)


def dummy_allreduce(x: np.ndarray, P: int = 256, max_outstanding_packets: int = 256,
                    num_worker_threads: int = 4, num_workers: int = 1, threaded: bool = False,
                    mode: int = MODE_ROUNDTRIP, out: np.ndarray | None = None, vcl: bool = False) -> np.ndarray:
    """The dummy-backend packet loop; vcl=True runs the VCL=1 build's vector
    loops (SSE2 restatement, RNE body) instead of the scalar VCL=0 path."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    if out is None:
        out = np.empty_like(x)
    rc = lib().orc_dummy_allreduce_ex(_p(x), _p(out), x.size, P, max_outstanding_packets,
                                      num_worker_threads, num_workers, int(threaded), mode, int(vcl))
    if rc != 0:
        raise RuntimeError(f"orc_dummy_allreduce failed rc={rc}")
    return out


def dummy_packet_stream(x: np.ndarray, P: int = 256, batch_max: int = 64, num_workers: int = 1):
    x = np.ascontiguousarray(x, dtype=np.float32)
    B = num_blocks(x.size, P)
    b = min(B, batch_max)
    pe = np.empty(B + b, dtype=np.int8)
    pp = np.empty((B + b) * P, dtype=np.uint32)
    out = np.empty_like(x)
    rc = lib().orc_dummy_packet_stream(_p(x), x.size, P, batch_max, num_workers, _p(pe), _p(pp), _p(out))
    if rc != 0:
        raise RuntimeError("orc_dummy_packet_stream failed")
    return pe, pp.reshape(B + b, P), out, b


def build_frames(x: np.ndarray, params, P: int = 256, num_workers: int = 1, batch_max: int = 64,
                 global_exps=None, stride: int | None = None) -> np.ndarray:
    """DPDK frames of one slice (BuildPacket + PreprocessSingle per packet).
    `params` is a ctypes structure with sml_frame_params' layout."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    B = num_blocks(x.size, P)
    b = min(B, batch_max)
    stride = stride or 52 + 4 * P
    out = np.zeros((B + b) * stride, dtype=np.uint8)
    ge = None if global_exps is None else np.ascontiguousarray(global_exps, dtype=np.int8)
    rc = lib().orc_build_frames(_p(x), x.size, P, num_workers, None if ge is None else _p(ge), batch_max,
                                ctypes.cast(ctypes.byref(params), ctypes.c_void_p), _p(out), stride)
    if rc != 0:
        raise RuntimeError("orc_build_frames failed")
    return out


class RxState:
    """Receive-side state of one slice for dequantize_frames (the PPP's
    scaling factors as exponents, the worker's rx bitmap, the output)."""

    def __init__(self, numel: int, P: int = 256, batch_max: int = 64):
        B = num_blocks(numel, P)
        self.numel, self.P, self.batch_max = numel, P, batch_max
        self.exps = np.zeros(B, dtype=np.int8)
        self.seen = np.zeros(max(1, B + min(B, batch_max)), dtype=np.uint8)
        self.out = np.zeros(numel, dtype=np.float32)
        self.counts = [0, 0]


def dequantize_frames(frames: np.ndarray, num_frames: int, stride: int, rx: RxState,
                      num_workers: int = 1, job_id: int = 0) -> RxState:
    """DpdkWorkerThread's receive loop over `num_frames` received frames in
    order; accumulates into `rx` (call repeatedly for successive rx bursts)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    assert frames.size >= num_frames * stride
    counts = np.zeros(2, dtype=np.uint64)
    lib().orc_dequantize_frames(_p(frames), num_frames, stride, rx.numel, rx.P, num_workers, rx.batch_max,
                                job_id, _p(rx.exps), _p(rx.seen), _p(rx.out), _p(counts))
    rx.counts = [rx.counts[0] + int(counts[0]), rx.counts[1] + int(counts[1])]
    return rx


def build_frames_i32(x: np.ndarray, params, P: int = 256, stride: int | None = None) -> np.ndarray:
    """DPDK frames of one INT32 slice: B frames (no extra batch), payload =
    htonl of each block's words (ppp.cc:158-190)."""
    x = np.ascontiguousarray(x, dtype=np.int32)
    B = num_blocks(x.size, P)
    stride = stride or 52 + 4 * P
    out = np.zeros(B * stride, dtype=np.uint8)
    rc = lib().orc_build_frames_i32(_p(x), x.size, P, ctypes.cast(ctypes.byref(params), ctypes.c_void_p),
                                    _p(out), stride)
    if rc != 0:
        raise RuntimeError("orc_build_frames_i32 failed")
    return out


class RxStateI32:
    """Receive-side state of one INT32 slice (rx bitmap over B pkt_ids, output)."""

    def __init__(self, numel: int, P: int = 256):
        self.numel, self.P = numel, P
        self.seen = np.zeros(max(1, num_blocks(numel, P)), dtype=np.uint8)
        self.out = np.zeros(numel, dtype=np.int32)
        self.counts = [0, 0]


def unpack_frames_i32(frames: np.ndarray, num_frames: int, stride: int, rx: RxStateI32, job_id: int = 0):
    """The receive loop over INT32 frames in order (ntohl into rx.out)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    assert frames.size >= num_frames * stride
    counts = np.zeros(2, dtype=np.uint64)
    lib().orc_unpack_frames_i32(_p(frames), num_frames, stride, rx.numel, rx.P, job_id, _p(rx.seen),
                                _p(rx.out), _p(counts))
    rx.counts = [rx.counts[0] + int(counts[0]), rx.counts[1] + int(counts[1])]
    return rx


def pool_index(pkt_id, start, shift, mop) -> int:
    return int(lib().orc_pkt_id_to_pool_index(pkt_id, start, shift, mop))


# ------------------------------------------- independent numpy restatement --

def _bswap(u: np.ndarray) -> np.ndarray:
    return u.astype(np.uint32).byteswap()


def np_scale_lut(num_workers: int) -> np.ndarray:
    e = np.arange(256, dtype=np.uint8).view(np.int8).astype(np.int32)
    with np.errstate(divide="ignore", over="ignore"):
        denom = np.float32(num_workers) * np.ldexp(np.float32(1.0), e).astype(np.float32)
        return (np.float64(2147483647) / denom.astype(np.float64)).astype(np.float32)


def np_exponents(x: np.ndarray, P: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    B = -(-x.size // P)
    pad = np.zeros(B * P, dtype=np.uint32)
    u = x.view(np.uint32) & np.uint32(0x7FFFFFFF)
    u = np.where(u > np.uint32(0x7F800000), np.uint32(0), u)  # NaN never selected
    pad[: x.size] = u
    m = pad.reshape(B, P).max(axis=1)
    e = ((m & np.uint32(0x7F800000)) >> np.uint32(23)).astype(np.int32) - 126
    return (e & 0xFF).astype(np.uint8).view(np.int8)


def _x86_f2u32(r: np.ndarray) -> np.ndarray:
    r64 = r.astype(np.float64)
    ok = np.abs(r64) < 2.0 ** 63
    v = np.where(ok, r64, 0.0).astype(np.int64)
    return (v & 0xFFFFFFFF).astype(np.uint32)


def _roundf_half_away(v: np.ndarray) -> np.ndarray:
    v64 = v.astype(np.float64)
    t = np.trunc(v64)
    with np.errstate(invalid="ignore"):
        frac = np.abs(v64 - t)
        r = t + np.where(frac >= 0.5, np.sign(v64), 0.0)
    return r  # exact in float64; integral values of float32 magnitude


def np_quantize(x: np.ndarray, P: int, num_workers: int = 1, global_exps=None) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    B = -(-x.size // P)
    e = np_exponents(x, P) if global_exps is None else np.asarray(global_exps, dtype=np.int8)
    lut = np_scale_lut(num_workers)
    s = np.repeat(lut[e.view(np.uint8)], P)[: x.size]
    with np.errstate(over="ignore", invalid="ignore"):
        prod = (x * s).astype(np.float32)
        r = _roundf_half_away(prod)
    q = _x86_f2u32(r)
    out = np.zeros(B * P, dtype=np.uint32)
    out[: x.size] = _bswap(q)
    return out


def np_dequantize(payload_be: np.ndarray, exps: np.ndarray, numel: int, P: int, num_workers: int = 1) -> np.ndarray:
    lut = np_scale_lut(num_workers)
    s = np.repeat(lut[np.asarray(exps, dtype=np.int8).view(np.uint8)], P)[:numel]
    q = _bswap(np.asarray(payload_be, dtype=np.uint32)[:numel]).view(np.int32)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (q.astype(np.float32) / s).astype(np.float32)


def np_switch(exps_per_worker, payload_per_worker):
    e = np.max(np.stack([np.asarray(a, dtype=np.int8) for a in exps_per_worker]), axis=0)
    acc = np.zeros_like(np.asarray(payload_per_worker[0], dtype=np.uint32))
    for p in payload_per_worker:
        acc = acc + _bswap(np.asarray(p, dtype=np.uint32))  # uint32 wraps
    return e, _bswap(acc)


# ------------------------------------------------------ data generators --

def c_glibc_rand(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    lib().orc_glibc_rand(seed, n, _p(out))
    return out


def c_ref_random_floats(seed: int, n: int) -> np.ndarray:
    """C version of ref_random_floats (fast for the 16M-element configs)."""
    out = np.empty(n, dtype=np.float32)
    lib().orc_ref_random_floats(seed, n, _p(out))
    return out


def glibc_rand_stream(seed: int, n: int) -> np.ndarray:
    """glibc random() TYPE_3 additive generator (what rand() returns after
    srand(seed)), restated so the reference's own data generators
    (benchmarks/allreduce_benchmark/main.cc:186-205) can be reproduced."""
    r = [0] * (34 + 310 + n)
    if seed == 0:
        seed = 1
    r[0] = seed
    for i in range(1, 31):
        hi, lo = divmod(r[i - 1], 127773)
        word = 16807 * lo - 2836 * hi
        if word < 0:
            word += 2147483647
        r[i] = word
    for i in range(31, 34):
        r[i] = r[i - 31]
    for i in range(34, 344 + n):
        r[i] = (r[i - 31] + r[i - 3]) & 0xFFFFFFFF
    return np.array([(v >> 1) for v in r[344:344 + n]], dtype=np.int64)


def ref_random_floats(seed: int, n: int) -> np.ndarray:
    """allreduce_benchmark/main.cc:197-205: r = rand(); bits = (r%2)<<31 | (r%254)<<23 | r%(1<<23)."""
    r = glibc_rand_stream(seed, n)
    bits = ((r % 2) << 31) | ((r % 254) << 23) | (r % (1 << 23))
    return (bits & 0xFFFFFFFF).astype(np.uint32).view(np.float32)


def ref_pattern_floats(n: int) -> np.ndarray:
    """allreduce_benchmark/main.cc:207-212: float(i) * sign, sign alternating +1/-1."""
    i = np.arange(n, dtype=np.int64)
    f = i.astype(np.float32)
    return np.where(i % 2 == 0, f, -f).astype(np.float32)


def splitmix_normal(seed: int, n: int, sigma: float = 1.0) -> np.ndarray:
    """Portable seeded N(0, sigma^2) fp32 (splitmix64 + Box-Muller); the same
    bytes on every host, so GPU-box and container runs see identical inputs."""
    idx = np.arange((n + 1) // 2, dtype=np.uint64)
    with np.errstate(over="ignore"):
        def mix(z):
            z = (z + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(0xFFFFFFFFFFFFFFFF)
            return z ^ (z >> np.uint64(31))
        base = np.uint64(seed) * np.uint64(0x2545F4914F6CDD1D)
        a = mix(base + idx * np.uint64(2))
        b = mix(base + idx * np.uint64(2) + np.uint64(1))
    u1 = ((a >> np.uint64(11)).astype(np.float64) + 1.0) / 9007199254740993.0
    u2 = (b >> np.uint64(11)).astype(np.float64) / 9007199254740992.0
    rad = np.sqrt(-2.0 * np.log(u1))
    z = np.empty(idx.size * 2, dtype=np.float64)
    z[0::2] = rad * np.cos(2 * np.pi * u2)
    z[1::2] = rad * np.sin(2 * np.pi * u2)
    return (z[:n] * sigma).astype(np.float32)


def splitmix_grad(seed: int, n: int) -> np.ndarray:
    """Gradient-like fp32 from integer arithmetic only (exact on every host,
    unlike a libm-based Box-Muller): a signed 24-bit mantissa from splitmix64
    scaled by 2^-(24 + k), k in 0..15, so magnitudes span ~2^-40..2^-1 and
    blocks get different exponents.  Used for the full-size golden digests."""
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + i * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
        z = ((z ^ (z >> np.uint64(31))) * np.uint64(0x94D049BB133111EB)) & np.uint64(0xFFFFFFFFFFFFFFFF)
        z = z ^ (z >> np.uint64(29))
    mant = (z >> np.uint64(40)).astype(np.int64) - (1 << 23)            # [-2^23, 2^23)
    k = ((i >> np.uint64(8)) * np.uint64(7) + (z & np.uint64(1))) % np.uint64(16)   # varies per 256-block
    return np.ldexp(mant.astype(np.float32), -(24 + k.astype(np.int32))).astype(np.float32)

