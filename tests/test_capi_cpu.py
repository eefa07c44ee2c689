"""CPU tests of the C-ABI boundary (no GPU needed): the HIP library loads,
exports every entry point include/switchml_hip.h declares, and its host-only
entry points (geometry, scale LUT, argument validation) behave — validation
returns before any HIP call, so these run without a device."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def sw():
    import switchml_amd
    switchml_amd.lib()
    return switchml_amd


def test_exports_every_header_symbol(sw):
    syms = sw.header_symbols()
    assert len(syms) >= 12
    L = sw.lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version_and_status_strings(sw):
    L = sw.lib()
    assert L.sml_abi_version() == 2
    for code, name in [(0, b"SML_OK"), (1, b"SML_ERR_INVALID_ARG"), (2, b"SML_ERR_UNSUPPORTED"),
                       (3, b"SML_ERR_ALIGNMENT"), (4, b"SML_ERR_HIP")]:
        assert L.sml_status_string(code) == name


@pytest.mark.parametrize("numel,P", [(0, 256), (1, 64), (255, 256), (256, 256), (257, 256),
                                     (16 * 2 ** 20, 256), (67_108_864, 1024), (10 ** 12 + 3, 64)])
def test_num_blocks_matches_oracle(sw, numel, P):
    assert sw.num_blocks(numel, P) == O.num_blocks(numel, P)


def test_num_blocks_no_byte_count_overflow(sw):
    # numel * 4 would wrap 64 bits; the block count must not
    for numel, P in [(2 ** 62 + 1, 256), (2 ** 64 - 1, 64), (2 ** 64 - 1, 1024)]:
        assert sw.num_blocks(numel, P) == -(-numel // P)


@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 7, 8, 16, 255, 256, 1000, 4096, 65535])
def test_host_scale_lut_matches_oracle(sw, W):
    assert np.array_equal(sw.scale_lut(W).view(np.uint32), O.scale_lut(W).view(np.uint32))


def test_argument_validation_without_gpu(sw):
    L = sw.lib()
    buf = (ctypes.c_float * 16)()
    pay = (ctypes.c_int32 * 1024)()
    # unsupported packet size
    assert L.sml_quantize_pack(buf, 16, 100, 1, None, pay, None, 0, None) == sw.SML_ERR_UNSUPPORTED
    assert L.sml_dequantize(pay, None, 16, 96, 1, buf, 0, None) == sw.SML_ERR_UNSUPPORTED
    # num_workers == 0
    assert L.sml_quantize_pack(buf, 16, 256, 0, None, pay, None, 0, None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_scale_lut(0, buf) == sw.SML_ERR_INVALID_ARG
    # empty job slices are a no-op (dummy_worker_thread.cc:87 skips numel <= 0)
    assert L.sml_quantize_pack(None, 0, 256, 1, None, None, None, 0, None) == sw.SML_OK
    assert L.sml_dequantize(None, None, 0, 256, 1, None, 0, None) == sw.SML_OK
    assert L.sml_bswap_i32(None, None, 0, None) == sw.SML_OK
    # null payload with work to do
    assert L.sml_quantize_pack(buf, 16, 256, 1, None, None, None, 0, None) == sw.SML_ERR_INVALID_ARG
    # misaligned payload plane
    addr = ctypes.addressof(pay) + 4
    assert L.sml_quantize_pack(buf, 16, 256, 1, None, ctypes.c_void_p(addr), None, 0, None) == sw.SML_ERR_ALIGNMENT
    # loopback count must cover whole 16-byte vectors
    assert L.sml_loopback_aggregate(pay, 6, 2, 0, None) == sw.SML_ERR_ALIGNMENT


def test_burst_validation_without_gpu(sw):
    """sml_{pre,post}process_burst / sml_exchange_burst refuse a malformed
    burst before any HIP call: too many packets, an id past B (+ b), a
    duplicate id, q and q + b together, a zero window for the exchange, a
    missing extra slot for a FLOAT32 packet that carries an exponent."""
    L = sw.lib()
    x = (ctypes.c_float * 4096)()
    o = (ctypes.c_float * 4096)()
    recv = (ctypes.c_int8 * 16)()
    ring = (ctypes.c_int32 * 256)()
    extra = (ctypes.c_uint8 * 2)()

    def burst(ids, b=4, with_extra=True, count=None):
        bt = sw.PacketBurst()
        bt.in_ = ctypes.addressof(x)
        bt.out = ctypes.addressof(o)
        bt.numel = 4096
        bt.packet_numel = 256                  # B = 16
        bt.num_workers = 1
        bt.data_type = 0
        bt.batch_num_ltus = b
        bt.recv_exps = ctypes.addressof(recv)
        bt.count = len(ids) if count is None else count
        for i, q in enumerate(ids):
            bt.pkt_ids[i] = q
            bt.entries[i] = ctypes.addressof(ring)
            bt.extras[i] = ctypes.addressof(extra) if with_extra else None
        return ctypes.byref(bt)

    bad = sw.SML_ERR_INVALID_ARG
    for fn in (L.sml_preprocess_burst, L.sml_postprocess_burst, L.sml_exchange_burst):
        assert fn(burst([0], count=65), None) == bad           # > SML_MAX_BURST
        assert fn(burst([20]), None) == bad                    # q >= B + b
        assert fn(burst([3, 3]), None) == bad                  # duplicate
        assert fn(burst([5, 1]), None) == bad                  # q and q + b (any order)
        assert fn(burst([2], with_extra=False), None) == bad   # q < B needs its extra slot
        assert fn(burst([]), None) == sw.SML_OK                # nothing to do
    assert L.sml_exchange_burst(burst([1], b=0), None) == bad  # the exchange needs its window
    assert L.sml_exchange_burst(burst([1], b=17), None) == bad  # b > B


def test_burst_server_validation_without_gpu(sw):
    """The burst server's entry points refuse bad arguments before any HIP
    call: no server, an unsupported packet size, unknown flags."""
    L = sw.lib()
    h = ctypes.c_void_p()
    assert L.sml_burst_server_create(100, 0, 0, ctypes.byref(h)) == sw.SML_ERR_UNSUPPORTED
    assert L.sml_burst_server_create(256, 0x8, 0, ctypes.byref(h)) == sw.SML_ERR_INVALID_ARG
    assert L.sml_burst_server_submit(None, 0, None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_burst_server_stop(None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_burst_server_destroy(None) == sw.SML_OK


def test_grid_limit_knob(sw):
    prev = sw.set_grid_limit(1024)
    assert sw.set_grid_limit(prev) == 1024


def test_xcd_chunk_knob_default_and_roundtrip(sw):
    """Workgroup order knob: default 64, returns the previous value."""
    prev = sw.set_xcd_chunk(7)
    assert prev == 64
    assert sw.set_xcd_chunk(prev) == 7


def test_python_wrapper_rejects_cpu_tensors(sw):
    torch = pytest.importorskip("torch")
    with pytest.raises(TypeError, match="no CPU fallback"):
        sw.quantize_pack(torch.zeros(16))


def test_frames_and_rdma_validation_without_gpu(sw):
    L = sw.lib()
    fp = sw.frame_params()
    buf = (ctypes.c_float * 16)()
    frames = (ctypes.c_uint8 * 8192)()
    assert sw.frame_bytes(256) == 52 + 1024 and sw.frame_bytes(64) == 52 + 256
    # unsupported packet size / stride too small / stride not a multiple of 4
    assert L.sml_quantize_pack_frames(buf, 16, 100, 1, None, 64, ctypes.byref(fp), frames, 4096, None) == sw.SML_ERR_UNSUPPORTED
    assert L.sml_quantize_pack_frames(buf, 16, 256, 1, None, 64, ctypes.byref(fp), frames, 1000, None) == sw.SML_ERR_ALIGNMENT
    assert L.sml_quantize_pack_frames(buf, 16, 256, 1, None, 64, ctypes.byref(fp), frames, 1078, None) == sw.SML_ERR_ALIGNMENT
    # no params / batch 0 / W 0
    assert L.sml_quantize_pack_frames(buf, 16, 256, 1, None, 64, None, frames, 1076, None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_quantize_pack_frames(buf, 16, 256, 1, None, 0, ctypes.byref(fp), frames, 1076, None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_quantize_pack_frames(buf, 16, 256, 0, None, 64, ctypes.byref(fp), frames, 1076, None) == sw.SML_ERR_INVALID_ARG
    # empty slice: nothing to do
    assert L.sml_quantize_pack_frames(None, 0, 256, 1, None, 64, ctypes.byref(fp), None, 1076, None) == sw.SML_OK
    assert L.sml_rdma_imm(None, 0, 64, None, None) == sw.SML_OK
    assert L.sml_rdma_imm(None, 10, 64, None, None) == sw.SML_ERR_INVALID_ARG
    # a null exponent plane is an error for FLOAT32 even with d_imm given
    # (the INT32 immediates have their own entry point)
    assert L.sml_rdma_imm(None, 10, 64, ctypes.c_void_p(16), None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_rdma_imm_int32(0, None, None) == sw.SML_OK
    assert L.sml_rdma_imm_int32(10, None, None) == sw.SML_ERR_INVALID_ARG
    assert L.sml_debug_stall(0, None) == sw.SML_OK
    assert L.sml_debug_stall(60_000_001, None) == sw.SML_ERR_INVALID_ARG


def test_frame_params_layout_matches_header(sw):
    """The ctypes mirror of sml_frame_params has the C layout (offsets per the
    natural alignment of include/switchml_hip.h's struct)."""
    F = sw.FrameParams
    assert F.dst_mac.offset == 0 and F.src_mac.offset == 6
    assert F.src_ip_be.offset == 12 and F.dst_ip_be.offset == 16
    assert F.src_port_be.offset == 20 and F.dst_port_be.offset == 22
    assert F.job_id.offset == 24 and F.pool_index_start.offset == 32
    assert ctypes.sizeof(F) == 48


def test_rx_frames_validation_without_gpu(sw):
    L = sw.lib()
    frames = (ctypes.c_uint8 * 4096)()
    st = (ctypes.c_uint64 * 16)()
    ex = (ctypes.c_int8 * 16)()
    out = (ctypes.c_float * 16)()
    f = L.sml_dequantize_frames
    assert f(frames, 1, 1076, 16, 100, 1, 64, 0, ex, st, out, None, None) == sw.SML_ERR_UNSUPPORTED
    assert f(frames, 1, 1076, 16, 256, 0, 64, 0, ex, st, out, None, None) == sw.SML_ERR_INVALID_ARG
    assert f(frames, 1, 1076, 16, 256, 1, 0, 0, ex, st, out, None, None) == sw.SML_ERR_INVALID_ARG
    assert f(frames, 0, 1076, 16, 256, 1, 64, 0, None, None, None, None, None) == sw.SML_OK
    assert f(frames, 1, 1076, 16, 256, 1, 64, 0, ex, None, out, None, None) == sw.SML_ERR_INVALID_ARG
    assert f(frames, 1, 1000, 16, 256, 1, 64, 0, ex, st, out, None, None) == sw.SML_ERR_ALIGNMENT
    assert f(frames, 1, 1078, 16, 256, 1, 64, 0, ex, st, out, None, None) == sw.SML_ERR_ALIGNMENT
    assert f(frames, 2 ** 32, 1076, 16, 256, 1, 64, 0, ex, st, out, None, None) == sw.SML_ERR_UNSUPPORTED
    cnt = (ctypes.c_uint64 * 3)()
    assert f(frames, 1, 1076, 16, 256, 1, 64, 0, ex, st, out, ctypes.addressof(cnt) + 4, None) == sw.SML_ERR_ALIGNMENT


@pytest.mark.parametrize("header", ["switchml_hip.h", "switchml_client.h"])
def test_public_header_is_plain_c(header, tmp_path):
    """The drop-in boundary is a C ABI: each public header compiles on its own
    as strict C99 (what a cgo / JNI / N-API stub includes) and as C++11, with
    every warning an error."""
    import os
    import shutil
    import subprocess
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    src = tmp_path / "inc.c"
    src.write_text(f'#include "{header}"\nint main(void) {{ return 0; }}\n')
    for cc, std in (("gcc", "-std=c99"), ("g++", "-std=c++11")):
        if not shutil.which(cc):
            pytest.skip(f"{cc} not found")
        lang = ["-x", "c++"] if cc == "g++" else []
        r = subprocess.run([cc, std, "-Wall", "-Wextra", "-pedantic", "-Werror", "-fsyntax-only", *lang, f"-I{inc}",
                            str(src)], capture_output=True, text=True)
        assert r.returncode == 0, (cc, r.stderr[-2000:])
