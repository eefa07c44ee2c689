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
    assert L.sml_abi_version() == 1
    for code, name in [(0, b"SML_OK"), (1, b"SML_ERR_INVALID_ARG"), (2, b"SML_ERR_UNSUPPORTED"),
                       (3, b"SML_ERR_ALIGNMENT"), (4, b"SML_ERR_HIP")]:
        assert L.sml_status_string(code) == name


@pytest.mark.parametrize("numel,P", [(0, 256), (1, 64), (255, 256), (256, 256), (257, 256),
                                     (16 * 2 ** 20, 256), (67_108_864, 1024), (10 ** 12 + 3, 64)])
def test_num_blocks_matches_oracle(sw, numel, P):
    assert sw.num_blocks(numel, P) == O.num_blocks(numel, P)


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


def test_grid_limit_knob(sw):
    prev = sw.set_grid_limit(1024)
    assert sw.set_grid_limit(prev) == 1024


def test_python_wrapper_rejects_cpu_tensors(sw):
    torch = pytest.importorskip("torch")
    with pytest.raises(TypeError, match="no CPU fallback"):
        sw.quantize_pack(torch.zeros(16))
