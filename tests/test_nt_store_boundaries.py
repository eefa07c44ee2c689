"""Non-temporal output stores across 32-bit address boundaries (GPU).

The 16-byte-aligned large outputs (K1 payload planes, K4, the fused round
trip, the frames rx output, the copy probe) take `sc1 nt` buffer stores whose
descriptor base is derived from the wave's first active lane's address
(`SML_NT_STORE16`, sml_device.h).  Round 4's first build of it sign-extended
the low address word, which faulted for every address whose low word is
>= 2^31.  Here each output is placed inside one 4 GiB + arena so that a
store slice straddles the low-word 2^31 boundary, then the 2^32 one (the
first lane below, the others above), with the non-temporal policy forced
(threshold 0); every byte must equal the oracle's / the default-policy run's.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sw(cuda):
    import switchml_amd as sw
    return sw


@pytest.fixture(scope="module")
def arena(cuda):
    import torch
    a = torch.empty((4 << 30) + (32 << 20), dtype=torch.uint8, device=cuda)
    yield a
    del a
    torch.cuda.empty_cache()


def _view(arena, boundary, nbytes, dtype):
    """A view of `nbytes` whose address crosses `boundary` (mod 2^32) 512
    bytes into a 1 KiB store slice."""
    base = arena.data_ptr()
    start = (boundary - nbytes // 2 - 512 - base) % (1 << 32)
    start -= start % 16
    assert start + nbytes <= arena.numel()
    v = arena[start:start + nbytes].view(dtype)
    lo0, lo1 = (v.data_ptr() % (1 << 32)), ((v.data_ptr() + nbytes) % (1 << 32))
    assert lo0 > lo1 if boundary == 1 << 32 else lo0 < boundary <= lo1
    return v


@pytest.mark.parametrize("boundary", [1 << 31, 1 << 32], ids=["2^31", "2^32"])
@pytest.mark.parametrize("P", [64, 256, 1024])
def test_nt_outputs_across_address_boundaries(sw, arena, boundary, P):
    import torch
    W, n = 2, 262_147
    x_np = O.splitmix_normal(P + 313, n)
    x = torch.from_numpy(x_np).cuda()
    B = sw.num_blocks(n, P)
    q, e = O.quantize(x_np, P, W), O.exponents(x_np, P)
    dq = O.dequantize(O.loopback_aggregate(q, W), e, n, P, W)
    orig = sw.set_payload_nt_threshold(0)
    try:
        # K1: payload plane across the boundary
        pl = _view(arena, boundary, 4 * B * P, torch.int32)
        _, exps = sw.quantize_pack(x, P, W, payload=pl)
        torch.cuda.synchronize()
        assert np.array_equal(pl.cpu().numpy().view(np.uint32), q)
        assert np.array_equal(exps.cpu().numpy(), e)
        # K4: fp32 output across the boundary
        agg = torch.from_numpy(O.loopback_aggregate(q, W).view(np.int32)).cuda()
        out = _view(arena, boundary, 4 * n, torch.float32)
        sw.dequantize(agg, exps, n, P, W, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), dq.view(np.uint32))
        # fused round trip
        out.zero_()
        sw.roundtrip_loopback(x, P, W, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), dq.view(np.uint32))
        # copy probe (whole tiles)
        m = 1 << 20
        src = torch.arange(m, dtype=torch.int32, device="cuda")
        dst = _view(arena, boundary, 4 * m, torch.int32)
        sw.stream_copy(src, dst)
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
    finally:
        sw.set_payload_nt_threshold(orig)


@pytest.mark.parametrize("boundary", [1 << 31, 1 << 32], ids=["2^31", "2^32"])
def test_frames_rx_output_across_address_boundaries(sw, arena, boundary):
    """The rx apply pass's fp32 output (W = 1 loopback frames) across the
    boundary: equal to the fused round trip."""
    import torch
    P, n = 256, 262_147
    x = torch.from_numpy(O.splitmix_normal(911, n)).cuda()
    fp = sw.frame_params(max_outstanding_pkts=64)
    frames = sw.quantize_pack_frames(x, fp, P, 1, batch_max=64)
    nframes = frames.numel() // sw.frame_bytes(P)
    ref = sw.roundtrip_loopback(x, P, 1)
    orig = sw.set_payload_nt_threshold(0)
    try:
        out = _view(arena, boundary, 4 * n, torch.float32)
        rx = sw.RxSlice(n, P, 64, device=x.device, out=out)
        rx.reset()
        sw.dequantize_frames(frames, nframes, rx, num_workers=1)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    finally:
        sw.set_payload_nt_threshold(orig)
