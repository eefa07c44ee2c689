"""GPU: the streaming kernels give the same bytes under every launch geometry.

The workgroup -> data mapping is a permutation (XCD-aware order,
`sml_set_xcd_chunk`) and the grid may be capped
(`sml_set_grid_limit`, grid-stride loops), so a bug in either would move or
drop tiles.  Every kernel of the path runs under several (grid cap, XCD chunk)
pairs — grid sizes that are and are not multiples of 8 x chunk, so the
permuted head and the identity tail both occur — and must reproduce the
oracle (or, for kernels without a direct oracle call, the default geometry's
output) bit for bit.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# (grid cap, xcd chunk): default, plain order, odd chunks, small caps (grid-stride), cap not a multiple of 8
GEOMETRIES = [(0, 64), (0, 0), (0, 1), (0, 3), (40, 64), (40, 1), (1000, 7), (13, 2), (8, 1)]


@pytest.fixture
def sw(cuda):
    import switchml_amd
    yield switchml_amd
    switchml_amd.set_grid_limit(0)
    switchml_amd.set_xcd_chunk(64)


def _run_all(sw, torch, x, P, W):
    dev = x.device
    n = x.numel()
    payload, exps = sw.quantize_pack(x, P, W)
    le, _ = sw.quantize_pack(x, P, W, global_exps=exps, flags=sw.FLAG_PAYLOAD_LE)
    e_only = sw.exponents(x, P)
    agg = payload.clone()
    sw.loopback_aggregate(agg, W)
    deq = sw.dequantize(agg, exps, n, P, W)
    rt = sw.roundtrip_loopback(x, P, W)
    sw_ = sw.bswap_i32(payload)
    fp = sw.frame_params(max_outstanding_pkts=64)
    frames = sw.quantize_pack_frames(x, fp, P, W, batch_max=64)
    rx = sw.RxSlice(n, P, 64, device=dev)
    nframes = frames.numel() // sw.frame_bytes(P)
    sw.dequantize_frames(frames, nframes, rx, num_workers=W)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy().copy() for k, v in dict(payload=payload, exps=exps, le=le, e_only=e_only,
                                                      agg=agg, deq=deq, rt=rt, bswap=sw_, frames=frames,
                                                      rx_out=rx.out, rx_exps=rx.exps).items()}


@pytest.mark.parametrize("P,n", [(256, 1_000_003), (64, 300_001), (1024, 777_777)])
def test_every_kernel_geometry_invariant(sw, P, n):
    import torch
    W = 3
    x_np = O.splitmix_normal(P + n, n)
    x = torch.from_numpy(x_np).cuda()
    ref = None
    for cap, chunk in GEOMETRIES:
        sw.set_grid_limit(cap)
        sw.set_xcd_chunk(chunk)
        got = _run_all(sw, torch, x, P, W)
        if ref is None:
            # the default geometry against the oracle first
            assert np.array_equal(got["payload"].view(np.uint32), O.quantize(x_np, P, W))
            assert np.array_equal(got["exps"], O.exponents(x_np, P))
            dq = O.dequantize(O.loopback_aggregate(O.quantize(x_np, P, W), W), O.exponents(x_np, P), n, P, W)
            assert np.array_equal(got["deq"].view(np.uint32), dq.view(np.uint32))
            assert np.array_equal(got["rt"].view(np.uint32), dq.view(np.uint32))
            # frames go tx -> rx without a switch in between: the sent words come back
            rx = O.dequantize(O.quantize(x_np, P, W), O.exponents(x_np, P), n, P, W)
            assert np.array_equal(got["rx_out"].view(np.uint32), rx.view(np.uint32))
            ref = got
            continue
        for k in ref:
            assert np.array_equal(got[k], ref[k]), (k, cap, chunk)


def test_misaligned_slice_geometry_invariant(sw):
    """4-byte-offset slices (the unaligned vector path) under capped grids."""
    import torch
    P, W, n = 256, 2, 262_147
    x_np = O.splitmix_normal(11, n + 3)
    xd = torch.from_numpy(x_np).cuda()
    for off in (1, 2, 3):
        xs = xd[off:off + n]
        want = O.quantize(x_np[off:off + n], P, W)
        for cap, chunk in GEOMETRIES:
            sw.set_grid_limit(cap)
            sw.set_xcd_chunk(chunk)
            payload, _ = sw.quantize_pack(xs, P, W)
            assert np.array_equal(payload.cpu().numpy().view(np.uint32), want), (off, cap, chunk)


@pytest.mark.parametrize("P", [64, 128, 256, 512, 1024])
def test_quantize_tile_slices_invariant(sw, P):
    """K1 / K2 / K3 with every wave-tile size (sml_set_quantize_tile_slices:
    0 = the default (2), 1, 2, 4 slices of 256 elements, never
    below P / 256) under capped grids
    and XCD orders, aligned and 4-byte-offset slices, RNE and LE flags: the
    same bytes as the oracle."""
    import torch
    W, n = 3, 200_003
    x_np = O.splitmix_normal(P + 5, n + 1)
    xd = torch.from_numpy(x_np).cuda()
    orig = sw.set_payload_nt_threshold(2 ** 64 - 1)       # the library default, restored below
    try:
        for off in (0, 1):
            xs, xn = xd[off:off + n], x_np[off:off + n]
            want_q, want_e = O.quantize(xn, P, W), O.exponents(xn, P)
            want_rne = O.quantize(xn, P, W, rounding=O.RNE_VCL)
            for sl, nt in ((0, 0), (1, 0), (2, 0), (4, 0), (4, 2 ** 64 - 1)):
                sw.set_quantize_tile_slices(sl)
                sw.set_payload_nt_threshold(nt)      # 0: non-temporal payload stores; max: default policy
                for cap, chunk in GEOMETRIES[:3] + GEOMETRIES[6:8]:
                    sw.set_grid_limit(cap)
                    sw.set_xcd_chunk(chunk)
                    payload, exps = sw.quantize_pack(xs, P, W)
                    e_only = sw.exponents(xs, P)
                    k3, _ = sw.quantize_pack(xs, P, W, global_exps=exps, flags=sw.FLAG_PAYLOAD_LE)
                    rne, _ = sw.quantize_pack(xs, P, W, flags=sw.FLAG_ROUND_RNE)
                    torch.cuda.synchronize()
                    tag = (off, sl, cap, chunk)
                    assert np.array_equal(payload.cpu().numpy().view(np.uint32), want_q), tag
                    assert np.array_equal(exps.cpu().numpy(), want_e), tag
                    assert np.array_equal(e_only.cpu().numpy(), want_e), tag
                    assert np.array_equal(k3.cpu().numpy().view(np.uint32), want_q.byteswap()), tag
                    assert np.array_equal(rne.cpu().numpy().view(np.uint32), want_rne), tag
    finally:
        sw.set_quantize_tile_slices(0)
        sw.set_payload_nt_threshold(orig)


@pytest.mark.parametrize("P", [64, 256, 1024])
def test_output_store_policy_invariant(sw, P):
    """K1, K4 and the fused round trip with their output planes written
    non-temporally (sml_set_payload_nt_threshold(0): what planes of 64 MiB
    and more get) and with default-policy stores: the same bytes
    as the oracle, aligned and 4-byte-offset slices."""
    import torch
    W, n = 3, 300_007
    x_np = O.splitmix_normal(P + 77, n + 1)
    xd = torch.from_numpy(x_np).cuda()
    orig = sw.set_payload_nt_threshold(2 ** 64 - 1)       # the library default, restored below
    try:
        for off in (0, 1):
            xs, xn = xd[off:off + n], x_np[off:off + n]
            q, e = O.quantize(xn, P, W), O.exponents(xn, P)
            dq = O.dequantize(O.loopback_aggregate(q, W), e, n, P, W)
            for nt in (0, 2 ** 64 - 1):
                sw.set_payload_nt_threshold(nt)
                payload, exps = sw.quantize_pack(xs, P, W)
                agg = payload.clone()
                sw.loopback_aggregate(agg, W)
                out = torch.empty(n + 1, device="cuda")[off:off + n]
                sw.dequantize(agg, exps, n, P, W, out=out)
                rt = torch.empty(n + 1, device="cuda")[off:off + n]
                sw.roundtrip_loopback(xs, P, W, out=rt)
                torch.cuda.synchronize()
                assert np.array_equal(payload.cpu().numpy().view(np.uint32), q), (off, nt)
                assert np.array_equal(out.cpu().numpy().view(np.uint32), dq.view(np.uint32)), (off, nt)
                assert np.array_equal(rt.cpu().numpy().view(np.uint32), dq.view(np.uint32)), (off, nt)
    finally:
        sw.set_payload_nt_threshold(orig)


@pytest.mark.parametrize("P", [64, 256, 512, 1024])
def test_stream_tile_slices_invariant(sw, P):
    """K4 and the fused round trip with 2- and 4-slice wave tiles
    (sml_set_stream_tile_slices; P = 1024 keeps 4 in the round trip), both
    store policies, capped grids and XCD orders, aligned and 4-byte-offset
    slices, W = 3 (IEEE division) and W = 4 (exact reciprocal): the oracle's
    bytes, and the round trip's payload and exponent planes too."""
    import torch
    n = 200_003
    x_np = O.splitmix_normal(P + 91, n + 1)
    xd = torch.from_numpy(x_np).cuda()
    orig = sw.set_payload_nt_threshold(2 ** 64 - 1)
    try:
        for W in (3, 4):
            for off in (0, 1):
                xs, xn = xd[off:off + n], x_np[off:off + n]
                q, e = O.quantize(xn, P, W), O.exponents(xn, P)
                dq = O.dequantize(O.loopback_aggregate(q, W), e, n, P, W)
                for sl, nt in ((2, 0), (4, 0), (2, 2 ** 64 - 1), (0, 0)):
                    sw.set_stream_tile_slices(sl)
                    sw.set_payload_nt_threshold(nt)
                    for cap, chunk in GEOMETRIES[:2] + GEOMETRIES[6:8]:
                        sw.set_grid_limit(cap)
                        sw.set_xcd_chunk(chunk)
                        payload, exps = sw.quantize_pack(xs, P, W)
                        sw.loopback_aggregate(payload, W)
                        out = torch.empty(n + 1, device="cuda")[off:off + n]
                        sw.dequantize(payload, exps, n, P, W, out=out)
                        rt = torch.empty(n + 1, device="cuda")[off:off + n]
                        rt_q = torch.empty_like(payload)
                        rt_e = torch.empty_like(exps)
                        sw.roundtrip_loopback(xs, P, W, out=rt, payload=rt_q, exps_out=rt_e)
                        torch.cuda.synchronize()
                        tag = (W, off, sl, nt, cap, chunk)
                        assert np.array_equal(out.cpu().numpy().view(np.uint32), dq.view(np.uint32)), tag
                        assert np.array_equal(rt.cpu().numpy().view(np.uint32), dq.view(np.uint32)), tag
                        assert np.array_equal(rt_q.cpu().numpy().view(np.uint32), q), tag
                        assert np.array_equal(rt_e.cpu().numpy(), e), tag
    finally:
        sw.set_stream_tile_slices(0)
        sw.set_grid_limit(0)
        sw.set_xcd_chunk(64)
        sw.set_payload_nt_threshold(orig)
