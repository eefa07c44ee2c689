"""K6 sml_switch_aggregate (the switch's aggregation over W worker planes,
fused with the dequantize) against the oracle's software switch.

Oracle chain, per case: W workers each quantize their own input with the
global exponents (O.quantize with global_exps = orc_switch_exps of the
workers' exponent planes: the look-ahead step, ppp.cc:115-156), then
orc_switch_payload (wrapping bit<32> sum of ntohl'd words,
p4/processor.p4:48-54) and orc_switch_exps (signed int8 max,
p4/exponents.p4:48-54), then orc_dequantize with W (ppp.cc:197-251).
Bit-exact on the raw words; the only tolerated difference is the NaN payload
bits of 0/0 (see test_gpu_parity.py).
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

from test_gpu_parity import float_bits_equal_nan_ok, host, special_values, to_dev  # noqa: E402


def sw():
    import switchml_amd
    return switchml_amd


def worker_planes(W, n, P, seed, special=False):
    rng = np.random.default_rng(seed)
    xs = [special_values(n, rng) if special and w == 0 else O.splitmix_normal(seed * 31 + w, n, sigma=10.0 ** -w)
          for w in range(W)]
    gexp = O.switch_exps([O.exponents(x, P) for x in xs])
    pls = [O.quantize(x, P, W, global_exps=gexp) for x in xs]
    return xs, gexp, pls


def oracle_switch(pls, exps, n, P, W):
    agg = O.switch_payload(pls)
    e = O.switch_exps(exps)
    return agg, e, O.dequantize(agg, e, n, P, W)


@pytest.mark.parametrize("P", (64, 128, 256, 512, 1024))
@pytest.mark.parametrize("W", (1, 2, 3, 8))
def test_switch_aggregate_matches_oracle(P, W):
    import torch
    dev = torch.device("cuda:0")
    n = 37 * 1024 + 101                     # ragged: partial last block and partial last tile
    xs, gexp, pls = worker_planes(W, n, P, seed=P + W, special=(W == 2))
    # each worker's exponent plane = the global one (what it got back from the switch);
    # perturb the non-zero workers downwards so the kernel's max is exercised
    exps = [gexp.copy() for _ in range(W)]
    for w in range(1, W):
        exps[w] = np.maximum(exps[w].astype(np.int16) - w, -128).astype(np.int8)
    agg, e, out = oracle_switch(pls, exps, n, P, W)
    B = O.num_blocks(n, P)
    d_pl = [to_dev(p.view(np.int32), dev) for p in pls]
    d_ex = [to_dev(x, dev) for x in exps]
    p_out = torch.empty(B * P, dtype=torch.int32, device=dev)
    e_out = torch.empty(B, dtype=torch.int8, device=dev)
    o = sw().switch_aggregate(d_pl, d_ex, n, P, payload_out=p_out, exps_out=e_out,
                              out=torch.empty(n, dtype=torch.float32, device=dev))
    torch.cuda.synchronize()
    assert np.array_equal(host(p_out).view(np.uint32), agg)
    assert np.array_equal(host(e_out), e)
    assert float_bits_equal_nan_ok(host(o), out)


@pytest.mark.parametrize("P", (64, 256))
def test_switch_aggregate_max_workers(P):
    """SML_MAX_SWITCH_WORKERS (16) planes, fused dequantize, W = 16 scale."""
    import torch
    dev = torch.device("cuda:0")
    W, n = 16, 5 * 1024 + 33
    _, gexp, pls = worker_planes(W, n, P, seed=16 + P)
    exps = [gexp] * W
    agg, e, out = oracle_switch(pls, exps, n, P, W)
    d_pl = [to_dev(p.view(np.int32), dev) for p in pls]
    d_ex = [to_dev(gexp, dev)] * W
    o = sw().switch_aggregate(d_pl, d_ex, n, P)
    torch.cuda.synchronize()
    assert float_bits_equal_nan_ok(host(o), out)


@pytest.mark.parametrize("W", (2, 5, 16))
def test_switch_aggregate_le_payload_only(W):
    """LE words (SML_FLAG_PAYLOAD_LE), payload only, in place into plane 0."""
    import torch
    dev = torch.device("cuda:0")
    P, n = 256, 64 * 1024
    _, _, pls = worker_planes(W, n, P, seed=W)
    agg_be = O.switch_payload(pls)
    d_pl = [to_dev(O.bswap32(p).view(np.int32), dev) for p in pls]   # host-order words
    sw().switch_aggregate(d_pl, None, n, P, payload_out=d_pl[0], flags=sw().FLAG_PAYLOAD_LE)
    torch.cuda.synchronize()
    assert np.array_equal(host(d_pl[0]).view(np.uint32), O.bswap32(agg_be))


def test_switch_aggregate_unaligned_out_and_exps():
    """fp32 output at a 4-byte (not 16-byte) offset and exponent planes at odd
    byte offsets (per-lane byte loads instead of the scalar slice load)."""
    import torch
    dev = torch.device("cuda:0")
    P, W, n = 64, 3, 9 * 1024 + 7
    _, gexp, pls = worker_planes(W, n, P, seed=5)
    exps = [gexp] * W
    _, _, out = oracle_switch(pls, exps, n, P, W)
    B = O.num_blocks(n, P)
    d_pl = [to_dev(p.view(np.int32), dev) for p in pls]
    raw = [torch.empty(B + 1, dtype=torch.int8, device=dev) for _ in range(W)]
    d_ex = [r[1:] for r in raw]
    for d in d_ex:
        d.copy_(to_dev(gexp, dev))
    big = torch.empty(n + 1, dtype=torch.float32, device=dev)
    sw().switch_aggregate(d_pl, d_ex, n, P, out=big[1:])
    torch.cuda.synchronize()
    assert float_bits_equal_nan_ok(host(big[1:]), out)


def test_switch_aggregate_equals_loopback_roundtrip():
    """W identical workers through K6 == the dummy backend's x W loopback
    round trip (dummy_backend.cc:72-84), bit for bit, at 16 M elements."""
    import torch
    dev = torch.device("cuda:0")
    P, W, n = 256, 4, 16 * 1024 * 1024
    x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    payload, exps = sw().quantize_pack(x, P, W)
    o = sw().switch_aggregate([payload] * W, [exps] * W, n, P)
    ref = sw().roundtrip_loopback(x, P, W)
    torch.cuda.synchronize()
    assert torch.equal(o.view(torch.int32), ref.view(torch.int32))


def test_switch_aggregate_rejects_bad_args():
    import torch
    dev = torch.device("cuda:0")
    S = sw()
    pl = torch.zeros(1024, dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        S.switch_aggregate([pl] * 17, None, 1024, 256, payload_out=pl)
    with pytest.raises(ValueError):
        S.switch_aggregate([pl, pl[:512]], None, 1024, 256, payload_out=pl)
    with pytest.raises(S.SwitchMLError):
        S.switch_aggregate([pl], None, 1024, 256)   # out needs exponents
    ptrs = (ctypes.c_void_p * 1)(pl.data_ptr())
    st = S.lib().sml_switch_aggregate(ctypes.cast(ptrs, ctypes.c_void_p), None, 1, 1024, 100,
                                      ctypes.c_void_p(pl.data_ptr()), None, None, 0, None)
    assert st == 2   # SML_ERR_UNSUPPORTED: packet_numel not in {64..1024}
    st = S.lib().sml_switch_aggregate(ctypes.cast(ptrs, ctypes.c_void_p), None, 1, 1024, 256,
                                      ctypes.c_void_p(pl.data_ptr() + 4), None, None, 0, None)
    assert st == 3   # SML_ERR_ALIGNMENT: output plane not 16-byte aligned


@pytest.mark.parametrize("sizes,offs", [
    ([1000, 1000, 999], [0, 0, 0]),
    ([16384 * 3 + 5, 0, 1, 17, 16384 * 16 + 1024, 33], [1, 0, 2, 3, 0, 1]),
    ([1 << 20] * 8, [0, 1, 2, 3, 0, 1, 2, 3]),
    ([(1 << 22) + 7] * 15 + [3], [3] * 16),
])
def test_copy_segments(cuda, sizes, offs):
    """sml_copy_segments (the in-node switch's multicast in one launch: tiles
    dealt round-robin over the segments in 64 KiB groups): every segment
    copied exactly — ragged, empty, one-word and 4-byte-offset segments —
    and nothing outside the segments written."""
    import torch
    import switchml_amd as sw
    g = torch.Generator(device="cuda")
    g.manual_seed(sum(sizes))
    total = sum(n + o for n, o in zip(sizes, offs)) + 64
    src = torch.randint(-2**31, 2**31 - 1, (total,), dtype=torch.int32, device="cuda", generator=g)
    dst = torch.full((total,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    want = dst.clone()
    pairs, pos = [], 0
    for n, o in zip(sizes, offs):
        pos += o
        pairs.append((src[pos:pos + n], dst[pos:pos + n]))
        want[pos:pos + n] = src[pos:pos + n]
        pos += n
    sw.copy_segments(pairs)
    torch.cuda.synchronize()
    assert torch.equal(dst, want)
