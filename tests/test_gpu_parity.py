"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Every comparison is bit-exact on the raw 32-bit words (payload planes are
compared as uint32, float outputs by their bit patterns).  The one documented
exception is the NaN payload of 0/0 in dequantize (scale 0 from a float
overflow of W*2^e, ppp.cc:258, times a zero word): x86 yields the default
NaN 0xffc00000, gfx950 0x7fc00000 — both sides are required to be NaN.

Oracle: oracle/sml_oracle.c (a CPU restatement of ppp.cc; "parity unpinned"
at the bit level).
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

PS = (64, 128, 256, 512, 1024)


def sw():
    import switchml_amd
    return switchml_amd


def to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def host(t):
    return t.detach().cpu().numpy()


def bits_equal(a, b):
    a = np.asarray(a).view(np.uint32)
    b = np.asarray(b).view(np.uint32)
    return np.array_equal(a, b)


def float_bits_equal_nan_ok(a, b):
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def special_values(n, rng):
    """Blocks of zeros, denormals, ties, NaN/inf, huge and tiny magnitudes."""
    x = rng.standard_normal(n).astype(np.float32)
    k = max(n // 16, 1)
    x[0:k] = 0.0
    x[k:2 * k] = (rng.integers(1, 1 << 23, size=len(x[k:2 * k])).astype(np.uint32)).view(np.float32)  # denormals
    x[2 * k:3 * k] = np.float32(1e-31) * rng.standard_normal(len(x[2 * k:3 * k])).astype(np.float32)
    x[3 * k:4 * k] = np.float32(3e38) * np.sign(rng.standard_normal(len(x[3 * k:4 * k]))).astype(np.float32)
    x[4 * k:5 * k] = (np.arange(len(x[4 * k:5 * k])) + 0.5).astype(np.float32) * np.float32(2.0 ** -20)  # ties
    if n > 8:
        x[5 * k + 1] = np.nan
        x[6 * k + 2] = np.inf
        x[6 * k + 3] = -np.inf
        x[7 * k + 1] = np.float32(2.0 ** -126)
        x[7 * k + 2] = -np.float32(2.0 ** -149)
    return x


def make_data(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        return O.splitmix_normal(seed + 42, n)
    if kind == "refrand":
        return O.c_ref_random_floats(seed + 1, n)
    if kind == "pattern":
        return O.ref_pattern_floats(n)
    if kind == "special":
        return special_values(n, rng)
    raise ValueError(kind)


SIZES = (1, 3, 63, 64, 65, 255, 256, 257, 1000, 1023, 1024, 1025, 4096 + 17, 100_003)


# ---------------------------------------------------------------- scales --

@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 7, 8, 16, 255, 256, 1000, 1024, 32768, 65535])
def test_scale_lut_device_equals_host_and_oracle(cuda, W):
    dev = host(sw().scale_lut_device(W, device=cuda))
    hst = sw().scale_lut(W)
    orc = O.scale_lut(W)
    assert bits_equal(dev, orc)
    assert bits_equal(hst, orc)


# ----------------------------------------------------------- K1 (fused) --

@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("kind", ["normal", "refrand", "pattern", "special"])
def test_quantize_pack_fused(cuda, P, kind):
    for W in (1, 2, 3, 8):
        for n in SIZES:
            x = make_data(kind, n, seed=n)
            payload, exps = sw().quantize_pack(to_dev(x, cuda), P, W)
            assert np.array_equal(host(exps), O.exponents(x, P)), (P, W, n)
            assert bits_equal(host(payload), O.quantize(x, P, W)), (P, W, n)


@pytest.mark.parametrize("P", PS)
def test_exponents_only(cuda, P):
    for n in SIZES:
        x = make_data("special", n, seed=n)
        e = sw().exponents(to_dev(x, cuda), P)
        assert np.array_equal(host(e), O.exponents(x, P)), (P, n)


@pytest.mark.parametrize("P", [64, 256, 1024])
@pytest.mark.parametrize("offset", [1, 2, 3, 5])
def test_misaligned_slice(cuda, P, offset):
    """Job slices start at arbitrary element offsets (fifo_scheduler.cc:93-109)."""
    import torch
    n = 50_000 + offset
    x = make_data("normal", n + 8, seed=offset)
    xd = to_dev(x, cuda)
    sl = xd[offset:offset + n]
    assert sl.data_ptr() % 16 != 0
    payload, exps = sw().quantize_pack(sl, P, 2)
    ref = O.quantize(x[offset:offset + n], P, 2)
    assert bits_equal(host(payload), ref)
    # dequantize into a misaligned output slice too
    outbuf = torch.zeros(n + 8, dtype=torch.float32, device=cuda)
    sw().dequantize(payload, exps, n, P, 2, out=outbuf[offset:offset + n])
    refd = O.dequantize(ref, host(exps), n, P, 2)
    assert float_bits_equal_nan_ok(host(outbuf[offset:offset + n]), refd)
    assert np.all(host(outbuf[:offset]) == 0) and np.all(host(outbuf[offset + n:]) == 0)


def test_slices_like_fifo_scheduler(cuda):
    """T=4 worker-thread slices of one job, blocks restarting at each slice."""
    N, T, P = 1_000_003, 4, 256
    x = make_data("normal", N, seed=7)
    xd = to_dev(x, cuda)
    for t in range(T):
        off, n = O.slice_geometry(N, T, t)
        payload, exps = sw().quantize_pack(xd[off:off + n], P, 1)
        assert bits_equal(host(payload), O.quantize(x[off:off + n], P, 1)), t
        assert np.array_equal(host(exps), O.exponents(x[off:off + n], P)), t


# ------------------------------------------------- K3 (global exponents) --

@pytest.mark.parametrize("P", PS)
def test_quantize_global_exponents(cuda, P):
    rng = np.random.default_rng(P)
    for n in (1, 257, 1025, 100_003):
        x = make_data("special", n, seed=n)
        B = O.num_blocks(n, P)
        local = O.exponents(x, P)
        # switch semantics (>= local) and arbitrary int8 exponents, which
        # drive products past 2^31 (the x86 64-bit-truncation path) and to inf.
        above = np.clip(local.astype(np.int32) + rng.integers(0, 4, B), -128, 127).astype(np.int8)
        arbitrary = rng.integers(-128, 128, B).astype(np.int8)
        for ge in (above, arbitrary):
            for W in (1, 3):
                payload, e = sw().quantize_pack(to_dev(x, cuda), P, W, global_exps=to_dev(ge, cuda))
                assert bits_equal(host(payload), O.quantize(x, P, W, global_exps=ge)), (P, n, W)


def test_wide_conversion_wraps_like_x86(cuda):
    """|round(x*s)| >= 2^31: gcc's cvttss2si-to-64-bit then truncate (ppp.cc:103)."""
    P = 256
    vals = np.array([2.0 ** 31, -2.0 ** 31, 2.0 ** 32 + 2.0 ** 9, 3.0 * 2.0 ** 40, -(2.0 ** 33 - 2.0 ** 9),
                     2.0 ** 62, 2.0 ** 63, -2.0 ** 63, 1e30, np.inf, -np.inf, np.nan], dtype=np.float32)
    x = np.zeros(P, dtype=np.float32)
    x[: vals.size] = vals
    ge = np.array([0], dtype=np.int8)  # scale 2^31 -> x*s = x*2^31
    for W in (1, 2):
        payload, _ = sw().quantize_pack(to_dev(x / np.float32(2.0 ** 31), cuda), P, W, global_exps=to_dev(ge, cuda))
        assert bits_equal(host(payload), O.quantize(x / np.float32(2.0 ** 31), P, W, global_exps=ge))


# ------------------------------------------------------------ flags ------

@pytest.mark.parametrize("P", PS)
def test_payload_le_flag(cuda, P):
    x = make_data("normal", 100_003, seed=P)
    be, _ = sw().quantize_pack(to_dev(x, cuda), P, 2)
    le, _ = sw().quantize_pack(to_dev(x, cuda), P, 2, flags=sw().FLAG_PAYLOAD_LE)
    assert bits_equal(host(le), O.bswap32(host(be)))


@pytest.mark.parametrize("P", PS)
def test_rne_vcl_mode(cuda, P):
    """VCL=1 semantics (parity unpinned; restated in the oracle as rounding=1)."""
    for n in (17, 255, 1025, 100_003):
        x = make_data("special", n, seed=n)
        payload, _ = sw().quantize_pack(to_dev(x, cuda), P, 1, flags=sw().FLAG_ROUND_RNE)
        assert bits_equal(host(payload), O.quantize(x, P, 1, rounding=O.RNE_VCL)), (P, n)


# ------------------------------------------------------------- K4 / K5 ---

@pytest.mark.parametrize("P", PS)
def test_dequantize_arbitrary_words(cuda, P):
    rng = np.random.default_rng(P + 1)
    for n in (1, 63, 1025, 100_003):
        B = O.num_blocks(n, P)
        words = rng.integers(0, 2 ** 32, B * P, dtype=np.uint64).astype(np.uint32)
        exps = rng.integers(-128, 128, B).astype(np.int8)
        for W in (1, 3, 8, 65535):
            out = sw().dequantize(to_dev(words.view(np.int32), cuda), to_dev(exps, cuda), n, P, W)
            assert float_bits_equal_nan_ok(host(out), O.dequantize(words, exps, n, P, W)), (P, n, W)


@pytest.mark.parametrize("W", [1, 2, 3, 8, 65535])
@pytest.mark.parametrize("count", [4096 * 4, 4100, 100_004])
def test_loopback_aggregate(cuda, W, count):
    rng = np.random.default_rng(W)
    words = rng.integers(0, 2 ** 32, count, dtype=np.uint64).astype(np.uint32)
    d = to_dev(words.view(np.int32), cuda)
    sw().loopback_aggregate(d, W)
    assert bits_equal(host(d), O.loopback_aggregate(words, W))
    d2 = to_dev(O.bswap32(words).view(np.int32), cuda)
    sw().loopback_aggregate(d2, W, flags=sw().FLAG_PAYLOAD_LE)
    assert bits_equal(O.bswap32(host(d2)), O.loopback_aggregate(words, W))


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 100_003])
@pytest.mark.parametrize("offset", [0, 1])
def test_bswap_int32(cuda, n, offset):
    rng = np.random.default_rng(n)
    words = rng.integers(-2 ** 31, 2 ** 31, n + 4, dtype=np.int64).astype(np.int32)
    d = to_dev(words, cuda)
    out = sw().bswap_i32(d[offset:offset + n])
    assert bits_equal(host(out), O.bswap32(words[offset:offset + n]))
    # in place (the reference swaps the packet buffer in place, ppp.cc:158-190)
    v = d[offset:offset + n]
    sw().bswap_i32(v, out=v)
    assert bits_equal(host(v), O.bswap32(words[offset:offset + n]))


# -------------------------------------------------------- round trips ----

@pytest.mark.parametrize("P", PS)
@pytest.mark.parametrize("kind", ["normal", "refrand", "special"])
def test_roundtrip_loopback_matches_dummy_packet_loop(cuda, P, kind):
    import torch
    for W in (1, 2, 3, 8):
        for n in (1, 257, 1025, 100_003):
            x = make_data(kind, n, seed=n)
            ref = O.dummy_allreduce(x, P=P, num_worker_threads=1, num_workers=W)
            xd = to_dev(x, cuda)
            B = O.num_blocks(n, P)
            payload = torch.empty(B * P, dtype=torch.int32, device=cuda)
            exps = torch.empty(B, dtype=torch.int8, device=cuda)
            out = sw().roundtrip_loopback(xd, P, W, payload=payload, exps_out=exps)
            assert float_bits_equal_nan_ok(host(out), ref), (P, W, n)
            assert bits_equal(host(payload), O.quantize(x, P, W))
            assert np.array_equal(host(exps), O.exponents(x, P))
            # the three-kernel path K1 -> K5 -> K4 gives the same bits
            p2, e2 = sw().quantize_pack(xd, P, W)
            sw().loopback_aggregate(p2, W)
            out2 = sw().dequantize(p2, e2, n, P, W)
            assert float_bits_equal_nan_ok(host(out2), ref)


def test_packet_stream_mapping(cuda):
    """Planes <-> the reference packet stream: packet p carries
    exps[p] (p < B) and payload block p-b (p >= b)."""
    P, n = 256, 40_000
    x = make_data("normal", n, seed=3)
    pkt_exps, pkt_payload, _, b = O.dummy_packet_stream(x, P=P, batch_max=64, num_workers=1)
    payload, exps = sw().quantize_pack(to_dev(x, cuda), P, 1)
    B = O.num_blocks(n, P)
    pl = host(payload).view(np.uint32).reshape(B, P)
    ex = host(exps)
    assert np.array_equal(pkt_exps[:B], ex)
    last_n = n - (B - 1) * P
    assert bits_equal(pkt_payload[b:b + B - 1], pl[:B - 1])
    assert bits_equal(pkt_payload[b + B - 1][:last_n], pl[B - 1][:last_n])


# ------------------------------------------------- full-size configs -----

def test_cfg2_64mib_bit_exact(cuda):
    """BASELINE configs[1]: 64 MiB fp32 bucket, 256-element packets, W=1."""
    N, P = 16 * 1024 * 1024, 256
    for x in (O.splitmix_normal(42, N), O.c_ref_random_floats(1, N)):
        payload, exps = sw().quantize_pack(to_dev(x, cuda), P, 1)
        assert np.array_equal(host(exps), O.exponents(x, P))
        assert bits_equal(host(payload), O.quantize(x, P, 1))


def test_cfg3_256mib_roundtrip(cuda):
    """BASELINE configs[2]: 256 MiB, quantize -> loopback (x W) -> dequantize.
    Output bit-identical to the oracle's packet loop.  Error vs W*x for a
    power-of-two W (scale exact, product exact): |out - W x| <= 1/2 * W^2 *
    2^(e-31) + 1/2 ulp(out)  (q rounding, times W, over s = 2^(31-e)/W; plus
    the int->float conversion of W*q)."""
    import torch
    N, P = 64 * 1024 * 1024, 256
    x = O.splitmix_normal(42, N)
    xd = to_dev(x, cuda)
    for W in (1, 2):
        out = sw().roundtrip_loopback(xd, P, W)
        ref = O.dummy_allreduce(x, P=P, num_worker_threads=1, num_workers=W)
        o = host(out)
        assert bits_equal(o, ref)
        e = O.exponents(x, P).astype(np.int32)
        bound = 0.5 * W * W * np.ldexp(1.0, np.repeat(e, P)[:N] - 31) + 0.5 * np.spacing(np.abs(o)).astype(np.float64)
        err = np.abs(o.astype(np.float64) - W * x.astype(np.float64))
        assert np.all(err <= bound * 1.0000001)
        del out
        torch.cuda.empty_cache()


def test_beyond_2_31_elements_sampled_blocks(cuda):
    """Maximum sizes: a 2^31 + 300-element slice (8 GiB fp32; element and byte
    offsets past 32 bits).  Blocks are independent once their exponent is
    known, so sampled blocks (first, around 2^31, the partial last) are
    checked against the oracle run on those blocks alone."""
    import torch
    N, P, W = (1 << 31) + 300, 256, 2
    g = torch.Generator(device=cuda)
    g.manual_seed(3)
    x = torch.randn(N, device=cuda, generator=g)
    payload, exps = sw().quantize_pack(x, P, W)
    B = O.num_blocks(N, P)
    assert payload.numel() == B * P
    for k in (0, 1, (1 << 23) - 1, 1 << 23, (1 << 23) + 1, B - 2, B - 1):
        blk = host(x[k * P:min((k + 1) * P, N)])
        assert int(host(exps[k:k + 1])[0]) == int(O.exponents(blk, P)[0]), k
        assert bits_equal(host(payload[k * P:(k + 1) * P]), O.quantize(blk, P, W)), k
    out = sw().dequantize(payload, exps, N, P, W)
    for k in (0, 1 << 23, B - 1):
        blk_q = host(payload[k * P:(k + 1) * P]).view(np.uint32)
        n = min(P, N - k * P)
        ref = O.dequantize(blk_q, host(exps[k:k + 1]), n, P, W)
        assert float_bits_equal_nan_ok(host(out[k * P:k * P + n]), ref), k
    del x, payload, exps, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("P", [64, 256, 1024])
def test_quantize_pack_launcher(cuda, P):
    """switchml_amd.quantize_pack_launcher (one prepared C call per launch, the
    bench's step): the same planes as the oracle, twice in a row, and K3 with
    global exponents through it."""
    import torch
    n, W = 100_003, 3
    x = O.splitmix_normal(P + 9, n)
    xd = torch.from_numpy(x).cuda()
    B = sw().num_blocks(n, P)
    pl = torch.empty(B * P, dtype=torch.int32, device="cuda")
    ex = torch.empty(B, dtype=torch.int8, device="cuda")
    go = sw().quantize_pack_launcher(xd, P, W, pl, exps_out=ex)
    for _ in range(2):
        pl.zero_()
        go()
        torch.cuda.synchronize()
        assert bits_equal(host(pl), O.quantize(x, P, W))
        assert np.array_equal(host(ex), O.exponents(x, P))
    g = torch.from_numpy(O.exponents(x, P) + 1).cuda()
    k3 = sw().quantize_pack_launcher(xd, P, W, pl, global_exps=g)
    k3()
    torch.cuda.synchronize()
    assert bits_equal(host(pl), O.quantize(x, P, W, global_exps=O.exponents(x, P) + 1))
    with pytest.raises(ValueError):
        sw().quantize_pack_launcher(xd, P, W, pl[:-1])
