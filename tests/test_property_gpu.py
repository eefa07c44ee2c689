"""GPU property tests: randomized slices (Hypothesis, derandomized so every
run checks the same cases) through every plane kernel, bit-exact against the
oracle.  Each example draws a slice length, a start offset inside a larger
buffer (4-byte misalignments included), a packet size, a worker count, a
magnitude scale and a data family, and checks

  K1 quantize+pack (BE and LE), K2 exponents, K3 with other global exponents,
  K4 dequantize of the loopback-aggregated payload, the fused round trip,
  and the RNE (VCL=1) mode

against oracle/sml_oracle.c.  The one documented non-bit-exact case, the
sign of the 0/0 NaN, is compared as "both NaN" (DESIGN.md §3).
"""
import numpy as np
import pytest

from oracle import oracle as O

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu


def _floats_bits_equal_nan_ok(a, b):
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _data(family, n, seed, scale_exp):
    rng = np.random.default_rng(seed)
    if family == "normal":
        x = O.splitmix_normal(seed, n)
    elif family == "refrand":
        x = O.c_ref_random_floats(seed % 100000 + 1, n)
    elif family == "ties":
        x = (rng.integers(-2000, 2000, n) + 0.5).astype(np.float32)
    elif family == "sparse":
        x = np.zeros(n, dtype=np.float32)
        idx = rng.integers(0, n, max(1, n // 50))
        x[idx] = rng.standard_normal(idx.size).astype(np.float32)
    else:  # "wide": magnitudes spread over ~2^60 inside a block
        x = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
    if family != "refrand":
        x = (x * np.float32(2.0 ** scale_exp)).astype(np.float32)
    return x


@settings(max_examples=300, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
@given(n=st.integers(1, 40_000), offset=st.integers(0, 7), P=st.sampled_from([64, 128, 256, 512, 1024]),
       W=st.sampled_from([1, 2, 3, 5, 8, 100, 65535]), scale_exp=st.integers(-60, 60),
       family=st.sampled_from(["normal", "refrand", "ties", "sparse", "wide"]), seed=st.integers(0, 2 ** 31))
def test_random_slices_bit_exact(cuda, n, offset, P, W, scale_exp, family, seed):
    import torch
    import switchml_amd as sw
    buf = _data(family, n + offset, seed, scale_exp)
    x = buf[offset:offset + n]
    xd = torch.from_numpy(buf).to(cuda)[offset:offset + n]
    B = O.num_blocks(n, P)

    payload, exps = sw.quantize_pack(xd, P, W)
    torch.cuda.synchronize()
    want_e = O.exponents(x, P)
    want_q = O.quantize(x, P, W)
    assert np.array_equal(exps.cpu().numpy(), want_e)
    assert np.array_equal(payload.cpu().numpy().view(np.uint32), want_q)

    # K2 alone, LE payload, RNE (VCL=1) mode
    assert np.array_equal(sw.exponents(xd, P).cpu().numpy(), want_e)
    le, _ = sw.quantize_pack(xd, P, W, flags=sw.FLAG_PAYLOAD_LE)
    assert np.array_equal(le.cpu().numpy().view(np.uint32), O.bswap32(want_q))
    rne, _ = sw.quantize_pack(xd, P, W, flags=sw.FLAG_ROUND_RNE)
    assert np.array_equal(rne.cpu().numpy().view(np.uint32), O.quantize(x, P, W, rounding=O.RNE_VCL))

    # K3 with global exponents that differ from the local ones (other workers' maxima)
    rng = np.random.default_rng(seed ^ 0x5A5A)
    ge = np.clip(want_e.astype(np.int32) + rng.integers(-2, 5, B), -128, 127).astype(np.int8)
    q3, _ = sw.quantize_pack(xd, P, W, global_exps=torch.from_numpy(ge).to(cuda))
    assert np.array_equal(q3.cpu().numpy().view(np.uint32), O.quantize(x, P, W, global_exps=ge))

    # K5 + K4 against the oracle, and the fused round trip against the same bits
    sw.loopback_aggregate(payload, W)
    out = sw.dequantize(payload, exps, n, P, W)
    rt = sw.roundtrip_loopback(xd, P, W)
    torch.cuda.synchronize()
    want_out = O.dequantize(O.loopback_aggregate(want_q, W), want_e, n, P, W)
    assert _floats_bits_equal_nan_ok(out.cpu().numpy(), want_out)
    assert _floats_bits_equal_nan_ok(rt.cpu().numpy(), want_out)
