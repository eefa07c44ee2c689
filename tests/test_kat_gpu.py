"""The hand-derived known-answer vectors (tests/golden/kat_vectors.json, made
by tests/golden/make_kat.py with exact rational arithmetic from a reading of
ppp.cc) through the HIP path on the GPU: K1 (fused exponent + quantize + BE
pack), K2 (exponents only), K3 (quantize with given global exponents), K5
loopback x W + K4 dequantize, and the fused round trip.  The same vectors pin
the C and numpy oracles on the CPU (tests/test_oracle.py::test_kat_*), so
this is the third implementation held to them.

Cases cover: ties (half away from zero), all-zero blocks, the e = -96 / -97
boundary where the scale becomes +inf, denormals, NaN skipped by the max,
+-inf, e = 128 wrapping to int8 -128, W * 2^e overflowing float (scale 0,
0/0 NaN), W = 3 / 65535, partial blocks, global exponents below the local
one (the x86 wrap path, ppp.cc:103)."""
import numpy as np
import pytest

from test_oracle import kat_arrays, load_kats, out_matches


@pytest.mark.gpu
@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_kat_hip_path(cuda, case):
    import torch
    import switchml_amd as sw
    x, payload, exps, ge = kat_arrays(case)
    P, W, n = case["P"], case["W"], x.size
    xd = torch.from_numpy(x.copy()).to(cuda)

    # K2: exponents only
    e2 = sw.exponents(xd, P)
    # K1: fused exponent + quantize + BE pack (local exponents)
    p1, e1 = sw.quantize_pack(xd, P, W)
    torch.cuda.synchronize()
    assert np.array_equal(e2.cpu().numpy(), exps), "K2 exponent plane"
    assert np.array_equal(e1.cpu().numpy(), exps), "K1 exponent plane"
    e_use = exps if ge is None else ge
    if ge is None:
        assert np.array_equal(p1.cpu().numpy().view(np.uint32), payload), "K1 payload plane"

    # K3: quantize with given global exponents (the switch's max; here the
    # case's global exponents, or the local ones when it has none)
    g = torch.from_numpy(e_use.copy()).to(cuda)
    p3, _ = sw.quantize_pack(xd, P, W, global_exps=g)
    torch.cuda.synchronize()
    assert np.array_equal(p3.cpu().numpy().view(np.uint32), payload), "K3 payload plane"

    # K5 loopback x W, then K4 dequantize with the exponents the packets carried
    sw.loopback_aggregate(p3, W)
    out = sw.dequantize(p3, g, n, P, W)
    torch.cuda.synchronize()
    assert out_matches(out.cpu().numpy(), case["loopback_out_bits"]), "K5 + K4 output"

    # the fused round trip (quantize -> x W -> dequantize in one kernel) runs
    # with local exponents, like the dummy backend's packet loop
    if ge is None:
        rt = sw.roundtrip_loopback(xd, P, W)
        torch.cuda.synchronize()
        assert out_matches(rt.cpu().numpy(), case["loopback_out_bits"]), "fused round trip"
