"""Full-size golden digests: SHA-256 of the
exponent plane, the BE payload plane and the loopback-dequantized output at
16 M and 64 M elements, committed in tests/golden/digests.json by
tests/golden/make_digests.py from the C oracle.

CPU: the oracle still produces the committed digests (fixture and oracle in
step).  GPU: the HIP path — K1 quantize+pack per FIFO slice, K5 loopback x W,
K4 dequantize, and the fused round trip — produces them too, with no oracle
on the GPU box.  Inputs come from integer-exact generators, so both hosts
hash the same bytes (the input digest is checked first)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "digests.json")) as _f:
    DIGESTS = json.load(_f)
with open(os.path.join(HERE, "golden", "digests_ext.json")) as _f:
    DIGESTS_EXT = json.load(_f)


def _gen():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_digests", os.path.join(HERE, "golden", "make_digests.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("name", sorted(DIGESTS))
def test_oracle_reproduces_digests(name):
    c = DIGESTS[name]
    got = _gen().oracle_digests(c["gen"], c["seed"], c["numel"], c["packet_numel"], c["num_workers"],
                                c["num_slices"])
    assert got == c["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(DIGESTS))
def test_hip_path_reproduces_digests(cuda, name):
    import torch
    import switchml_amd as sw
    m = _gen()
    c = DIGESTS[name]
    n, P, W, T = c["numel"], c["packet_numel"], c["num_workers"], c["num_slices"]
    x_host = m.make_input(c["gen"], c["seed"], n)
    assert hashlib.sha256(x_host.tobytes()).hexdigest() == c["sha256"]["input"], "input generator differs"
    x = torch.from_numpy(x_host).to(cuda)
    del x_host
    h = {k: hashlib.sha256() for k in ("exps", "payload", "out", "fused")}
    for t in range(T):
        off, ns = O.slice_geometry(n, T, t)
        if ns == 0:
            continue
        xs = x[off:off + ns]
        payload, exps = sw.quantize_pack(xs, P, W)
        torch.cuda.synchronize()
        h["exps"].update(exps.cpu().numpy().tobytes())
        h["payload"].update(payload.cpu().numpy().tobytes())
        sw.loopback_aggregate(payload, W)
        out = sw.dequantize(payload, exps, ns, P, W)
        fused = sw.roundtrip_loopback(xs, P, W)
        torch.cuda.synchronize()
        h["out"].update(m.canonical_nan(out.cpu().numpy()).tobytes())
        h["fused"].update(m.canonical_nan(fused.cpu().numpy()).tobytes())
        del payload, exps, out, fused
    want = c["sha256"]
    assert h["exps"].hexdigest() == want["exps"]
    assert h["payload"].hexdigest() == want["payload"]
    assert h["out"].hexdigest() == want["out"]
    assert h["fused"].hexdigest() == want["out"]


@pytest.mark.parametrize("name", sorted(DIGESTS_EXT))
def test_oracle_reproduces_ext_digests(name):
    c = DIGESTS_EXT[name]
    got = _gen().oracle_ext_digest(c["kind"], c["gen"], c["seed"], c["numel"], c["packet_numel"],
                                   c["num_workers"], c["extra"])
    assert got == c["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(DIGESTS_EXT))
def test_hip_path_reproduces_ext_digests(cuda, name):
    """Full-size DPDK frames (sml_quantize_pack_frames) and the VCL=1
    rounding mode (SML_FLAG_ROUND_RNE) against the oracle's digests."""
    import torch
    import switchml_amd as sw
    m = _gen()
    c = DIGESTS_EXT[name]
    n, P, W, ex = c["numel"], c["packet_numel"], c["num_workers"], c["extra"]
    x = torch.from_numpy(m.make_input(c["gen"], c["seed"], n)).to(cuda)
    if c["kind"] == "frames":
        out = sw.quantize_pack_frames(x, m.frame_params(ex), P, W, batch_max=ex["batch_max"])
    else:
        out, _ = sw.quantize_pack(x, P, W, flags=sw.FLAG_ROUND_RNE)
    torch.cuda.synchronize()
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == c["sha256"]
