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
from mp_ranks import spawn

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


with open(os.path.join(HERE, "golden", "digests_switch.json")) as _f:
    DIGESTS_SWITCH = json.load(_f)


@pytest.mark.parametrize("name", sorted(DIGESTS_SWITCH))
def test_oracle_reproduces_switch_digests(name):
    c = DIGESTS_SWITCH[name]
    got = _gen().oracle_switch_digests(c["gen"], c["seed"], c["numel"], c["packet_numel"], c["num_workers"])
    assert got == c["sha256"]


def _switch_rank(rank, world, init, name):
    """One worker of configs[3]'s switch simulation: its own 64 MiB bucket
    through SwitchSimAllReduce (K2 -> int8 MAX -> K3 -> int32 SUM -> K4) and
    PeerSwitchAllReduce (K2 -> int8 MAX -> K3 -> K6 over the peers' planes ->
    all_gather); digests of what this worker ends with."""
    from test_switchsim_dist import _init
    _init(rank, world, init)
    import torch
    import switchml_amd as sw
    from switchml_amd.p2pswitch import PeerSwitchAllReduce
    from switchml_amd.switchsim import SwitchSimAllReduce
    m = _gen()
    c = DIGESTS_SWITCH[name]
    n, P = c["numel"], c["packet_numel"]
    dev = torch.device("cuda:0")
    x = torch.from_numpy(m.switch_input(c["gen"], c["seed"], rank, n)).to(dev)
    ss = SwitchSimAllReduce(n, P, dev)
    out = ss(x)
    torch.cuda.synchronize()
    got = {"global_exps": hashlib.sha256(ss.exps.cpu().numpy().tobytes()).hexdigest(),
           # the exchange ran on host-order words; the switch's wire words are their byteswap
           "payload": hashlib.sha256(sw.bswap_i32(ss.payload).cpu().numpy().tobytes()).hexdigest(),
           "out": hashlib.sha256(m.canonical_nan(out.cpu().numpy()).tobytes()).hexdigest()}
    del ss, out
    ar = PeerSwitchAllReduce(n, P, dev)
    for i in range(2):   # planes and peer mappings reused across calls
        o2 = ar(x)
        torch.cuda.synchronize()
        got[f"p2p_out_{i}"] = hashlib.sha256(m.canonical_nan(o2.cpu().numpy()).tobytes()).hexdigest()
    ar.close()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(DIGESTS_SWITCH))
def test_switch_sim_w8_reproduces_digests(cuda, name):
    """configs[3]'s switch simulation at W = 8: eight worker processes (gloo,
    all on cuda:0 here; one GPU each on a node) with distinct 64 MiB buckets.
    Every worker's global exponents, aggregated BE payload and dequantized sum
    — through the RCCL-style ring switch and through the peer-to-peer switch
    — hash to the oracle's digests (p4/exponents.p4:48-54,
    p4/processor.p4:48-54, ppp.cc:194-251)."""
    c = DIGESTS_SWITCH[name]
    world = c["num_workers"]
    res = spawn(_switch_rank, world, (name,), timeout=300, what=f"switch W={world} {name}")
    want = c["sha256"]
    for rank, got, err in res:
        assert got is not None, (rank, err)
        assert got["global_exps"] == want["global_exps"], rank
        assert got["payload"] == want["payload"], rank
        assert got["out"] == want["out"], rank
        assert got["p2p_out_0"] == want["out"] and got["p2p_out_1"] == want["out"], rank
