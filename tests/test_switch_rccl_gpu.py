"""configs[3]'s switch data path through RCCL (torch.distributed backend
"nccl"), on one MI355X: W ranks share cuda:0, each an RCCL host of its own
(NCCL_HOSTID; switchml_amd.rccl_collnet.same_gpu_rccl_env), so the exchange
steps run in RCCL's own ring kernels — ncclInt8 MAX on the exponent plane,
wrapping ncclInt32 SUM on the payload plane — exactly the calls the driver's
N-GPU run makes, instead of gloo's host reductions.

Reference semantics: the switch keeps, per slot, the signed int<8> max of the
workers' exponents (p4/exponents.p4:48-54, types.p4:119) and the bit<32>
wrapping sum of their payload words (p4/processor.p4:48-54).

* `wrap_case` builds buckets whose quantized sum crosses 2^31 in hundreds of
  slots (both signs) and whose exponents are negative, with blocks where the
  signed max differs from an unsigned one; a CPU test proves that of the
  construction with the oracle, so the GPU test cannot pass vacuously;
* SwitchSimAllReduce (K2 -> RCCL int8 MAX -> K3 -> RCCL int32 SUM -> K4) and
  PeerSwitchAllReduce (K2 -> RCCL int8 MAX -> K3 -> K6 -> RCCL all_gather)
  are bit-exact against the oracle's lockstep switch on it, FLOAT32 and INT32;
* the W = 8 full-size case reproduces tests/golden/digests_switch.json.
"""
import hashlib
import os
import uuid

import numpy as np
import pytest

from oracle import oracle as O
from mp_ranks import init_pg, spawn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HUGE = np.float32(1.5 * 2.0 ** 127)     # exponent field 254 -> e = 128 -> int8 -128 (ppp.cc:148-156)


def wrap_case(rank: int, world: int, n: int, P: int, e_wrap: int = -60) -> np.ndarray:
    """Worker `rank`'s FLOAT32 bucket.  Random blocks: N(0,1) x 2^k, k drawn
    per block and per worker from [-60, 20] (negative exponents, and blocks
    where one worker's exponent is negative and another's positive).  Then:
      block 0: worker 0 holds HUGE (its exponent wraps to int8 -128, below
               everyone's e_wrap) and values in [0.9, 0.99] x W x 2^e_wrap,
               which quantize to ~0.9-0.99 x 2^31 with the global exponent
               e_wrap; the others hold [0.5, 0.99) x 2^e_wrap (~2^31 / W
               each): the slot sums cross +2^31 and wrap;
      block 1: the mirror image, negative, HUGE at the last worker: wrap
               below -2^31;
      block 2: every worker ~2^-105: scale(W, e) = +inf, payload 0
               (the x86 conversion of inf, ppp.cc:101-109)."""
    assert n >= 3 * P
    rng = np.random.default_rng(500 + rank)
    B = -(-n // P)
    k = rng.integers(-60, 21, B)
    x = (rng.standard_normal(B * P) * np.repeat(np.exp2(k.astype(np.float64)), P))[:n]
    u = 2.0 ** e_wrap
    for blk, sign, holder in ((0, 1.0, 0), (1, -1.0, world - 1)):
        s = slice(blk * P, (blk + 1) * P)
        if rank == holder:
            x[s] = sign * rng.uniform(0.9, 0.99, P) * world * u
            x[blk * P + 7] = sign * HUGE
        else:
            x[s] = sign * rng.uniform(0.5, 0.99, P) * u
    x[2 * P:3 * P] = rng.standard_normal(P) * 2.0 ** -105
    return x.astype(np.float32)


def int32_wrap_case(rank: int, n: int) -> np.ndarray:
    """INT32 bucket near the ends of the int32 range: sums wrap both ways."""
    rng = np.random.default_rng(900 + rank)
    v = rng.integers(2 ** 30, 2 ** 31, n, dtype=np.int64)
    v[rng.random(n) < 0.5] *= -1
    return v.clip(-2 ** 31, 2 ** 31 - 1).astype(np.int32)


def oracle_switch(xs, P):
    """(global exps, aggregated BE payload, dequantized sum) of the lockstep
    W-worker switch (oracle/sml_oracle.c)."""
    W, n = len(xs), xs[0].size
    g = O.switch_exps([O.exponents(x, P) for x in xs])
    agg = O.switch_payload([O.quantize(x, P, W, global_exps=g) for x in xs])
    return g, agg, O.dequantize(agg, g, n, P, W)


@pytest.mark.parametrize("world,P", [(2, 256), (3, 64), (8, 256)])
def test_wrap_case_wraps_and_needs_signed_max(world, P):
    """The construction does what the GPU test relies on (oracle only)."""
    n = 64 * P + 13
    xs = [wrap_case(r, world, n, P) for r in range(world)]
    g = O.switch_exps([O.exponents(x, P) for x in xs])
    qs = [O.bswap32(O.quantize(x, P, world, global_exps=g)).view(np.int32).astype(np.int64) for x in xs]
    s = np.sum(np.stack(qs), axis=0)
    assert np.sum(s > 2 ** 31 - 1) >= P // 2 and np.sum(s < -2 ** 31) >= P // 2
    unsigned = np.max(np.stack([O.exponents(x, P).view(np.uint8) for x in xs]), axis=0).view(np.int8)
    assert np.sum(unsigned != g) > 0                      # an unsigned max would differ
    assert g[0] == -60 and g[1] == -60 and (g[3:] < 0).any() and (g[3:] > 0).any()
    _, agg, out = oracle_switch(xs, P)
    assert np.all(out[2 * P:3 * P] == 0)                  # scale +inf: payload 0
    assert np.all(out[:P][np.arange(P) != 7] < 0)         # the wrapped positive sums come back negative


def _rank(rank, world, init, session, net, n, P, digest_name):
    from switchml_amd.rccl_collnet import same_gpu_rccl_env
    os.environ.update(same_gpu_rccl_env(rank, session, net))
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    init_pg("nccl", init, rank, world, device_id=dev)
    import switchml_amd as sw
    from switchml_amd.p2pswitch import PeerSwitchAllReduce
    from switchml_amd.switchsim import SwitchSimAllReduce
    res = {"backend": dist.get_backend()}

    def u32(t):
        return t.cpu().numpy().view(np.uint32)

    if digest_name is None:
        xs = [wrap_case(r, world, n, P) for r in range(world)]
        g, agg, ref = oracle_switch(xs, P)
        x = torch.from_numpy(xs[rank]).to(dev)
        ss = SwitchSimAllReduce(n, P, dev)
        out = ss(x)
        torch.cuda.synchronize()
        res["ss_exps"] = bool(np.array_equal(ss.exps.cpu().numpy(), g))
        res["ss_payload"] = bool(np.array_equal(u32(sw.bswap_i32(ss.payload)), agg))
        res["ss_out"] = bool(np.array_equal(u32(out), ref.view(np.uint32)))
        ar = PeerSwitchAllReduce(n, P, dev)
        res["p2p_out"] = True
        for _ in range(2):    # planes and peer mappings reused across calls
            res["p2p_out"] &= bool(np.array_equal(u32(ar(x)), ref.view(np.uint32)))
        res["p2p_exps"] = bool(np.array_equal(ar.exps.cpu().numpy(), g))
        ar.close()
        # INT32 buckets: htonl, the switch's wrapping sum, ntohl (ppp.cc:158-190, 262-298)
        xi = [int32_wrap_case(r, n) for r in range(world)]
        refi = O.bswap32(O.switch_payload([O.bswap32(v) for v in xi]))
        ti = torch.from_numpy(xi[rank]).to(dev)
        res["ss_int32"] = bool(np.array_equal(u32(SwitchSimAllReduce(n, P, dev)(ti)), refi))
        ar = PeerSwitchAllReduce(n, P, dev)
        res["p2p_int32"] = bool(np.array_equal(u32(ar(ti)), refi))
        ar.close()
    else:
        import importlib.util
        import json
        gd = os.path.join(ROOT, "tests", "golden")
        spec = importlib.util.spec_from_file_location("make_digests", os.path.join(gd, "make_digests.py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        with open(os.path.join(gd, "digests_switch.json")) as f:
            c = json.load(f)[digest_name]
        x = torch.from_numpy(m.switch_input(c["gen"], c["seed"], rank, n)).to(dev)
        want = c["sha256"]

        def sha(a):
            return hashlib.sha256(a.tobytes()).hexdigest()

        ss = SwitchSimAllReduce(n, P, dev)
        out = ss(x)
        torch.cuda.synchronize()
        res["ss_exps"] = sha(ss.exps.cpu().numpy()) == want["global_exps"]
        res["ss_payload"] = sha(sw.bswap_i32(ss.payload).cpu().numpy()) == want["payload"]
        res["ss_out"] = sha(m.canonical_nan(out.cpu().numpy())) == want["out"]
        del ss, out
        ar = PeerSwitchAllReduce(n, P, dev)
        res["p2p_out"] = all(sha(m.canonical_nan(ar(x).cpu().numpy())) == want["out"] for _ in range(2))
        ar.close()
    return res


def _run(world, n, P, net, digest_name=None, timeout=300):
    res = spawn(_rank, world, (uuid.uuid4().hex[:8], net, n, P, digest_name), timeout=timeout,
                what=f"rccl switch W={world} {net}")
    for rank, r, err in res:
        assert r is not None, (rank, err)
        assert r.pop("backend") == "nccl"
        assert all(r.values()), (rank, r)


@pytest.mark.gpu
@pytest.mark.parametrize("net", ["switchml", "socket"])
@pytest.mark.parametrize("world,n,P", [(2, 100_003, 256), (3, 4 * 1024 * 64 + 5, 64)])
def test_switch_paths_rccl_wrap_one_gpu(cuda, world, n, P, net):
    """Both switch paths under RCCL, on buckets whose slot sums wrap past
    +-2^31 and whose exponents are negative and need the SIGNED max:
    global exponents, aggregated wire words and dequantized sums bit-exact
    against the oracle switch; INT32 buckets likewise."""
    _run(world, n, P, net)


@pytest.mark.gpu
def test_switch_w8_rccl_reproduces_digests(cuda):
    """configs[3]'s W = 8 switch simulation with RCCL doing the exchange (8
    ranks on cuda:0, one RCCL host each): every worker's global exponents,
    aggregated payload and dequantized sum hash to digests_switch.json."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "digests_switch.json")) as f:
        name, c = sorted(json.load(f).items())[0]
    _run(c["num_workers"], c["numel"], c["packet_numel"], "switchml", digest_name=name, timeout=600)
