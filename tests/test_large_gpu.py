"""Past 4 GiB: slices whose byte offsets exceed 2^32 (the largest configs
elsewhere stop at 1 GiB).  Every streaming kernel indexes with 64-bit
element and byte offsets; these cases would catch a 32-bit wrap anywhere on
the path.  Checked against the oracle on sampled blocks (first, last, around
the 2^32-byte boundary, random) — blocks are independent, so a block's
planes and output depend only on its own elements (ppp.cc:54-156,
197-260) — and through size-independent round-trip properties."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 5 * 2 ** 28 + 333           # 1 342 177 613 elements: 5 GiB of fp32, ragged last block
P, W = 256, 3


def _sample(B, rng):
    edge = (2 ** 30) // P          # element 2^30 = byte 2^32
    ks = {0, 1, 2, B - 3, B - 2, B - 1, edge - 2, edge - 1, edge, edge + 1, 2 * edge, 4 * edge + 7}
    ks |= set(int(k) for k in rng.integers(0, B, 200))
    return sorted(k for k in ks if 0 <= k < B)


def _x(torch, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(20240)
    return torch.randn(N, device=dev, generator=g) * 3.0


def test_planes_and_dequantize_past_4GiB(cuda):
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    x = _x(torch, dev)
    B = sw.num_blocks(N, P)
    payload, exps = sw.quantize_pack(x, P, W)          # K1: 5 GiB in, 5 GiB of planes out
    out = sw.dequantize(payload, exps, N, P, W)        # K4
    torch.cuda.synchronize()
    for k in _sample(B, np.random.default_rng(1)):
        lo, hi = k * P, min((k + 1) * P, N)
        xb = x[lo:hi].cpu().numpy()
        eb = O.exponents(xb, P)
        qb = O.quantize(xb, P, W)
        assert int(exps[k]) == int(eb[0]), k
        assert np.array_equal(payload[lo:lo + P].cpu().numpy().view(np.uint32), qb), k
        want = O.dequantize(qb, eb, hi - lo, P, W)
        assert np.array_equal(out[lo:hi].cpu().numpy().view(np.uint32), want.view(np.uint32)), k
    # K3 with global exponents (the switch's max of one worker = its own) and
    # K6 over two planes of the worker: the same bytes past 4 GiB
    p3, _ = sw.quantize_pack(x, P, W, global_exps=exps)
    assert torch.equal(p3, payload)
    del p3, out
    s_out = sw.switch_aggregate([payload, payload], [exps, exps], N, P, out=torch.empty_like(x))
    torch.cuda.synchronize()
    for k in _sample(B, np.random.default_rng(3))[::4]:
        lo, hi = k * P, min((k + 1) * P, N)
        xb = x[lo:hi].cpu().numpy()
        qb, eb = O.quantize(xb, P, W), O.exponents(xb, P)
        want = O.dequantize(O.switch_payload([qb, qb]), O.switch_exps([eb, eb]), hi - lo, P, 2)
        assert np.array_equal(s_out[lo:hi].cpu().numpy().view(np.uint32), want.view(np.uint32)), k
    del payload, exps, s_out
    rt = sw.roundtrip_loopback(x, P, W)                # fused round trip over the same 5 GiB
    torch.cuda.synchronize()
    for k in _sample(B, np.random.default_rng(2)):
        lo, hi = k * P, min((k + 1) * P, N)
        xb = x[lo:hi].cpu().numpy()
        want = O.dequantize(O.loopback_aggregate(O.quantize(xb, P, W), W), O.exponents(xb, P), hi - lo, P, W)
        assert np.array_equal(rt[lo:hi].cpu().numpy().view(np.uint32), want.view(np.uint32)), k


def test_frames_round_trip_past_4GiB(cuda):
    """DPDK frames of a 5 GiB slice (≈ 5.6 GB of frames): tx -> rx equals the
    fused loopback round trip, element for element."""
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    x = _x(torch, dev)
    fr = sw.quantize_pack_frames(x, sw.frame_params(job_id=9), packet_numel=P, num_workers=1, batch_max=64)
    F = fr.numel() // sw.frame_bytes(P)
    rx = sw.RxSlice(N, P, 64, device=dev)
    sw.dequantize_frames(fr, F, rx, num_workers=1, job_id=9)
    del fr
    ref = sw.roundtrip_loopback(x, P, 1)
    torch.cuda.synchronize()
    assert torch.equal(rx.out.view(torch.int32), ref.view(torch.int32))
    assert rx.counts.tolist() == [F, 0]


def test_int32_frames_round_trip_past_4GiB(cuda):
    """An INT32 slice of 5 GiB (≈ 5.3 GB of frames, pkt_ids past 2^20 and byte
    offsets past 2^32 on both sides): tx, then the one-pass rx over the frames
    in REVERSED order (every wave's stores far from the last one's), gives
    the words back; every frame accepted."""
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    xi = _x(torch, dev).view(torch.int32)
    fr = sw.pack_frames_int32(xi, sw.frame_params(job_id=5), packet_numel=P)
    fb = sw.frame_bytes(P)
    F = fr.numel() // fb
    fr = fr.view(F, fb).flip(0).contiguous().view(-1)
    rx = sw.RxSliceInt32(N, P, device=dev)
    rx.reset()
    sw.unpack_frames_int32(fr, F, rx, job_id=5)
    del fr
    torch.cuda.synchronize()
    assert rx.counts.tolist() == [F, 0]
    assert torch.equal(rx.out, xi)


def test_batch_kernel_past_4GiB(cuda):
    """The batched round trip with a slice table spanning > 4 GiB (FIFO
    slices of one 5 GiB job, T = 3): equal to the single-slice launches."""
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    x = _x(torch, dev)
    out = torch.empty_like(x)
    sl = []
    for t in range(3):
        q, r = divmod(N, 3)
        m = q + (t < r)
        off = t * m if t < r else t * m + r
        sl.append((off, m))
    sw.roundtrip_loopback_batch([(x[a:a + m], out[a:a + m]) for a, m in sl], P, W)
    ref = torch.empty_like(x)
    for a, m in sl:
        sw.roundtrip_loopback(x[a:a + m], P, W, out=ref[a:a + m])
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("mode", ["fused", "bulk"])
def test_client_allreduce_past_4GiB(cuda, mode):
    """Context::AllReduce of a 5 GiB device tensor, T = 4 FIFO slices (batched
    launch in fused mode, K1 -> K5 -> K4 per slice in bulk mode): equal to
    one fused round trip per FIFO slice."""
    import torch
    import switchml_amd as sw
    from switchml_amd import client as C
    dev = torch.device("cuda:0")
    T, Wc = 4, 2
    x = _x(torch, dev)
    out = torch.empty_like(x)
    C.start(C.make_config(num_workers=Wc, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                          mode=mode, bandwidth=0))
    try:
        C.allreduce(x, out)
    finally:
        C.stop()
    ref = torch.empty_like(x)
    for t in range(T):
        q, r = divmod(N, T)
        m = q + (t < r)
        off = t * m if t < r else t * m + r
        sw.roundtrip_loopback(x[off:off + m], P, Wc, out=ref[off:off + m])
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
