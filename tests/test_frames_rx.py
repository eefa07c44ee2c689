"""Receive side of the DPDK backend (the inverse direction):
DpdkWorkerThread's receive loop + PostprocessSingle over the frames the
switch returns (client_lib/src/backends/dpdk/dpdk_worker_thread.cc:300-345,
ppp.cc:197-260).

The "switch" here is the dummy backend's (dummy_backend.cc:72-84): every BE
payload word x W, the exponent byte unchanged.  Streams are built the way a
real rx ring sees them: frames reordered within windows of b packets (the
switch returns a window's packets in any order, but packet p + b is only sent
after packet p came back — so exponent k always precedes payload k),
duplicates of already received packets (a retransmission answered twice; the
later copy carries garbage and must be discarded), frames of another job
and an out-of-range pkt_id.

CPU tests pin the oracle's receive loop (oracle/sml_oracle.c:
orc_dequantize_frames) to the plane-level oracle; GPU tests compare
sml_dequantize_frames with it bit for bit.
"""
import numpy as np
import pytest

from oracle import oracle as O


def _params(job_id):
    import switchml_amd as sw
    return sw.frame_params(job_id=job_id, pool_index_start=0, pool_index_shift=0, max_outstanding_pkts=64)


def switch_return(sent, stride, P, W):
    """DummyBackend::ProcessPacket on every frame: BE payload words x W (wrap)."""
    f = sent.reshape(-1, stride).copy()
    pl = f[:, 52:52 + 4 * P].copy().view(">u4").astype(np.uint64)
    f[:, 52:52 + 4 * P] = ((pl * W) & 0xFFFFFFFF).astype(">u4").view(np.uint8)
    return f


def rx_stream(x, P, W, batch_max, job_id, seed, n_dups=3, n_wrong=2, bad_pid=True, shuffle=True):
    """(frames [F, stride] uint8 in rx order, number of frames that must be discarded).
    shuffle=False keeps the switch's return order (frame f carries pkt_id f)
    before the anomalies are inserted."""
    stride = 52 + 4 * P
    sent = O.build_frames(x, _params(job_id), P=P, num_workers=W, batch_max=batch_max)
    ret = switch_return(sent, stride, P, W)
    B = O.num_blocks(x.size, P)
    b = min(B, batch_max)
    rng = np.random.default_rng(seed)
    order = []
    for w0 in range(0, B + b, b):
        win = list(range(w0, min(w0 + b, B + b)))
        if shuffle:
            rng.shuffle(win)
        order += win
    rows = [ret[i] for i in order]
    discard = 0
    for _ in range(n_dups):                        # a later garbage copy of a received packet
        pos = int(rng.integers(0, len(rows)))
        dup = rows[pos].copy()
        dup[50] ^= 0x5A
        dup[52:] = rng.integers(0, 256, dup.size - 52, dtype=np.uint8)
        rows.insert(int(rng.integers(pos + 1, len(rows) + 1)), dup)
        discard += 1
    for _ in range(n_wrong):                       # another job's frame, anywhere
        src = rows[int(rng.integers(0, len(rows)))].copy()
        src[43] = (job_id + 1) & 0xFF
        src[52:] = 0xEE
        rows.insert(int(rng.integers(0, len(rows) + 1)), src)
        discard += 1
    if bad_pid:
        bad = rows[0].copy()
        bad[44:48] = np.frombuffer(np.uint32(B + b + 5).tobytes(), dtype=np.uint8)
        rows.insert(int(rng.integers(0, len(rows) + 1)), bad)
        discard += 1
    return np.stack(rows), discard


def expected_planes(x, P, W):
    """Plane-level oracle: quantize -> loopback x W -> dequantize."""
    q = O.quantize(x, P, W)
    e = O.exponents(x, P)
    return O.dequantize(O.loopback_aggregate(q, W), e, x.size, P, W), e


# ---------------------------------------------------------------- CPU --

@pytest.mark.parametrize("P,n,W,bm", [(256, 1, 1, 64), (256, 5000, 3, 4), (64, 777, 2, 8),
                                      (1024, 9000, 8, 2), (256, 256 * 20, 1, 64)])
def test_oracle_rx_loop_matches_planes(P, n, W, bm):
    x = O.splitmix_normal(100 + n, n)
    frames, disc = rx_stream(x, P, W, bm, job_id=7, seed=n)
    B = O.num_blocks(n, P)
    b = min(B, bm)
    rx = O.dequantize_frames(frames, frames.shape[0], frames.shape[1], O.RxState(n, P, bm), W, job_id=7)
    want, e = expected_planes(x, P, W)
    assert np.array_equal(rx.out.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(rx.exps, e)
    assert rx.counts == [B + b, disc]


def test_oracle_rx_loop_across_calls():
    """The rx bitmap and exponents persist across rx bursts of one slice."""
    P, n, W, bm = 256, 256 * 40 + 3, 2, 8
    x = O.splitmix_normal(5, n)
    frames, disc = rx_stream(x, P, W, bm, job_id=1, seed=9, n_dups=0, n_wrong=0, bad_pid=False)
    # a late duplicate of the very first frame, in the last burst
    frames = np.concatenate([frames, frames[:1]])
    cuts = [0, 13, 31, frames.shape[0]]
    rx = O.RxState(n, P, bm)
    for a, c in zip(cuts[:-1], cuts[1:]):
        O.dequantize_frames(frames[a:c], c - a, frames.shape[1], rx, W, job_id=1)
    want, _ = expected_planes(x, P, W)
    assert np.array_equal(rx.out.view(np.uint32), want.view(np.uint32))
    B = O.num_blocks(n, P)
    assert rx.counts == [B + min(B, bm), 1]


# ---------------------------------------------------------------- GPU --

def _run_gpu(torch, sw, frames, P, W, bm, job, n, where, calls=1):
    dev = torch.device("cuda:0")
    F, stride = frames.shape
    t = torch.from_numpy(frames.reshape(-1).copy())
    t = t.to(dev) if where == "device" else t.pin_memory()
    rx = sw.RxSlice(n, P, bm, device=dev)
    cuts = np.linspace(0, F, calls + 1).astype(int)
    for a, c in zip(cuts[:-1], cuts[1:]):
        sw.dequantize_frames(t[a * stride:c * stride], int(c - a), rx, num_workers=W, job_id=job, stride=stride)
    torch.cuda.synchronize()
    return rx.out.cpu().numpy(), rx.exps.cpu().numpy(), [int(v) for v in rx.counts.cpu()]


@pytest.mark.gpu
@pytest.mark.parametrize("P,n,W,bm", [(256, 1, 1, 64), (256, 5000, 3, 4), (64, 777, 2, 8), (128, 4099, 5, 16),
                                      (512, 3000, 4, 3), (1024, 9000, 8, 2), (256, 300_001, 7, 64)])
@pytest.mark.parametrize("where", ["device", "pinned"])
def test_rx_frames_match_oracle(cuda, P, n, W, bm, where):
    import torch
    import switchml_amd as sw
    x = O.splitmix_normal(200 + n, n)
    frames, _ = rx_stream(x, P, W, bm, job_id=0x3C, seed=n + P)
    ref = O.dequantize_frames(frames, frames.shape[0], frames.shape[1], O.RxState(n, P, bm), W, job_id=0x3C)
    out, exps, cnt = _run_gpu(torch, sw, frames, P, W, bm, 0x3C, n, where)
    assert np.array_equal(out.view(np.uint32), ref.out.view(np.uint32))
    assert np.array_equal(exps, ref.exps)
    assert cnt == ref.counts


@pytest.mark.gpu
@pytest.mark.parametrize("P,pad", [(256, 12), (64, 2048 - 52 - 4 * 64), (1024, 4)])
def test_rx_frames_padded_stride(cuda, P, pad):
    """Frames at an mbuf-like stride (frame bytes + padding, e.g. a 2 KiB data
    room): padding bytes are ignored, results equal the oracle's loop."""
    import torch
    import switchml_amd as sw
    n, W, bm = 40_000 + P // 3, 3, 16
    x = O.splitmix_normal(31 + P, n)
    frames, _ = rx_stream(x, P, W, bm, job_id=7, seed=P)
    F, fb = frames.shape
    padded = np.full((F, fb + pad), 0xCD, dtype=np.uint8)
    padded[:, :fb] = frames
    ref = O.dequantize_frames(frames, F, fb, O.RxState(n, P, bm), W, job_id=7)
    out, exps, cnt = _run_gpu(torch, sw, padded, P, W, bm, 7, n, "device")
    assert np.array_equal(out.view(np.uint32), ref.out.view(np.uint32))
    assert np.array_equal(exps, ref.exps)
    assert cnt == ref.counts


@pytest.mark.gpu
def test_rx_frames_across_calls(cuda):
    import torch
    import switchml_amd as sw
    P, n, W, bm = 256, 256 * 300 + 17, 3, 16
    x = O.splitmix_normal(77, n)
    frames, _ = rx_stream(x, P, W, bm, job_id=9, seed=3)
    frames = np.concatenate([frames, frames[5:9]])           # late duplicates in the last burst
    ref = O.RxState(n, P, bm)
    cuts = np.linspace(0, frames.shape[0], 5).astype(int)
    for a, c in zip(cuts[:-1], cuts[1:]):
        O.dequantize_frames(frames[a:c], int(c - a), frames.shape[1], ref, W, job_id=9)
    out, exps, gcnt = _run_gpu(torch, sw, frames, P, W, bm, 9, n, "device", calls=4)
    assert np.array_equal(out.view(np.uint32), ref.out.view(np.uint32))
    assert np.array_equal(exps, ref.exps)
    assert gcnt == ref.counts and ref.counts[1] >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("W", [1, 6])
def test_frames_tx_rx_round_trip_equals_fused_loopback(cuda, W):
    """Size-independent property at a large size: quantize into frames ->
    switch (x W on the wire words) -> dequantize from frames gives exactly the
    fused loopback round trip (sml_roundtrip_loopback)."""
    import torch
    import switchml_amd as sw
    P, bm = 256, 64
    n = 16 * 2 ** 20 + 333
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(W)
    x = torch.randn(n, device=dev, generator=g)
    stride = sw.frame_bytes(P)
    fr = sw.quantize_pack_frames(x, sw.frame_params(job_id=4), packet_numel=P, num_workers=W, batch_max=bm)
    F = fr.numel() // stride
    v = fr.view(F, stride)[:, 52:52 + 4 * P].contiguous().view(torch.int32)
    v = (v.view(torch.uint8).view(F, P, 4).flip(-1).contiguous().view(torch.int32) * W)   # ntohl, x W (wraps)
    v = v.view(torch.uint8).view(F, P, 4).flip(-1).contiguous().view(F, 4 * P)           # htonl
    fr.view(F, stride)[:, 52:52 + 4 * P] = v
    ref = sw.roundtrip_loopback(x, P, W)
    # both output store policies of the apply pass (non-temporal from the
    # threshold on — 0 here — or default): the same bytes
    orig = sw.set_payload_nt_threshold(0)
    try:
        for thr in (0, 2 ** 64 - 1):
            sw.set_payload_nt_threshold(thr)
            rx = sw.RxSlice(n, P, bm, device=dev)
            sw.dequantize_frames(fr, F, rx, num_workers=W, job_id=4)
            torch.cuda.synchronize()
            assert torch.equal(rx.out.view(torch.int32), ref.view(torch.int32)), thr
            assert rx.counts.tolist() == [F, 0]
    finally:
        sw.set_payload_nt_threshold(orig)


# ------------------------------------------------------ randomized (GPU) --

@pytest.mark.gpu
def test_rx_frames_random_streams(cuda):
    """Hypothesis (derandomized): random slice length, P, W, batch size, job id,
    duplicate / wrong-job / bad-pkt_id counts, shuffle seed and number of rx
    calls; the GPU receive path equals the oracle's sequential loop (output,
    exponents and accepted/discarded counters)."""
    hyp = pytest.importorskip("hypothesis")
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import torch
    import switchml_amd as sw

    @settings(max_examples=80, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(n=st.integers(1, 20_000), P=st.sampled_from([64, 128, 256, 512, 1024]), W=st.sampled_from([1, 2, 3, 8]),
           bm=st.integers(1, 70), job=st.integers(0, 255), dups=st.integers(0, 6), wrong=st.integers(0, 4),
           bad=st.booleans(), seed=st.integers(0, 2 ** 31), calls=st.integers(1, 4))
    def check(n, P, W, bm, job, dups, wrong, bad, seed, calls):
        x = O.splitmix_normal(seed, n)
        frames, _ = rx_stream(x, P, W, bm, job_id=job, seed=seed, n_dups=dups, n_wrong=wrong, bad_pid=bad)
        F = frames.shape[0]
        calls = min(calls, F)
        ref = O.RxState(n, P, bm)
        cuts = np.linspace(0, F, calls + 1).astype(int)
        for a, c in zip(cuts[:-1], cuts[1:]):
            O.dequantize_frames(frames[a:c], int(c - a), frames.shape[1], ref, W, job_id=job)
        out, exps, cnt = _run_gpu(torch, sw, frames, P, W, bm, job, n, "device", calls=calls)
        assert np.array_equal(out.view(np.uint32), ref.out.view(np.uint32))
        assert np.array_equal(exps, ref.exps)
        assert cnt == ref.counts

    check()


# ------------------------------------------------------ in-order streams --
# The switch's return order (frame f carries pkt_id p0 + f), split into rx
# bursts, with and without one anomaly deep inside a later burst: the common
# case of the receive loop, and the edge cases an in-order fast path would
# have to get right (one was tried and measured slower).

def _in_order_case(torch, sw, n, P, W, bm, job, cuts, edit=None, where="device"):
    x = O.splitmix_normal(n + 7 * P + W, n)
    frames, _ = rx_stream(x, P, W, bm, job_id=job, seed=n, n_dups=0, n_wrong=0, bad_pid=False, shuffle=False)
    if edit is not None:
        frames = edit(frames)
    F = frames.shape[0]
    cuts = [0] + [c for c in cuts if 0 < c < F] + [F]
    ref = O.RxState(n, P, bm)
    for a, c in zip(cuts[:-1], cuts[1:]):
        O.dequantize_frames(frames[a:c], int(c - a), frames.shape[1], ref, W, job_id=job)
    dev = torch.device("cuda:0")
    stride = frames.shape[1]
    t = torch.from_numpy(frames.reshape(-1).copy())
    t = t.to(dev) if where == "device" else t.pin_memory()
    rx = sw.RxSlice(n, P, bm, device=dev)
    for a, c in zip(cuts[:-1], cuts[1:]):
        sw.dequantize_frames(t[a * stride:c * stride], int(c - a), rx, num_workers=W, job_id=job, stride=stride)
    torch.cuda.synchronize()
    assert np.array_equal(rx.out.cpu().numpy().view(np.uint32), ref.out.view(np.uint32))
    assert np.array_equal(rx.exps.cpu().numpy(), ref.exps)
    assert [int(v) for v in rx.counts.cpu()] == ref.counts
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("P", [64, 128, 256, 512, 1024])
@pytest.mark.parametrize("where", ["device", "pinned"])
def test_rx_in_order_bursts(cuda, P, where):
    """In-order bursts of one slice (p0 > 0 after the first), counters included."""
    import torch
    import switchml_amd as sw
    n = 200_000 + P + 3
    ref = _in_order_case(torch, sw, n, P, 3, 16, 0x21, cuts=[1, 40, 1000, 1001, 2500], where=where)
    assert ref.counts[1] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("P", [64, 256, 1024])
@pytest.mark.parametrize("kind", ["wrong_job", "dup_of_earlier_call", "swap", "bad_pid", "dup_in_call"])
def test_rx_in_order_then_miss(cuda, P, kind):
    """An in-order stream with one anomaly deep inside a later call: the
    result equals the oracle loop's."""
    import torch
    import switchml_amd as sw
    n, bm = 150_000 + 5, 8

    def edit(fr):
        fr = fr.copy()
        i = fr.shape[0] * 2 // 3
        if kind == "wrong_job":
            fr[i, 43] ^= 0x01
        elif kind == "dup_of_earlier_call":         # a copy of frame 3 (first call) inside the second call
            fr = np.concatenate([fr[:i], fr[3:4], fr[i:]])
        elif kind == "swap":
            fr[[i, i + 1]] = fr[[i + 1, i]]
        elif kind == "bad_pid":
            fr[i, 44:48] = np.frombuffer(np.uint32(0xFFFFFF00).tobytes(), dtype=np.uint8)
        else:                                     # garbage second copy of frame i, right after it
            d = fr[i].copy()
            d[52:] ^= 0xA5
            fr = np.concatenate([fr[:i + 1], d[None], fr[i + 1:]])
        return fr
    B = O.num_blocks(n, P)
    _in_order_case(torch, sw, n, P, 2, bm, 0x5A, cuts=[(B + bm) // 3], edit=edit)


@pytest.mark.gpu
def test_rx_in_order_random(cuda):
    """Hypothesis (derandomized): in-order streams split into random bursts,
    with 0-2 anomalies (swap, duplicate of an earlier frame, wrong job, bad
    pkt_id) at random places, vs the oracle loop."""
    pytest.importorskip("hypothesis")
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import torch
    import switchml_amd as sw

    @settings(max_examples=60, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(n=st.integers(1, 30_000), P=st.sampled_from([64, 128, 256, 512, 1024]), W=st.sampled_from([1, 2, 3, 8]),
           bm=st.integers(1, 70), job=st.integers(0, 255), calls=st.integers(1, 5), seed=st.integers(0, 2 ** 31),
           anomalies=st.lists(st.tuples(st.sampled_from(["swap", "dup", "job", "pid"]), st.floats(0, 1)),
                              max_size=2))
    def check(n, P, W, bm, job, calls, seed, anomalies):
        rng = np.random.default_rng(seed)

        def edit(fr):
            fr = fr.copy()
            for kind, at in anomalies:
                i = min(int(at * fr.shape[0]), fr.shape[0] - 1)
                if kind == "swap" and i + 1 < fr.shape[0]:
                    fr[[i, i + 1]] = fr[[i + 1, i]]
                elif kind == "dup":
                    j = int(rng.integers(0, i + 1))
                    fr = np.concatenate([fr[:i + 1], fr[j:j + 1], fr[i + 1:]])
                elif kind == "job":
                    fr[i, 43] ^= 0x80
                elif kind == "pid":
                    fr[i, 44:48] = np.frombuffer(np.uint32(int(rng.integers(0, 2 ** 32))).tobytes(), dtype=np.uint8)
            return fr
        B = O.num_blocks(n, P)
        F = B + min(B, bm)
        cuts = sorted(int(c) for c in rng.integers(1, F + 2, calls - 1)) if calls > 1 else []
        _in_order_case(torch, sw, n, P, W, bm, job, cuts=cuts, edit=edit)

    check()
