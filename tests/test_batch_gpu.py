"""Batched dispatch: sml_roundtrip_loopback_batch (every slice of several
jobs in one launch) and the client's batch worker (backend.hip.batch_jobs,
mode = fused) — bit-exact against the per-slice kernel and the oracle's
packet loop (FIFO slices of T worker threads, fifo_scheduler.cc:93-109)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def fifo_slices(n, T):
    """(offset, numel) of the T FIFO slices of an n-element job."""
    out = []
    for t in range(T):
        q, r = divmod(n, T)
        m = q + (t < r)
        off = t * m if t < r else t * m + r
        out.append((off, m))
    return out


@pytest.mark.parametrize("P", [64, 128, 256, 512, 1024])
@pytest.mark.parametrize("W", [1, 3, 8])
def test_batch_kernel_equals_per_slice(cuda, P, W):
    """Several jobs' FIFO slices (ragged, 4-byte-aligned starts, one empty
    slice, in place and not) in one launch == one sml_roundtrip_loopback per
    slice, bit for bit; and == the oracle's packet loop per job."""
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    sizes = [(100_003, 4), (1, 3), (257 * P + 5, 2), (5_000, 7), (0, 2)]
    xs = [torch.from_numpy(O.splitmix_normal(11 * i + P + W, n)).to(dev) for i, (n, _) in enumerate(sizes)]
    outs = [torch.full_like(x, float("nan")) for x in xs]
    ref = [torch.empty_like(x) for x in xs]
    batch = []
    for (n, T), x, o, r in zip(sizes, xs, outs, ref):
        for off, m in fifo_slices(n, T):
            batch.append((x[off:off + m], o[off:off + m]))
            if m:
                sw.roundtrip_loopback(x[off:off + m], P, W, out=r[off:off + m])
    assert len(batch) <= sw.MAX_BATCH_SLICES
    sw.roundtrip_loopback_batch(batch, P, W)
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o.view(torch.int32), r.view(torch.int32))
    for (n, T), x, o in zip(sizes, xs, outs):
        if n:
            want = O.dummy_allreduce(x.cpu().numpy(), P=P, num_worker_threads=T, num_workers=W,
                                     max_outstanding_packets=64 * T)
            assert bits_equal(o.cpu().numpy(), want)


def test_batch_kernel_in_place_rne_pinned_and_max_slices(cuda):
    import torch
    import switchml_amd as sw
    P, W = 256, 2
    dev = torch.device("cuda:0")
    n, T = 64 * 1000 + 13, sw.MAX_BATCH_SLICES
    x = torch.from_numpy(O.splitmix_normal(3, n)).to(dev)
    y = x.clone()
    ref = torch.empty_like(x)
    sl = fifo_slices(n, T)
    for off, m in sl:
        sw.roundtrip_loopback(x[off:off + m], P, W, out=ref[off:off + m], flags=sw.FLAG_ROUND_RNE)
    sw.roundtrip_loopback_batch([(y[off:off + m], y[off:off + m]) for off, m in sl], P, W, flags=sw.FLAG_ROUND_RNE)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int32), ref.view(torch.int32))
    # pinned host slices (zero-copy over PCIe)
    hx = x.cpu().pin_memory()
    ho = torch.empty_like(hx).pin_memory()
    sw.roundtrip_loopback_batch([(hx[off:off + m], ho[off:off + m]) for off, m in fifo_slices(n, 4)], P, W)
    torch.cuda.synchronize()
    want = O.dummy_allreduce(hx.numpy(), P=P, num_worker_threads=4, num_workers=W, max_outstanding_packets=256)
    assert bits_equal(ho.numpy(), want)
    with pytest.raises(RuntimeError):
        sw.roundtrip_loopback_batch([(x[:10], ref[:10])] * (sw.MAX_BATCH_SLICES + 1), P, W)


@pytest.fixture
def C(cuda):
    from switchml_amd import client
    yield client
    if client.state() == client.RUNNING:
        client.stop()


@pytest.mark.parametrize("batch_jobs", [16, 1, 0])
@pytest.mark.parametrize("T,W,P", [(4, 8, 256), (3, 2, 64), (1, 3, 1024)])
def test_client_batch_mode_many_jobs(C, batch_jobs, T, W, P):
    """Many async jobs through the batch worker (and the threaded path,
    batch_jobs = 0): distinct device buckets, an in-place job issued twice on
    the same buffer (the second must see the first's result: buffers that
    overlap an earlier job of the batch start a new launch), INT32 and
    pageable-host jobs mixed in; every result bit-exact vs the oracle."""
    import torch
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                          mode="fused", bandwidth=0, batch_jobs=batch_jobs))
    sizes = [6_553_600 // 64, 777, 100_003, 1, 40_000]
    xs = [O.splitmix_normal(i + 100 * T, n) for i, n in enumerate(sizes)]
    dx = [torch.from_numpy(x).cuda() for x in xs]
    do = [torch.empty_like(d) for d in dx]
    inplace = torch.from_numpy(xs[2].copy()).cuda()
    xi = np.random.default_rng(T).integers(-2 ** 31, 2 ** 31, 9_999, dtype=np.int64).astype(np.int32)
    oi = np.empty_like(xi)
    hp = O.splitmix_normal(77, 12_345)          # pageable host (staged)
    hpo = np.empty_like(hp)
    jobs = [C.allreduce_async(d, o) for d, o in zip(dx, do)]
    jobs.append(C.allreduce_async(inplace))
    jobs.append(C.allreduce_async(xi, oi))
    jobs.append(C.allreduce_async(inplace))
    jobs.append(C.allreduce_async(hp, hpo))
    C.wait_for_all_jobs()
    assert all(j.status() == C.JOB_FINISHED for j in jobs)

    def ref(x):
        return O.dummy_allreduce(x, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W)
    for x, o in zip(xs, do):
        assert bits_equal(o.cpu().numpy(), ref(x))
    assert bits_equal(inplace.cpu().numpy(), ref(ref(xs[2])))
    assert np.array_equal(oi, (xi.astype(np.int64) * W).astype(np.int32))
    assert bits_equal(hpo, ref(hp))
    C.stop()


def test_client_batch_mode_fault_and_stop(C):
    """The batch worker keeps the threaded path's failure semantics: a slice
    of the injected failing worker thread fails its job (published only
    after the job's other slices ran), and Stop with jobs queued fails them
    without hanging."""
    import torch
    C.start(C.make_config(num_workers=2, num_worker_threads=4, packet_numel=256, mode="fused", bandwidth=0,
                          batch_jobs=16, fail_worker_thread=2))
    x = torch.randn(100_000, device="cuda")
    o = torch.empty_like(x)
    j = C.allreduce_async(x, o)
    with pytest.raises(C.ContextError):
        j.wait()
    assert j.status() == C.JOB_FAILED
    j2 = C.allreduce_async(x[:1000], o[:1000])
    with pytest.raises(C.ContextError):    # slice 2 of 4 fails here too
        j2.wait()
    C.stop()
    C.start(C.make_config(num_workers=2, num_worker_threads=4, packet_numel=256, mode="fused", bandwidth=0,
                          batch_jobs=16))
    big = torch.randn(16 * 2 ** 20, device="cuda")
    jobs = [C.allreduce_async(big) for _ in range(40)]
    C.stop()
    assert all(j.status() in (C.JOB_FINISHED, C.JOB_FAILED) for j in jobs)


def test_batch_kernel_random_slice_tables(cuda):
    """Hypothesis (derandomized): random batches — 1-8 jobs of 0-40 000
    elements at random element offsets of one buffer (any 4-byte
    alignment), T = 1-8 FIFO slices each, P, W, RNE — one batched launch ==
    one sml_roundtrip_loopback per slice, bit for bit."""
    pytest.importorskip("hypothesis")
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import torch
    import switchml_amd as sw
    dev = torch.device("cuda:0")
    pool = torch.from_numpy(O.splitmix_normal(99, 400_000)).to(dev)

    @settings(max_examples=60, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(jobs=st.lists(st.tuples(st.integers(0, 40_000), st.integers(1, 8)), min_size=1, max_size=8),
           P=st.sampled_from([64, 128, 256, 512, 1024]), W=st.sampled_from([1, 2, 3, 8, 255]),
           rne=st.booleans(), seed=st.integers(0, 2 ** 31))
    def check(jobs, P, W, rne, seed):
        rng = np.random.default_rng(seed)
        flags = sw.FLAG_ROUND_RNE if rne else 0
        out = torch.full_like(pool, float("nan"))
        ref = torch.full_like(pool, float("nan"))
        batch, pos = [], 0
        for n, T in jobs:
            pos += int(rng.integers(0, 9))              # gaps: any element offset
            if pos + n > pool.numel():
                break
            for off, m in fifo_slices(n, T):
                if len(batch) == sw.MAX_BATCH_SLICES:
                    break
                a = pos + off
                batch.append((pool[a:a + m], out[a:a + m]))
                if m:
                    sw.roundtrip_loopback(pool[a:a + m], P, W, out=ref[a:a + m], flags=flags)
            pos += n
        sw.roundtrip_loopback_batch(batch, P, W, flags=flags)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))

    check()
