"""Randomized client-level parity (Hypothesis, derandomized): the whole
reference call path — Context::AllReduceAsync → FIFO slices → worker threads
→ HIP pre/post-processor → loopback "switch" → completion — against the
oracle's restatement of the dummy-backend packet loop (DummyWorkerThread +
CpuExponentQuantizerPPP, dummy_worker_thread.cc:86-177, ppp.cc:54-306).

Each example draws the worker-thread count T, W, P, the backend mode, the
job count and sizes (ragged, including sizes below T and below one packet),
where the tensors live (device / pinned host / pageable host), in place or
not, FLOAT32 or INT32; all jobs are submitted asynchronously before any is
waited for (the worker threads overlap jobs), then every output is checked
bit for bit.  Also: Stop() with jobs in flight leaves every job FINISHED or
FAILED and nothing running."""
import numpy as np
import pytest

from oracle import oracle as O

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture
def C(cuda):
    from switchml_amd import client
    yield client
    if client.state() == client.RUNNING:
        client.stop()


def _bits(a):
    return np.asarray(a).view(np.uint32)


def _place(torch, arr, where):
    t = torch.from_numpy(arr.copy())
    if where == "device":
        return t.cuda()
    if where == "pinned":
        return t.pin_memory()
    return t   # pageable


def _host(torch, t):
    return t.cpu().numpy() if t.is_cuda else t.numpy()


@settings(max_examples=25, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(T=st.sampled_from([1, 2, 3, 4, 7]), W=st.sampled_from([1, 2, 3, 8]), P=st.sampled_from([64, 256, 1024]),
       mode=st.sampled_from(["bulk", "fused"]), where=st.sampled_from(["device", "pinned", "pageable"]),
       inplace=st.booleans(), int32=st.booleans(),
       sizes=st.lists(st.integers(min_value=0, max_value=70_000), min_size=1, max_size=5),
       seed=st.integers(min_value=1, max_value=10_000))
def test_client_random_jobs_match_oracle(C, T, W, P, mode, where, inplace, int32, sizes, seed):
    import torch
    mop = 64 * T
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=mop,
                          mode=mode, bandwidth=0))
    try:
        jobs, checks = [], []
        for i, n in enumerate(sizes):
            if int32:
                x = np.random.default_rng(seed + i).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
                ref = (x.astype(np.int64) * W).astype(np.int32)          # INT32 PPP: bswap, x W (wraps), bswap
            else:
                x = O.splitmix_normal(seed + i, n) * np.float32(2.0 ** ((seed + i) % 40 - 20))
                ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=mop, num_worker_threads=T, num_workers=W)
            xin = _place(torch, x, where)
            xout = xin if inplace else _place(torch, np.zeros_like(x), where)
            jobs.append(C.allreduce_async(xin, xout, numel=n))
            checks.append((x, xin, xout, ref))
        C.wait_for_all_jobs()
        assert all(j.status() == C.JOB_FINISHED for j in jobs)
        torch.cuda.synchronize()
        for x, xin, xout, ref in checks:
            assert np.array_equal(_bits(_host(torch, xout)), _bits(ref))
            if not inplace:
                assert np.array_equal(_bits(_host(torch, xin)), _bits(x))    # input untouched
    finally:
        C.stop()


def test_stop_with_jobs_in_flight(C):
    """Stop() while device jobs are queued and running: every job ends
    FINISHED or FAILED, Stop returns after the worker threads (and their
    in-flight kernels) are done, and the context can be started again."""
    import torch
    T, n = 4, 16 * 1024 * 1024
    C.start(C.make_config(num_workers=2, num_worker_threads=T, packet_numel=256, mode="bulk", bandwidth=0))
    bufs = [torch.randn(n, device="cuda") for _ in range(6)]
    jobs = [C.allreduce_async(b) for b in bufs]
    C.stop()
    states = [j.status() for j in jobs]
    assert all(s in (C.JOB_FINISHED, C.JOB_FAILED) for s in states), states
    torch.cuda.synchronize()
    del bufs
    C.start(C.make_config(num_workers=2, num_worker_threads=T, packet_numel=256, mode="fused", bandwidth=0))
    x = O.splitmix_normal(3, 10_007)
    out = np.empty_like(x)
    C.allreduce(x, out)
    ref = O.dummy_allreduce(x, P=256, max_outstanding_packets=256, num_worker_threads=T, num_workers=2)
    assert np.array_equal(_bits(out), _bits(ref))
    C.stop()
