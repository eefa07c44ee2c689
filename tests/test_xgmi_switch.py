"""The in-node switch backend (general.backend = "xgmi",
csrc/client/xgmi_switch.{h,cc}): W worker processes run the reference's
client API (Context::AllReduce via include/switchml_client.h, and the CollNet
plugin table) and reduce across each other through their planes' IPC
mappings — the Tofino switch's int8 exponent max and wrapping int32 sum
(p4/exponents.p4:48-54, p4/processor.p4:48-54), each FIFO slice
(fifo_scheduler.cc:93-109) exchanged on its own, then dequantized
(ppp.cc:194-251).  Checked bit for bit against the oracle's software switch
over the same W workers.  Here the W processes share cuda:0 (IPC inside one
device); on a node each worker has its own GPU and the mappings cross xGMI.

CPU: configuration validation of the backend."""
import os
import uuid

import numpy as np
import pytest
import torch

from oracle import oracle as O
from mp_ranks import spawn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def oracle_switch_allreduce(xs, P, T, rounding=O.HALF_AWAY):
    """W workers' buckets through the reference's switch, slice by slice
    (rounding = O.RNE_VCL: the reference's VCL=1 build)."""
    W, n = len(xs), xs[0].size
    out = np.empty(n, dtype=np.float32)
    for t in range(T):
        off, m = O.slice_geometry(n, T, t)
        if m == 0:
            continue
        parts = [x[off:off + m] for x in xs]
        g = O.switch_exps([O.exponents(p, P) for p in parts])
        agg = O.switch_payload([O.quantize(p, P, W, global_exps=g, rounding=rounding) for p in parts])
        out[off:off + m] = O.dequantize(agg, g, m, P, W)
    return out


def worker_bucket(rank, n, seed):
    return O.splitmix_normal(seed * 31 + rank, n) * np.float32(2.0 ** (rank % 3 - 1))


def _client_worker(rank, W, init, T, P, session, cap, push):
    from switchml_amd import client as C
    C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=T, packet_numel=P,
                          max_outstanding_packets=64 * T, mode="bulk", bandwidth=0, device=0,
                          session=session, max_slice_numel=cap, push=push))
    res = []
    sizes = [100_003, 1, 3 * cap + 517, 0, 4 * P * W + 5]
    for i, n in enumerate(sizes):
        where = ("device", "pageable", "pinned")[i % 3]
        xs = [worker_bucket(r, n, i) for r in range(W)]
        x = torch.from_numpy(xs[rank].copy())
        if where == "device":
            x = x.cuda()
        elif where == "pinned":
            x = x.pin_memory()
        inplace = i % 2 == 0
        out = x if inplace else torch.empty_like(x)
        C.allreduce(x, out)
        got = out.cpu().numpy() if out.is_cuda else out.numpy()
        ref = oracle_switch_allreduce(xs, P, T)
        res.append(bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32))))
    # INT32: the words' wrapping sum over the workers
    n = 50_021
    xi = [np.random.default_rng(5 + r).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
          for r in range(W)]
    t = torch.from_numpy(xi[rank].copy()).cuda()
    C.allreduce(t)
    ref = O.bswap32(O.switch_payload([O.bswap32(v) for v in xi]))
    res.append(bool(np.array_equal(t.cpu().numpy().view(np.uint32), ref)))
    # several jobs in flight at once, the same order on every worker
    xs = [[worker_bucket(r, 70_001 + j, 100 + j) for r in range(W)] for j in range(4)]
    ts = [torch.from_numpy(xs[j][rank].copy()).cuda() for j in range(4)]
    jobs = [C.allreduce_async(tt) for tt in ts]
    C.wait_for_all_jobs()
    for j in range(4):
        ref = oracle_switch_allreduce(xs[j], P, T)
        res.append(jobs[j].status() == C.JOB_FINISHED and
                   bool(np.array_equal(ts[j].cpu().numpy().view(np.uint32), ref.view(np.uint32))))
    C.stop()
    return res


def _run(target, W, args, timeout=240):
    """Run `target` in W spawned worker processes (tests/mp_ranks.py: the
    first failing or dead worker ends the wait, a hung one dumps its stack)."""
    return spawn(target, W, args, timeout=timeout, what=f"xgmi workers W={W}")


@pytest.mark.gpu
@pytest.mark.parametrize("W,T,P,push", [(2, 1, 256, False), (3, 2, 64, False), (4, 4, 1024, False),
                                        (2, 1, 256, True), (3, 2, 64, True), (5, 2, 1024, True)])
def test_xgmi_backend_allreduce_matches_oracle_switch(cuda, W, T, P, push):
    """Context::AllReduce with backend = xgmi on W worker processes: FLOAT32
    buckets (device, pageable and pinned host tensors; in place and not;
    ragged sizes, one element, empty, and slices exchanged in several chunks of
    max_slice_numel), INT32 buckets, and four jobs in flight — every result
    bit-exact against the oracle switch over the same W workers, in the pull
    and the push form (backend.xgmi.push: K3 writes into the owners' inboxes)."""
    session = "test-" + uuid.uuid4().hex
    cap = 8192 * (P // 64)
    for rank, res, err in _run(_client_worker, W, (T, P, session, cap, push)):
        assert res is not None, (rank, err)
        assert all(res), (rank, res)


def _client_vcl_worker(rank, W, init, T, P, session, push):
    """backend.hip.vcl = true on the in-node switch: K3 with the reference's
    VCL=1 rounding on tie-heavy buckets, every worker's result bit-exact
    against the oracle switch in that rounding (and different from the
    half-away result, so the flag demonstrably reached the kernel)."""
    from test_client_gpu import tie_bucket
    from switchml_amd import client as C
    C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=T, packet_numel=P,
                          max_outstanding_packets=64 * T, mode="bulk", bandwidth=0, device=0,
                          session=session, push=push, vcl=True))
    res = []
    for i, n in enumerate([100_003, 3 * P + 5]):
        xs = [tie_bucket(n, P, W, 1000 * i + r) for r in range(W)]
        t = torch.from_numpy(xs[rank].copy()).cuda()
        C.allreduce(t)
        ref = oracle_switch_allreduce(xs, P, T, rounding=O.RNE_VCL)
        away = oracle_switch_allreduce(xs, P, T)
        got = t.cpu().numpy().view(np.uint32)
        res.append(bool(np.array_equal(got, ref.view(np.uint32))))
        res.append(i > 0 or not np.array_equal(ref.view(np.uint32), away.view(np.uint32)))
    C.stop()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("W,T,P,push", [(2, 2, 256, False), (4, 1, 64, True)])
def test_xgmi_backend_vcl_rounding(cuda, W, T, P, push):
    session = "vcl-" + uuid.uuid4().hex
    for rank, res, err in _run(_client_vcl_worker, W, (T, P, session, push)):
        assert res is not None, (rank, err)
        assert all(res), (rank, res)


def _plugin_worker(rank, W, init, session):
    ini = ("[general]\nbackend = xgmi\nrank = %d\nnum_workers = %d\nnum_worker_threads = 2\npacket_numel = 256\n"
           "max_outstanding_packets = 128\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = bulk\n"
           "device = 0\n[backend.xgmi]\nsession = %s\n" % (rank, W, session))
    os.environ["SWITCHML_CONFIG_INI"] = ini
    os.environ.pop("SWITCHML_COLLNET_LOOPBACK", None)
    from switchml_amd.collnet import CollNetComm, NCCL_FLOAT32, CollNetError
    comm = CollNetComm(nranks=W, rank=rank)
    sizes = [6_553_600, 5_896_232, 1000]     # ResNet-50 DDP buckets (two of them) + a small one
    xs = [[worker_bucket(r, n, 7 + j) for r in range(W)] for j, n in enumerate(sizes)]
    send = [torch.from_numpy(xs[j][rank].copy()).cuda() for j in range(len(sizes))]
    recv = [torch.empty_like(s) for s in send]
    comm.allreduce_buckets([(s.data_ptr(), r.data_ptr(), s.numel()) for s, r in zip(send, recv)], NCCL_FLOAT32)
    ok = [bool(np.array_equal(recv[j].cpu().numpy().view(np.uint32),
                              oracle_switch_allreduce(xs[j], 256, 2).view(np.uint32))) for j in range(len(sizes))]
    # a communicator that is not the session's workers is refused
    try:
        CollNetComm(nranks=W + 1, rank=rank)
        ok.append(False)
    except CollNetError:
        ok.append(True)
    comm.close()
    from switchml_amd import client as C
    C.stop()
    return ok


@pytest.mark.gpu
def test_collnet_plugin_over_xgmi_backend(cuda):
    """The CollNet table (iallreduce / test, switchml_plugin.cc:293-387) on a
    2-rank communicator with the in-node switch behind it: a real cross-rank
    SwitchML all-reduce of configs[4]-sized buckets, no loopback opt-in."""
    session = "plug-" + uuid.uuid4().hex
    for rank, res, err in _run(_plugin_worker, 2, (session,)):
        assert res is not None, (rank, err)
        assert all(res), (rank, res)


def test_xgmi_config_validation():
    from switchml_amd import client as C
    bad = [dict(backend="xgmi", prepostprocessor="hip_exponent_quantizer"),                 # no session
           dict(backend="xgmi", session="a b"),                                             # bad name
           dict(backend="xgmi", session="ok", rank=2, num_workers=2),                       # rank >= W
           dict(backend="xgmi", session="ok", num_workers=17),
           dict(backend="xgmi", session="ok", prepostprocessor="bypass")]
    for kw in bad:
        with pytest.raises(C.ContextError):
            C.start(C.make_config(bandwidth=0, **kw))
        assert C.state() != C.RUNNING


def _failing_worker(rank, W, init, session, fail_rank):
    """Worker `fail_rank` injects a fault on worker thread 0 of every job
    (backend.dummy.fail_worker_thread); the session is poisoned, so every
    worker's job fails — none hangs on a barrier, none reports FINISHED —
    and the jobs after it fail too (no out-of-phase barriers)."""
    import time
    from switchml_amd import client as C
    kw = dict(fail_worker_thread=0) if rank == fail_rank else {}
    C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=2, packet_numel=256,
                          max_outstanding_packets=128, mode="bulk", bandwidth=0, device=0, session=session,
                          timeout_ms=30000, **kw))
    t0 = time.time()
    sts = []
    for j in range(3):
        x = torch.from_numpy(worker_bucket(rank, 200_000, j)).cuda()
        job = C.allreduce_async(x)
        C.wait_for_all_jobs()
        sts.append(job.status())
    took = time.time() - t0
    C.stop()
    return {"statuses": sts, "seconds": took}


@pytest.mark.gpu
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_xgmi_failure_poisons_session(cuda, fail_rank):
    from switchml_amd import client as C
    session = "fail-" + uuid.uuid4().hex
    for rank, res, err in _run(_failing_worker, 2, (session, fail_rank)):
        assert res is not None, (rank, err)
        assert res["statuses"] == [C.JOB_FAILED] * 3, (rank, res)
        assert res["seconds"] < 20, (rank, res)    # failed fast: no barrier timeout waited out
    assert not os.path.exists(f"/dev/shm/switchml-{session}")


@pytest.mark.gpu
def test_xgmi_replaces_stale_segment(cuda):
    """A segment left by a crashed run (its worker 0 gone, its barrier counts
    and attach count stale) is replaced by the next run's worker 0 instead of
    being joined."""
    import subprocess
    import sys
    session = "stale-" + uuid.uuid4().hex
    p = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True, text=True)
    dead_pid = int(p.stdout)          # a process that has exited
    path = f"/dev/shm/switchml-{session}"
    with open(path, "wb") as f:      # magic "SMLX", W=T=1, stale counters, creator = the dead process
        import struct
        hdr = struct.pack("<IIIIQiIII", 0x534D4C58, 2, 1, 256, 1 << 20, dead_pid, 0, 2, 0)
        f.write(hdr + b"\0" * (1 << 16))
    for rank, res, err in _run(_client_worker, 2, (1, 256, session, 8192 * 4, False)):
        assert res is not None, (rank, err)
        assert all(res), (rank, res)
    assert not os.path.exists(path)


def _stalled_worker(rank, W, init, session, stall_rank, stall_ms, timeout_ms):
    """Worker `stall_rank` queues a kernel that keeps its worker stream busy
    for stall_ms (backend.dummy.stall_worker_thread / stall_ms:
    sml_debug_stall, which ends on its own) before its slice — a device that
    does not finish within backend.xgmi.timeout_ms.  ADVICE r5: the slice must
    be reported FAILED within about timeout_ms, not block the worker thread in
    an unbounded stream synchronize; later jobs fail at once (wedged worker
    or poisoned session); and once the stalled kernel has ended on its own,
    a new session on the same device works again (the wedged switch's reaper
    has freed its planes and closed its peer mappings by then; the new
    switch waits for it)."""
    import time
    from switchml_amd import client as C
    kw = dict(stall_worker_thread=0, stall_ms=stall_ms) if rank == stall_rank else {}
    C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=1, packet_numel=256,
                          max_outstanding_packets=64, mode="bulk", bandwidth=0, device=0, session=session,
                          timeout_ms=timeout_ms, **kw))
    t_start = time.time()
    sts, secs = [], []
    for j in range(2):
        x = torch.from_numpy(worker_bucket(rank, 100_000, j)).cuda()
        t0 = time.time()
        job = C.allreduce_async(x)
        C.wait_for_all_jobs()
        secs.append(time.time() - t0)
        sts.append(job.status())
    C.stop()
    # the stalled kernel ends stall_ms after it started: then the device is usable again
    time.sleep(max(0.0, stall_ms / 1e3 - (time.time() - t_start)) + 0.5)
    torch.cuda.synchronize()
    C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=1, packet_numel=256,
                          max_outstanding_packets=64, mode="bulk", bandwidth=0, device=0,
                          session=session + "-after", timeout_ms=30000))
    xs = [worker_bucket(r, 50_000, 9) for r in range(W)]
    t = torch.from_numpy(xs[rank].copy()).cuda()
    C.allreduce(t)
    after_ok = bool(np.array_equal(t.cpu().numpy().view(np.uint32), oracle_switch_allreduce(xs, 256, 1).view(np.uint32)))
    C.stop()
    return {"statuses": sts, "seconds": secs, "after_ok": after_ok}


@pytest.mark.gpu
@pytest.mark.parametrize("W", [1, 2])
def test_xgmi_stalled_device_fails_slice_within_timeout(cuda, W):
    from switchml_amd import client as C
    session = "stall-" + uuid.uuid4().hex
    stall_ms, timeout_ms = 4000, 300
    out = _run(_stalled_worker, W, (session, 0, stall_ms, timeout_ms), timeout=120)
    for rank, res, err in out:
        assert res is not None, (rank, err)
    allres = {rank: res for rank, res, _ in out}
    for rank, res in allres.items():
        assert res["statuses"] == [C.JOB_FAILED] * 2, allres
        # reported within ~timeout_ms (a few bounded waits at most), long before the stall ends
        assert res["seconds"][0] < 2.0 and res["seconds"][1] < 1.0, allres
        assert res["after_ok"], allres


def _setup_failing_worker(rank, W, init, session, fail_rank):
    """Worker `fail_rank` fails right after joining the session
    (backend.xgmi.fail_setup: what a worker that cannot map a peer's plane
    on its first contact with another GPU does).  It must poison the session
    (first contact): the other workers' Context starts, but their
    first job fails at once — not after backend.xgmi.timeout_ms at a barrier
    the failed worker never reaches — and their Stop does not wait either."""
    import time
    from switchml_amd import client as C
    t0 = time.time()
    try:
        C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=1, packet_numel=256,
                              max_outstanding_packets=64, mode="bulk", bandwidth=0, device=0, session=session,
                              timeout_ms=30000, fail_setup=rank == fail_rank))
    except C.ContextError as e:
        return {"started": False, "error": str(e), "seconds": time.time() - t0}
    x = torch.from_numpy(worker_bucket(rank, 100_000, 1)).cuda()
    job = C.allreduce_async(x)
    try:
        C.wait_for_all_jobs()
    except C.ContextError:
        pass
    st = job.status()
    C.stop()
    return {"started": True, "status": st, "seconds": time.time() - t0}


@pytest.mark.gpu
def test_xgmi_setup_failure_poisons_session(cuda):
    from switchml_amd import client as C
    session = "setupfail-" + uuid.uuid4().hex
    out = {rank: res for rank, res, err in _run(_setup_failing_worker, 2, (session, 1), timeout=120)}
    assert set(out) == {0, 1} and all(v is not None for v in out.values()), out
    assert out[1]["started"] is False and "injected setup failure" in out[1]["error"], out
    assert out[0]["started"] is True and out[0]["status"] == C.JOB_FAILED, out
    assert max(v["seconds"] for v in out.values()) < 20, out      # no 30 s barrier timeout waited out
    assert not os.path.exists(f"/dev/shm/switchml-{session}")
