"""CPU tests of the C++ client (Context / FIFO scheduler / loopback backend)
through include/switchml_client.h.  They use the reference's `bypass` PPP
(bypass_ppp.h: counts packets, moves no data) or instant_job_completion, so
no GPU is touched: job lifecycle, slicing into packets, config validation."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def client():
    from switchml_amd import client as C
    return C


@pytest.fixture
def ctx(client):
    yield client
    if client.state() == client.RUNNING:
        client.stop()


def test_start_stop_states(ctx):
    C = ctx
    assert C.state() in (C.CREATED, C.STOPPED)
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=2, bandwidth=0))
    assert C.state() == C.RUNNING
    with pytest.raises(C.ContextError):
        C.start(C.make_config(prepostprocessor="bypass"))   # already running
    C.stop()
    assert C.state() == C.STOPPED
    with pytest.raises(C.ContextError):
        C.stop()


@pytest.mark.parametrize("T", [1, 3, 4, 8])
@pytest.mark.parametrize("numel", [1, 255, 256, 257, 1_000_003])
def test_bypass_jobs_slices_and_packet_counts(ctx, T, numel):
    """Every job is cut into T FIFO slices (fifo_scheduler.cc:93-109); each
    slice needs ceil(slice_bytes / ltu) packets (bypass has no extra batch)."""
    C = ctx
    P = 256
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=T, packet_numel=P,
                          max_outstanding_packets=256, bandwidth=0))
    x = np.zeros(numel, dtype=np.float32)
    jobs = [C.allreduce_async(x) for _ in range(3)]
    C.wait_for_all_jobs()
    assert all(j.status() == C.JOB_FINISHED for j in jobs)
    assert len({j.id for j in jobs}) == 3
    st = C.stats()
    expect_packets = 0
    nonempty = 0
    for t in range(T):
        off, n = O.slice_geometry(numel, T, t)
        expect_packets += O.num_blocks(n, P)
        nonempty += n > 0
    assert st["jobs_submitted"] == 3 and st["jobs_finished"] == 3
    assert st["numel_submitted"] == 3 * numel
    assert st["slices"] == 3 * nonempty
    assert st["packets"] == 3 * expect_packets
    C.stop()


def test_instant_job_completion(ctx):
    C = ctx
    C.start(C.make_config(prepostprocessor="hip_exponent_quantizer", instant_job_completion=True,
                          num_worker_threads=4, bandwidth=0, device=0))
    x = np.ones(1000, dtype=np.float32)
    j = C.allreduce_async(x)
    j.wait()
    assert j.status() == C.JOB_FINISHED
    assert np.all(x == 1)   # untouched
    C.stop()


def test_config_validation(ctx):
    C = ctx
    # max_outstanding_packets rounded to a multiple of num_worker_threads (config.cc:160-170)
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=3, max_outstanding_packets=256, bandwidth=0))
    assert "max_outstanding_packets = 255" in C.config_text()
    C.stop()
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=4, max_outstanding_packets=255, bandwidth=0))
    assert "max_outstanding_packets = 256" in C.config_text()
    assert "coalesce_us = 20" in C.config_text()          # zero-copy coalescing window, default
    C.stop()
    C.start(C.make_config(prepostprocessor="bypass", coalesce_us=0, bandwidth=0))
    assert "coalesce_us = 0" in C.config_text()
    assert "burst_server = false" in C.config_text() and "push = false" in C.config_text()   # defaults
    C.stop()
    C.start(C.make_config(prepostprocessor="bypass", burst_server=True, push=True, bandwidth=0))
    assert "burst_server = true" in C.config_text() and "push = true" in C.config_text()
    C.stop()
    # the VCL=1 build's rounding (backend.hip.vcl): off by default, on when asked
    C.start(C.make_config(prepostprocessor="bypass", bandwidth=0))
    assert "vcl = false" in C.config_text()
    C.stop()
    C.start(C.make_config(prepostprocessor="bypass", vcl=True, bandwidth=0))
    assert "vcl = true" in C.config_text()
    C.stop()
    # the fault-injection keys (round 6): a stalled worker stream, a failed xgmi setup — off by default
    C.start(C.make_config(prepostprocessor="bypass", bandwidth=0))
    t = C.config_text()
    assert "stall_worker_thread = -1" in t and "stall_ms = 0" in t and "fail_setup = false" in t
    C.stop()
    C.start(C.make_config(prepostprocessor="bypass", bandwidth=0, stall_worker_thread=1, stall_ms=250,
                          fail_setup=True))
    t = C.config_text()
    assert "stall_worker_thread = 1" in t and "stall_ms = 250" in t and "fail_setup = true" in t
    C.stop()
    with pytest.raises(C.ContextError):                    # at most 60 s of injected stall
        C.start(C.make_config(prepostprocessor="bypass", bandwidth=0, stall_ms=60001))
    for bad in (dict(prepostprocessor="nope"), dict(backend="dpdk"), dict(mode="turbo"),
                dict(num_worker_threads=8, max_outstanding_packets=4)):
        kw = dict(prepostprocessor="bypass", bandwidth=0)
        kw.update(bad)
        with pytest.raises(C.ContextError):
            C.start(C.make_config(**kw))
        if C.state() == C.RUNNING:   # a bad PPP name fails in the workers, not at Start
            C.stop()


def test_reference_style_config_starts_unchanged(ctx):
    """A user's switchml.cfg as the reference's Makefile assembles it (the
    [general] keys of client_lib/src/configs/general.cfg, a backend section as
    dummy.cfg's, the [timeouts] of timeouts.cfg — key names from those files,
    values chosen here) starts the Context as it is: every [general] key is
    read, controller_* are kept (no controller in this build), keys of
    subsystems out of scope are ignored with a note, never fatal."""
    C = ctx
    ini = """
# switchml.cfg
[general]
rank = 0
num_workers = 2
num_worker_threads = 4
max_outstanding_packets = 256
packet_numel = 256
backend = dummy
scheduler = fifo
prepostprocessor = bypass
instant_job_completion = false
controller_ip = 10.0.0.7
controller_port = 50099

[backend.dummy]
bandwidth = 0
process_packets = true

[timeouts]
timeout = 10
timeout_threshold = 100
timeout_threshold_increment = 100
"""
    C.start(ini)
    txt = C.config_text()
    for want in ("num_workers = 2", "num_worker_threads = 4", "max_outstanding_packets = 256", "packet_numel = 256",
                 "backend = dummy", "scheduler = fifo", "prepostprocessor = bypass", "controller_ip = 10.0.0.7",
                 "controller_port = 50099"):
        assert want in txt, want
    j = C.allreduce_async(np.ones(10_000, dtype=np.float32))
    j.wait()
    assert j.status() == C.JOB_FINISHED
    C.stop()


def test_bad_ppp_name_fails_jobs_not_process(ctx):
    C = ctx
    try:
        C.start(C.make_config(prepostprocessor="no_such_ppp", bandwidth=0))
    except C.ContextError:
        return  # rejected up front is fine too
    j = C.allreduce_async(np.ones(10, dtype=np.float32))
    with pytest.raises(C.ContextError):
        j.wait()
    assert j.status() == C.JOB_FAILED
    C.stop()


def test_job_wait_after_stop_fails_queued(ctx):
    C = ctx
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=2, bandwidth=1e-3))  # slow "wire"
    x = np.zeros(1 << 16, dtype=np.float32)
    jobs = [C.allreduce_async(x) for _ in range(4)]
    C.stop()
    states = [j.status() for j in jobs]
    assert all(s in (C.JOB_FINISHED, C.JOB_FAILED) for s in states)
    assert C.JOB_FAILED in states


def test_empty_job_finishes(ctx):
    """numel = 0: every slice is empty and the job completes without the PPP
    (dummy_worker_thread.cc:87)."""
    C = ctx
    C.start(C.make_config(prepostprocessor="hip_exponent_quantizer", num_worker_threads=3, bandwidth=0, device=0))
    x = np.zeros(0, dtype=np.float32)
    j = C.allreduce_async(x)
    j.wait()
    assert j.status() == C.JOB_FINISHED
    C.stop()


def test_failed_slice_publishes_only_after_siblings(ctx):
    """One worker thread fails its slice at once (backend.dummy.fail_worker_thread,
    fault injection); its siblings are still on the simulated wire.  The job
    must not be published FAILED — waking sml_job_wait / WaitToComplete —
    until every sibling slice has stopped touching the buffers (ADVICE r1:
    a caller freeing its buffers on FAILED raced the running slices)."""
    import time
    C = ctx
    T, numel = 4, 1 << 20
    # bypass PPP: every slice of 2^18 elements = 1024 packets of 1 KiB; at
    # 80 Mbps x T the wire wait per healthy slice is ~0.4 s
    C.start(C.make_config(prepostprocessor="bypass", num_worker_threads=T, packet_numel=256,
                          max_outstanding_packets=256, bandwidth=80, fail_worker_thread=1))
    x = np.zeros(numel, dtype=np.float32)
    t0 = time.perf_counter()
    j = C.allreduce_async(x)
    with pytest.raises(C.ContextError):
        j.wait()
    waited = time.perf_counter() - t0
    assert j.status() == C.JOB_FAILED
    expect_wire = 1024 * 256 * 4 * 8 * T / 80e6
    assert waited >= 0.8 * expect_wire, (waited, expect_wire)
    st = C.stats()
    assert st["slices"] == T - 1          # the three healthy slices all ran to the end
    C.wait_for_all_jobs()
    C.stop()
