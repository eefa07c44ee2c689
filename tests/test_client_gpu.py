"""GPU tests of the C++ client: Context::AllReduce through the loopback
("dummy") backend and the HIP pre/post-processor, in every backend mode,
against the oracle's restatement of the reference packet loop
(DummyWorkerThread + CpuExponentQuantizerPPP, T worker-thread slices).
Bit-exact on the fp32 output words."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "p4app-switchml_amd", "bin")


@pytest.fixture
def C(cuda):
    from switchml_amd import client
    yield client
    if client.state() == client.RUNNING:
        client.stop()


def bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def _mode(mode):
    """'fused-threads': mode fused with batched dispatch off (batch_jobs = 0)."""
    return dict(mode="fused", batch_jobs=0) if mode == "fused-threads" else dict(mode=mode)


@pytest.mark.parametrize("mode", ["bulk", "fused", "fused-threads", "packet"])
@pytest.mark.parametrize("T,W,P", [(1, 1, 256), (4, 2, 256), (3, 3, 64), (2, 8, 1024), (2, 5, 128), (3, 4, 512)])
def test_allreduce_float_host_tensors(C, mode, T, W, P):
    n = 100_003 if mode != "packet" else 20_011
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                          bandwidth=0, **_mode(mode)))
    x = O.splitmix_normal(T * 100 + W, n)
    ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W)
    out = np.empty_like(x)
    C.allreduce(x, out)
    assert bits_equal(out, ref)
    # in place, twice (the allreduce_benchmark --inplace pattern)
    y = x.copy()
    C.allreduce(y)
    C.allreduce(y)
    ref2 = O.dummy_allreduce(ref, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W)
    assert bits_equal(y, ref2)
    C.stop()


@pytest.mark.parametrize("ring", ["device", "pinned", "pageable", "pinned+server"])
@pytest.mark.parametrize("T,W,P,n", [(2, 2, 256, 20_011), (1, 3, 64, 4_099), (3, 8, 1024, 30_001)])
def test_packet_mode_ring_placements(C, ring, T, W, P, n):
    """The per-LTU PreprocessSingle / PostprocessSingle calls with the packet
    ring in HBM (kernels write / read the packets in place, stream-ordered),
    in pinned host memory (kernels over PCIe, synchronous calls; "+server":
    through the persistent burst server, backend.hip.burst_server) and in
    pageable host memory (staged through HBM): the reference's packet stream
    (dummy_worker_thread.cc:86-177), bit-exact with the oracle, FLOAT32
    and INT32."""
    place, server = ring.split("+")[0], ring.endswith("+server")
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=16 * T,
                          mode="packet", packet_ring=place, burst_server=server, bandwidth=0))
    x = O.splitmix_normal(n + W, n)
    ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=16 * T, num_worker_threads=T, num_workers=W)
    out = np.empty_like(x)
    C.allreduce(x, out)
    assert bits_equal(out, ref)
    xi = np.random.default_rng(n).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    oi = np.empty_like(xi)
    C.allreduce(xi, oi)
    assert np.array_equal(oi, (xi.astype(np.int64) * W).astype(np.int32))
    C.stop()


@pytest.mark.parametrize("mode", ["bulk", "fused", "fused-threads", "packet"])
def test_allreduce_pinned_host_tensors(C, mode):
    """Pinned (page-locked) host tensors go to the kernels through their
    device mapping — zero-copy over PCIe, no staging copies; in place and
    not, ragged T = 3 slices (misaligned slice starts), bit-exact."""
    import torch
    T, W, P = 3, 2, 256
    n = 100_003 if mode != "packet" else 20_011
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                          bandwidth=0, **_mode(mode)))
    x = O.splitmix_normal(17, n)
    ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W)
    hx = torch.from_numpy(x.copy()).pin_memory()
    ho = torch.empty_like(hx).pin_memory()
    C.allreduce(hx, ho)
    assert bits_equal(ho.numpy(), ref)
    assert bits_equal(hx.numpy(), x)          # input untouched
    C.allreduce(hx)                           # in place
    assert bits_equal(hx.numpy(), ref)
    C.stop()


@pytest.mark.parametrize("mode", ["bulk", "fused", "fused-threads"])
def test_allreduce_device_tensors(C, mode):
    import torch
    T, W, P, n = 4, 2, 256, 1_000_003
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, bandwidth=0, **_mode(mode)))
    x = O.splitmix_normal(5, n)
    xd = torch.from_numpy(x).cuda()
    outd = torch.empty_like(xd)
    jobs = [C.allreduce_async(xd, outd) for _ in range(3)]
    C.wait_for_all_jobs()
    assert all(j.status() == C.JOB_FINISHED for j in jobs)
    ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=256, num_worker_threads=T, num_workers=W)
    assert bits_equal(outd.cpu().numpy(), ref)
    C.stop()


@pytest.mark.parametrize("mode", ["bulk", "packet"])
def test_allreduce_int32(C, mode):
    """INT32 jobs: byteswap pre/post, loopback x W with int32 wrap (dummy_backend.cc:72-84)."""
    T, W, n = 4, 3, 50_001
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=256, mode=mode, bandwidth=0))
    rng = np.random.default_rng(1)
    x = rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    out = np.empty_like(x)
    C.allreduce(x, out)
    expect = (x.astype(np.int64) * W).astype(np.int32)   # wraps
    assert np.array_equal(out, expect)
    C.stop()


def test_hello_world_binary(cuda):
    r = subprocess.run([os.path.join(BIN, "hello_world")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Data verified successfully" in r.stdout


@pytest.mark.parametrize("ttype", ["float", "int32"])
@pytest.mark.parametrize("device", ["cpu", "gpu"])
def test_allreduce_benchmark_not_in_place(cuda, device, ttype):
    """--inplace false: the output is W x input and the input buffer is
    verified untouched, as main.cc:352-391 checks both buffers.  (float uses
    the fixed pattern: the reference's random float bit patterns span ~2^250
    inside one packet, so the quantizer — the reference's too — rounds the
    small elements of a block to 0 and its own 1 % check fails on them.)"""
    r = subprocess.run([os.path.join(BIN, "allreduce_benchmark"), "--tensor-numel", "300007",
                        "--tensor-type", ttype, "--verify", "true", "--inplace", "false", "--num-workers", "3",
                        "--num-jobs", "3", "--num-warmup-jobs", "1", "--bandwidth", "0", "--device", device,
                        "--mode", "fused"] + (["--random", "true", "--seed", "5"] if ttype == "int32" else []),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Data verified successfully." in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("mode", ["packet"])
def test_allreduce_benchmark_packet_mode(cuda, mode):
    """The per-LTU path at a real size (4 M elements, T = 4): every packet is
    two stream-ordered launches into the HBM ring, no host sync per packet."""
    r = subprocess.run([os.path.join(BIN, "allreduce_benchmark"), "--tensor-numel", "4194304",
                        "--tensor-type", "float", "--verify", "true", "--num-workers", "2", "--num-jobs", "2",
                        "--num-warmup-jobs", "1", "--bandwidth", "0", "--device", "gpu", "--mode", mode],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Data verified successfully." in r.stdout, r.stdout[-2000:]
    print([l for l in r.stdout.splitlines() if l.startswith("Median")])


@pytest.mark.parametrize("device", ["cpu", "gpu"])
def test_allreduce_benchmark_cfg1(cuda, device):
    """configs[0]: allreduce benchmark, loopback backend, 4 MiB float tensor,
    num_workers = 2 (each of the reference's 2 processes is independent under
    the dummy backend), --verify with the reference's formula."""
    r = subprocess.run([os.path.join(BIN, "allreduce_benchmark"), "--tensor-numel", "1048576",
                        "--tensor-type", "float", "--verify", "true", "--num-workers", "2",
                        "--bandwidth", "0", "--device", device, "--mode", "bulk"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Data verified successfully." in r.stdout
    assert "Median" in r.stdout and "Gbps" in r.stdout


def test_dnn_benchmark_example_model_device(C):
    """dnn_benchmark's flow on its example model (models/example.csv, via
    tests/golden/dnn_example_model.json): one device buffer, each layer a
    slice of it (ragged numels: most slices start 4-12 bytes off a 16-B
    boundary), AllReduceAsync of every layer in place in backward order
    (dnn_benchmark/main.cc:312-318), all jobs in flight, then WaitForAllJobs;
    bit-exact against the oracle's per-layer packet loop (T = 4 FIFO slices)."""
    import json
    import torch
    with open(os.path.join(ROOT, "tests", "golden", "dnn_example_model.json")) as f:
        layers = [l[1] for l in json.load(f)["layers"]]
    T, W, P, iters = 4, 2, 256, 2
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=256,
                          mode="bulk", bandwidth=0))
    x = O.ref_pattern_floats(sum(layers))
    offs = np.concatenate([[0], np.cumsum(layers)]).astype(np.int64)
    xd = torch.from_numpy(x).cuda()
    ref = x.copy()
    for _ in range(iters):
        jobs = []
        for li in reversed(range(len(layers))):
            v = xd[offs[li]:offs[li + 1]]
            jobs.append(C.allreduce_async(v))
            r = ref[offs[li]:offs[li + 1]]
            O.dummy_allreduce(r, P=P, max_outstanding_packets=256, num_worker_threads=T, num_workers=W,
                              threaded=True, out=r)
        C.wait_for_all_jobs()
        del jobs
    torch.cuda.synchronize()
    assert bits_equal(xd.cpu().numpy(), ref)


def _busy(torch):
    """Keep torch's current stream busy for a while (so the kernels queued
    after this still wait when the next host call runs)."""
    a = torch.randn(2048, 2048, device="cuda")
    for _ in range(40):
        a = a @ a
        a = a / a.abs().max()
    return a


@pytest.mark.parametrize("mode", ["fused", "bulk"])
def test_allreduce_waits_for_the_producing_stream(C, mode):
    """Device tensors still being produced on torch's stream when the job is
    submitted: the Python client makes them ready first (the reference's
    ProcessGroupSML synchronizes its stream before AllReduceAsync,
    ProcessGroupSML.cpp:137-151).  Without that the worker stream reads the
    input before the producing kernel wrote it, and writes an output block
    the caching allocator has just recycled from a tensor a queued kernel
    still reads (what made a 5 GiB test fail inside the full suite)."""
    import torch
    n, W, T = 1 << 22, 2, 4
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=256, max_outstanding_packets=64 * T,
                          bandwidth=0, mode=mode))
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    src = torch.randn(n, device="cuda", generator=g)
    torch.cuda.synchronize()
    want_in = src * 3.0
    _busy(torch)                        # queued ahead of the producer below
    t = src.clone()
    x = t * 3.0                         # producer, queued behind the busy work
    del t                               # its block may come back as `out`
    out = torch.empty_like(x)
    C.allreduce(x, out)
    torch.cuda.synchronize()
    assert torch.equal(x, want_in)
    ref = O.dummy_allreduce(want_in.cpu().numpy(), P=256, max_outstanding_packets=64 * T, num_worker_threads=T,
                            num_workers=W)
    assert bits_equal(out.cpu().numpy(), ref)


def tie_bucket(n, P, W, seed):
    """FLOAT32 bucket whose quantized values are mostly exact .5 ties: every
    block holds a 1.0 (exponent e = 1, scale = 2^30 / W, exact for
    power-of-two W) and elements ±(m + 0.5)·W·2^-30 (x·scale = ±(m + 0.5),
    exact), the rest N(0, 0.25) clipped inside (-1, 1)."""
    rng = np.random.default_rng(seed)
    x = np.clip(rng.standard_normal(n) * 0.25, -0.99, 0.99).astype(np.float32)
    m = rng.integers(0, 1 << 20, n)
    ties = ((m + 0.5) * W * 2.0 ** -30 * np.where(rng.random(n) < 0.5, -1.0, 1.0)).astype(np.float32)
    sel = rng.random(n) < 0.6
    x[sel] = ties[sel]
    x[::P] = 1.0
    return x


@pytest.mark.parametrize("mode", ["bulk", "fused", "fused-threads", "packet", "packet-pinned-server"])
@pytest.mark.parametrize("T,W,P", [(1, 1, 256), (4, 2, 256), (3, 8, 64), (2, 2, 1024)])
def test_vcl_rounding_through_context(C, mode, T, W, P):
    """backend.hip.vcl = true: the reference's VCL=1 build (its default,
    client_lib/Makefile:26,113-120) — round-to-nearest-even on each packet's
    16-element vector body, roundf on the tail (ppp.cc:88-99) — through
    every dispatch of the Context, bit-exact against the oracle's VCL=1
    packet loop; on tie-heavy buckets, so the two builds' results differ."""
    n = 100_003 if not mode.startswith("packet") else 20_011
    kw = _mode(mode) if not mode.startswith("packet") else dict(mode="packet")
    if mode == "packet-pinned-server":
        kw.update(packet_ring="pinned", burst_server=True)
    C.start(C.make_config(num_workers=W, num_worker_threads=T, packet_numel=P, max_outstanding_packets=64 * T,
                          bandwidth=0, vcl=True, **kw))
    assert "vcl = true" in C.config_text()
    x = tie_bucket(n, P, W, T * 10 + W)
    ref = O.dummy_allreduce(x, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W, vcl=True)
    away = O.dummy_allreduce(x, P=P, max_outstanding_packets=64 * T, num_worker_threads=T, num_workers=W)
    assert not bits_equal(ref, away)          # the ties make the two builds differ
    out = np.empty_like(x)
    C.allreduce(x, out)
    assert bits_equal(out, ref)
    C.stop()
