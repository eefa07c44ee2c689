"""The per-LTU trap.  A reference worker that keeps its
config (`prepostprocessor = cpu_exponent_quantizer`, the reference default)
and calls PreprocessSingle / PostprocessSingle once per 1 KiB packet
(DpdkWorkerThread's BuildPacket, dpdk_worker_thread_utils.inc:134) would get
the MI355X quantizer at one launch + host sync per packet, ~100x slower than
the CPU loop, with no warning.  Under that name the per-LTU calls now refuse
with an error that names `hip_exponent_quantizer` and the burst hooks; the
bulk / burst hooks this repo's backends use are unaffected.

CPU: the factory's policy through the C-ABI (sml_ppp_per_ltu_calls).
GPU: bin/per_ltu_worker, the reference's per-packet call pattern through the
factory: refused under cpu_exponent_quantizer; under hip_exponent_quantizer
the packets it builds dequantize bit-exact to the oracle's loopback."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "p4app-switchml_amd", "bin", "per_ltu_worker")


def test_factory_per_ltu_policy():
    from switchml_amd import client as C
    assert C.ppp_per_ltu_calls("hip_exponent_quantizer") is True
    assert C.ppp_per_ltu_calls("bypass") is True
    assert C.ppp_per_ltu_calls("cpu_exponent_quantizer") is False
    with pytest.raises(C.ContextError, match="not a valid prepostprocessor"):
        C.ppp_per_ltu_calls("gpu_magic")


def test_per_ltu_worker_is_built():
    assert os.access(BIN, os.X_OK), "build() makes bin/per_ltu_worker"


def test_per_packet_worker_refused_at_setup(tmp_path):
    """a per-packet worker asks the factory's policy at setup
    (sml_ppp_per_ltu_calls / PrePostProcessor::PerLtuCalls), so the
    reference's default name fails at configuration time — before any HIP
    call or packet (this runs without a GPU) — naming the hooks to use."""
    r = subprocess.run([BIN, "cpu_exponent_quantizer", "70001", str(tmp_path / "o.f32")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3, r.stdout + r.stderr
    assert r.stdout.startswith("REFUSED at setup:")
    assert "hip_exponent_quantizer" in r.stdout and "PreprocessBurst" in r.stdout
    assert not (tmp_path / "o.f32").exists()
    r = subprocess.run([BIN, "gpu_magic", "70001", str(tmp_path / "o.f32")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1 and "not a valid prepostprocessor" in r.stdout


@pytest.mark.gpu
def test_reference_per_packet_caller_is_refused(cuda, tmp_path):
    """The data-path trap behind the setup check: a worker that skips it
    still gets the PPP's refusal at its first packet."""
    r = subprocess.run([BIN, "cpu_exponent_quantizer", "70001", str(tmp_path / "o.f32")], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, PER_LTU_NO_SETUP_CHECK="1"))
    assert r.returncode == 3, r.stdout + r.stderr
    assert r.stdout.startswith("REFUSED PreprocessSingle:")
    assert "hip_exponent_quantizer" in r.stdout and "PreprocessBurst" in r.stdout
    assert not (tmp_path / "o.f32").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("numel", [70_001, 256 * 64, 300])
def test_per_packet_caller_under_hip_name_is_exact(cuda, tmp_path, numel):
    out = tmp_path / "o.f32"
    r = subprocess.run([BIN, "hip_exponent_quantizer", str(numel), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    x = np.arange(numel, dtype=np.float32) * np.where(np.arange(numel) % 2, -1, 1).astype(np.float32)
    ref = O.dummy_allreduce(x, P=256, max_outstanding_packets=64, num_worker_threads=1, num_workers=1)
    got = np.fromfile(out, dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cpu_exponent_quantizer", "hip_exponent_quantizer"])
def test_burst_hooks_over_registered_pools_are_exact(cuda, tmp_path, name):
    """the burst hooks over a NIC-like pool — ring and extra-info
    slots in two separate hipHostRegister'd allocations, whose device
    addresses may differ from their host addresses and from each other's
    offset — translate every buffer by its own registration.  The reference
    name takes the burst hooks (only its per-packet calls are refused)."""
    out = tmp_path / "o.f32"
    numel = 70_001
    r = subprocess.run([BIN, name, str(numel), str(out), "burst-registered"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    x = np.arange(numel, dtype=np.float32) * np.where(np.arange(numel) % 2, -1, 1).astype(np.float32)
    ref = O.dummy_allreduce(x, P=256, max_outstanding_packets=64, num_worker_threads=1, num_workers=1)
    assert np.array_equal(np.fromfile(out, dtype=np.float32).view(np.uint32), ref.view(np.uint32))
