"""GPU: a plain C program drives the kernel C-ABI (include/switchml_hip.h)
without Python or C++ (p4app-switchml_amd/benchmarks/capi_roundtrip.c):
quantize+pack -> loopback x W -> dequantize of one slice, checked against
the reference's verify rule (allreduce_benchmark/main.cc:343-356) and the
quantizer's error bound.  The bit-exact checks of the same entry points are
tests/test_gpu_parity.py (through ctypes)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "p4app-switchml_amd", "bin",
                   "capi_roundtrip")


@pytest.mark.parametrize("args", [("1000003", "256", "4"), ("65537", "64", "1"), ("4194305", "1024", "8"),
                                  ("1", "128", "3")])
def test_c_program_round_trip(cuda, args):
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi ok" in r.stdout
