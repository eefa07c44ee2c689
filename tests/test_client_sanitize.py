"""Host-code sanitizers over the client's threading (CPU only).

tools/sanitize/run.sh builds tools/sanitize/client_stress.cc with the client
sources under -fsanitize=thread (and address): four submitter threads post
ragged jobs to the Context concurrently, wait on some, WaitForAllJobs, and the
context is stopped and restarted with 1, 3 and 5 worker threads.  The bypass
pre/post-processor keeps it off the GPU.  Any sanitizer report fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "p4app-switchml_amd", "switchml_amd", "libswitchml_hip.so")


@pytest.mark.parametrize("san", ["thread", "address"])
def test_client_stress_under_sanitizer(san):
    if shutil.which("g++") is None or not os.path.exists(LIB):
        pytest.skip("needs g++ and the built library")
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize", "run.sh"), san], capture_output=True, text=True,
                       timeout=600)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    assert "client stress ok" in log
    assert "ThreadSanitizer" not in log and "AddressSanitizer" not in log and "LeakSanitizer" not in log, log[-3000:]
