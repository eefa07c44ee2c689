import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "p4app-switchml_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    # heartbeats of long multi-process tests go past pytest's output capture
    # (tests/mp_ranks.py heartbeat): a slow test stays visibly alive
    import mp_ranks
    mp_ranks.CAPTURE_MANAGER = config.pluginmanager.getplugin("capturemanager")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
