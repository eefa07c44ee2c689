"""RCCL with the SwitchML plugin library loaded (switchml_amd/rccl_collnet.py):
two worker processes share cuda:0 as two RCCL "nodes" (distinct NCCL_HOSTID),
NCCL_NET_PLUGIN = librccl-net-switchml.so, NCCL_COLLNET_ENABLE=1.

* RCCL loads the library's net table, whose TCP net initialises (no
  SWITCHML_NET_PLUGIN needed) and carries RCCL's p2p traffic: RCCL's
  all-reduce of integer-valued data equals the exact sum bit for bit;
* the CollNet table declines RCCL (RCCL 7.2's CollNet AllReduce does not
  reduce / hangs on MI355X): RCCL logs its fallback, and no
  all-reduce reaches iallreduce behind the caller's back;
* the same table driven by hand in the same processes (the in-node xgmi
  switch behind it) equals the exact sum on the integer data and stays
  within the quantization bound on N(0,1) data.
Reference: frameworks_integration/nccl_plugin/switchml_plugin.cc:37,389-402."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_rccl_runs_over_switchml_net_and_collnet_declines(cuda, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
    from switchml_amd import rccl_collnet as R
    rep = R.launch(2, same_gpu=True, numel=1 << 20, iters=1, timeout=200, log_dir=str(tmp_path))
    assert rep["returncodes"] == [0, 0], rep.get("tails")
    assert rep["collnet_declined"] and not rep["collnet_dispatched_by_rccl"]
    for r in rep["ranks"]:
        assert r["int_exact"] and r["hand_int_exact"] and r["int_equal_direct"] and r["normal_within_bound"], r
        assert r["stats_after_first"]["iallreduce"] == r["stats_before"]["iallreduce"]
    assert rep["ok"]
    logs = "".join(open(os.path.join(tmp_path, f), errors="replace").read()
                   for f in os.listdir(tmp_path) if f.startswith("rccl."))
    assert "Loaded net plugin SWITCHML" in logs and "Loaded collnet plugin SWITCHMLv1" in logs
    assert "NET/SWITCHML : TCP net" in logs
    assert "via NET/SWITCHML" in logs                     # RCCL's connections use the library's net
    assert "not offered to RCCL" in logs


def test_worker_env_drops_launcher_state():
    """Workers started from a torch.distributed.run rank must not inherit its
    agent-store rendezvous (a tcp:// init would wait for a store server that
    never starts) or its RANK / WORLD_SIZE / MASTER_*."""
    sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
    from switchml_amd import rccl_collnet as R
    parent = {"TORCHELASTIC_USE_AGENT_STORE": "True", "TORCHELASTIC_RESTART_COUNT": "0", "RANK": "3",
              "WORLD_SIZE": "8", "LOCAL_RANK": "3", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29500",
              "GROUP_RANK": "0", "SWITCHML_NET_PLUGIN": "/x.so", "PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    env = R.worker_env(parent, 1, 2, 1, "s1", extra_env={"FOO": "1"})
    for k in ("TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RESTART_COUNT", "RANK", "WORLD_SIZE", "LOCAL_RANK",
              "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK", "SWITCHML_NET_PLUGIN"):
        assert k not in env, k
    assert env["PATH"] == "/usr/bin" and env["FOO"] == "1"
    assert env["NCCL_NET_PLUGIN"].endswith("librccl-net-switchml.so") and env["NCCL_COLLNET_ENABLE"] == "1"
    assert env["NCCL_HOSTID"] == "switchml-worker-s1-1"
    assert "rank = 1" in env["SWITCHML_CONFIG_INI"] and "device = 1" in env["SWITCHML_CONFIG_INI"]


def test_installed_rccl_has_no_collnet_allreduce_device_code():
    """Why the CollNet table declines RCCL: the RCCL builds
    on this image hold AllReduce device functions for RING and TREE only —
    no ncclDevFunc_AllReduce_COLLNET_* exists, so no CollNet plugin can be
    handed an all-reduce by them (tools/rccl_devfuncs.py)."""
    import importlib.util
    import json
    import subprocess
    libs = ["/opt/rocm/lib/librccl.so"]
    spec = importlib.util.find_spec("torch")
    if spec is not None:
        libs.append(os.path.join(os.path.dirname(spec.origin), "lib", "librccl.so"))
    libs = [l for l in libs if os.path.exists(l)]
    if not libs:
        pytest.skip("no librccl.so on this machine")
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "rccl_devfuncs.py")
    for lib in libs:
        out = subprocess.run([sys.executable, tool, lib], capture_output=True, text=True, check=True).stdout
        rep = json.loads(out)
        assert rep["device_functions"] > 100, lib
        assert "RING" in rep["allreduce_algorithms_with_device_code"], lib
        assert rep["collnet_allreduce_device_functions"] == [], lib


def test_same_gpu_rccl_env():
    """W ranks sharing one GPU under RCCL (tests/test_switch_rccl_gpu.py, the
    bench rehearsal): a distinct NCCL_HOSTID per rank, and a net between them
    — this library's TCP net or RCCL's socket net on the loopback."""
    sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
    from switchml_amd import rccl_collnet as R
    a, b = R.same_gpu_rccl_env(0, "s"), R.same_gpu_rccl_env(1, "s")
    assert a["NCCL_HOSTID"] != b["NCCL_HOSTID"]
    assert a["NCCL_NET_PLUGIN"].endswith("librccl-net-switchml.so") and "NCCL_COLLNET_ENABLE" not in a
    s = R.same_gpu_rccl_env(1, "s", net="socket")
    assert s["NCCL_NET"] == "Socket" and s["NCCL_SOCKET_IFNAME"] == "lo" and s["NCCL_NET_PLUGIN"] == "none"
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in (a, b, s))
    with pytest.raises(ValueError):
        R.same_gpu_rccl_env(0, "s", net="ib")
