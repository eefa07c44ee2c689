"""The RCCL CollNet plugin driven through its exported v6
function table exactly as RCCL's proxy would call it: init, devices,
getProperties, listen/connect, reduceSupport, regMr, iallreduce, test,
deregMr, close.  Reference semantics: frameworks_integration/nccl_plugin/
switchml_plugin.cc:135-402 (iallreduce -> Context::AllReduceAsync, test polls
the Job).  CPU: the table, the bypass PPP (no GPU) and the uint8 widening;
GPU: device and host buffers through the HIP quantizer, bit-exact vs the
oracle's dummy-backend packet loop.

A live RCCL CollNet run needs a multi-node CollNet topology (RCCL disables
CollNet below NCCL_COLLNET_NODE_THRESHOLD nodes), so RCCL itself loading the
plugin is not exercised here."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUGIN = os.path.join(ROOT, "p4app-switchml_amd", "switchml_amd", "librccl-net-switchml.so")

R = ctypes.c_int
vp = ctypes.c_void_p
LOGGER = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p)


class Props(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("pciPath", ctypes.c_char_p), ("guid", ctypes.c_uint64),
                ("ptrSupport", ctypes.c_int), ("speed", ctypes.c_int), ("port", ctypes.c_int),
                ("latency", ctypes.c_float), ("maxComms", ctypes.c_int), ("maxRecvs", ctypes.c_int)]


class CollNetV6(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char_p),
        ("init", ctypes.CFUNCTYPE(R, LOGGER)),
        ("devices", ctypes.CFUNCTYPE(R, ctypes.POINTER(ctypes.c_int))),
        ("getProperties", ctypes.CFUNCTYPE(R, ctypes.c_int, ctypes.POINTER(Props))),
        ("listen", ctypes.CFUNCTYPE(R, ctypes.c_int, vp, ctypes.POINTER(vp))),
        ("connect", ctypes.CFUNCTYPE(R, ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp))),
        ("reduceSupport", ctypes.CFUNCTYPE(R, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int))),
        ("regMr", ctypes.CFUNCTYPE(R, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp))),
        ("regMrDmaBuf", ctypes.CFUNCTYPE(R, vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.POINTER(vp))),
        ("deregMr", ctypes.CFUNCTYPE(R, vp, vp)),
        ("iallreduce", ctypes.CFUNCTYPE(R, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                        ctypes.POINTER(vp))),
        ("iflush", ctypes.CFUNCTYPE(R, vp, vp, ctypes.c_int, vp, ctypes.POINTER(vp))),
        ("test", ctypes.CFUNCTYPE(R, vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))),
        ("closeColl", ctypes.CFUNCTYPE(R, vp)),
        ("closeListen", ctypes.CFUNCTYPE(R, vp)),
    ]


NCCL_UINT8, NCCL_INT32, NCCL_FLOAT32, NCCL_FLOAT64 = 1, 2, 7, 8
NCCL_SUM, NCCL_MAX = 0, 2

DRIVER = r'''
import ctypes, sys, os, json, numpy as np
{preload}
sys.path[:0] = [{root!r}, os.path.join({root!r}, "tests")]
from test_collnet_plugin import CollNetV6, Props, LOGGER, PLUGIN, vp
lib = ctypes.CDLL(PLUGIN)
tbl = CollNetV6.in_dll(lib, "ncclCollNetPlugin_v6")
logger = LOGGER(lambda *a: None)
out = {{"name": tbl.name.decode(), "init": tbl.init(logger)}}
n = ctypes.c_int(); tbl.devices(ctypes.byref(n)); out["ndev"] = n.value
p = Props(); tbl.getProperties(0, ctypes.byref(p))
out["ptrSupport"] = p.ptrSupport; out["maxComms"] = p.maxComms
sup = {{}}
for dt in (1, 2, 7, 8):
    for op in (0, 2):
        s = ctypes.c_int(); tbl.reduceSupport(dt, op, ctypes.byref(s)); sup[f"{{dt}},{{op}}"] = s.value
out["support"] = sup
handle = (ctypes.c_char * 128)(); lcomm = vp()
tbl.listen(0, ctypes.cast(handle, vp), ctypes.byref(lcomm))
handles = (vp * 1)(ctypes.cast(handle, vp)); coll = vp()
out["connect"] = tbl.connect(handles, 1, 0, lcomm, ctypes.byref(coll))
out["connect_bad_rank"] = tbl.connect(handles, 1, -1, lcomm, ctypes.byref(vp()))
def run(send, recv, count, dtype):
    mh = vp(); tbl.regMr(coll, send, 0, 1, ctypes.byref(mh))
    req = vp()
    rc = tbl.iallreduce(coll, send, recv, count, dtype, 0, mh, mh, ctypes.byref(req))
    if rc: return rc
    done, size = ctypes.c_int(0), ctypes.c_int(0)
    while not done.value:
        rc = tbl.test(req, ctypes.byref(done), ctypes.byref(size))
        if rc: return rc
    tbl.deregMr(coll, mh)
    return size.value
{body}
tbl.closeColl(coll); tbl.closeListen(lcomm)
print(json.dumps(out))
'''


def run_driver(body, env_ini, preload=""):
    # With torch in the process, torch must load first: it bundles its own
    # libamdhip64.so.7 (same SONAME as /opt/rocm's), and whichever loads first
    # is the one every library in the process binds to.
    code = DRIVER.format(root=ROOT, body=body, preload=preload)
    env = dict(os.environ, SWITCHML_CONFIG_INI=env_ini)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_plugin_table_and_bypass_allreduce():
    """CPU: the v6 table, properties, reduceSupport, connect, and a bypass-PPP
    all-reduce (no GPU touched), plus the uint8 widening of :318-337."""
    body = '''
x = np.arange(1000, dtype=np.float32)
out["size_f32"] = run(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(x.ctypes.data), 1000, 7)
u = np.arange(200, dtype=np.uint8)
out["size_u8"] = run(ctypes.c_void_p(u.ctypes.data), ctypes.c_void_p(u.ctypes.data), 200, 1)
out["u8_roundtrip"] = bool((u == np.arange(200, dtype=np.uint8)).all())
out["bad_op"] = tbl.iallreduce(coll, None, None, 1, 7, 2, None, None, ctypes.byref(vp()))
'''
    ini = "[general]\nprepostprocessor = bypass\nnum_worker_threads = 2\n[backend.dummy]\nbandwidth = 0\n"
    out = run_driver(body, ini)
    assert out["name"] == "SWITCHMLv1" and out["init"] == 0 and out["ndev"] == 1
    assert out["ptrSupport"] == 3 and out["maxComms"] == 1
    assert out["support"] == {"1,0": 1, "1,2": 0, "2,0": 1, "2,2": 0, "7,0": 1, "7,2": 0, "8,0": 0, "8,2": 0}
    assert out["connect"] == 0 and out["connect_bad_rank"] == 3
    assert out["size_f32"] == 4000 and out["size_u8"] == 200 and out["u8_roundtrip"]
    assert out["bad_op"] == 4


@pytest.mark.gpu
def test_plugin_allreduce_device_and_host_buffers(cuda):
    body = '''
import torch
from oracle import oracle as O
x = O.splitmix_normal(3, 100_003)
ref = O.dummy_allreduce(x, P=256, max_outstanding_packets=256, num_worker_threads=4, num_workers=2)
xd = torch.from_numpy(x).cuda(); od = torch.empty_like(xd)
out["dev_size"] = run(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(od.data_ptr()), x.size, 7)
out["dev_ok"] = bool(np.array_equal(od.cpu().numpy().view(np.uint32), ref.view(np.uint32)))
h = x.copy()
out["host_size"] = run(ctypes.c_void_p(h.ctypes.data), ctypes.c_void_p(h.ctypes.data), x.size, 7)
out["host_ok"] = bool(np.array_equal(h.view(np.uint32), ref.view(np.uint32)))
i = np.arange(-5000, 5000, dtype=np.int32)
run(ctypes.c_void_p(i.ctypes.data), ctypes.c_void_p(i.ctypes.data), i.size, 2)
out["int_ok"] = bool((i == np.arange(-5000, 5000, dtype=np.int32) * 2).all())
ud = torch.zeros(16, dtype=torch.uint8, device="cuda")
out["dev_u8"] = run(ctypes.c_void_p(ud.data_ptr()), ctypes.c_void_p(ud.data_ptr()), 16, 1)
'''
    ini = ("[general]\nnum_workers = 2\nnum_worker_threads = 4\npacket_numel = 256\n"
           "max_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = bulk\n")
    out = run_driver(body, ini, preload="import torch")
    assert out["init"] == 0
    assert out["dev_size"] == 4 * 100_003 and out["dev_ok"]
    assert out["host_size"] == 4 * 100_003 and out["host_ok"]
    assert out["int_ok"]
    assert out["dev_u8"] == 4   # device uint8: ncclInvalidArgument
