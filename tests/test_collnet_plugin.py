"""The RCCL CollNet plugin driven through its exported v6
function table exactly as RCCL's proxy would call it: init, devices,
getProperties, listen/connect, reduceSupport, regMr, iallreduce, test,
deregMr, close.  Reference semantics: frameworks_integration/nccl_plugin/
switchml_plugin.cc:135-402 (iallreduce -> Context::AllReduceAsync, test polls
the Job).  CPU: the table, the bypass PPP (no GPU) and the uint8 widening;
GPU: device and host buffers through the HIP quantizer, bit-exact vs the
oracle's dummy-backend packet loop.

RCCL itself calling the table (every rank its own CollNet "node" through
NCCL_HOSTID, the xgmi in-node switch as backend) is
tests/test_rccl_collnet.py; here the table is driven by hand."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUGIN = os.path.join(ROOT, "p4app-switchml_amd", "switchml_amd", "librccl-net-switchml.so")

sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
from switchml_amd.collnet import (LOGGER, NCCL_FLOAT32, NCCL_FLOAT64, NCCL_INT32, NCCL_MAX,  # noqa: E402,F401
                                  NCCL_SUM, NCCL_UINT8, CollNetV6, Props, vp)

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


def run_driver(body, env_ini, preload="", loopback_opt_in=True):
    # With torch in the process, torch must load first: it bundles its own
    # libamdhip64.so.7 (same SONAME as /opt/rocm's), and whichever loads first
    # is the one every library in the process binds to.
    code = DRIVER.format(root=ROOT, body=body, preload=preload)
    env = dict(os.environ, SWITCHML_CONFIG_INI=env_ini)
    env.pop("SWITCHML_COLLNET_LOOPBACK", None)
    if loopback_opt_in:   # the loopback backend does not reduce across ranks: explicit opt-in
        env["SWITCHML_COLLNET_LOOPBACK"] = "1"
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
uv = (np.arange(1000) * 37 % 256).astype(np.uint8)
ud = torch.from_numpy(uv).cuda(); uo = torch.full((1000,), 7, dtype=torch.uint8, device="cuda")
out["dev_u8"] = run(ctypes.c_void_p(ud.data_ptr()), ctypes.c_void_p(uo.data_ptr()), 1000, 1)
out["dev_u8_ok"] = bool(np.array_equal(uo.cpu().numpy(), (uv.astype(np.int64) * 2 % 256).astype(np.uint8)))
out["dev_u8_send_untouched"] = bool(np.array_equal(ud.cpu().numpy(), uv))
uh = np.zeros(16, np.uint8)
out["mixed_u8"] = run(ctypes.c_void_p(ud.data_ptr()), ctypes.c_void_p(uh.ctypes.data), 16, 1)
'''
    ini = ("[general]\nnum_workers = 2\nnum_worker_threads = 4\npacket_numel = 256\n"
           "max_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = bulk\n")
    out = run_driver(body, ini, preload="import torch")
    assert out["init"] == 0
    assert out["dev_size"] == 4 * 100_003 and out["dev_ok"]
    assert out["host_size"] == 4 * 100_003 and out["host_ok"]
    assert out["int_ok"]
    # device uint8 (RCCL hands device buffers, NCCL_PTR_CUDA): widened on the
    # GPU, all-reduced as INT32 (loopback: x2), narrowed mod 256 — :318-337, 370-378
    assert out["dev_u8"] == 1000 and out["dev_u8_ok"] and out["dev_u8_send_untouched"]
    assert out["mixed_u8"] == 4   # one device and one host buffer: ncclInvalidArgument


def test_loopback_collnet_needs_opt_in():
    """the loopback backend multiplies a rank's own buffer by
    num_workers, it does not sum across ranks — init() refuses
    (ncclInvalidUsage) unless SWITCHML_COLLNET_LOOPBACK=1."""
    ini = "[general]\nprepostprocessor = bypass\nnum_worker_threads = 2\n[backend.dummy]\nbandwidth = 0\n"
    code = (f"import ctypes, sys; sys.path[:0] = [{ROOT!r}, {os.path.join(ROOT, 'tests')!r}]\n"
            "from test_collnet_plugin import CollNetV6, LOGGER, PLUGIN\n"
            "tbl = CollNetV6.in_dll(ctypes.CDLL(PLUGIN), 'ncclCollNetPlugin_v6')\n"
            "print(tbl.init(LOGGER(lambda *a: None)))\n")
    env = dict(os.environ, SWITCHML_CONFIG_INI=ini)
    env.pop("SWITCHML_COLLNET_LOOPBACK", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "5"   # ncclInvalidUsage


class NetV6(ctypes.Structure):
    """nccl/net_v6.h ncclNet_v6_t (plugins/rccl_collnet/collnet_abi.h)."""
    _fields_ = [("name", ctypes.c_char_p), ("init", vp), ("devices", vp), ("getProperties", vp),
                ("listen", vp), ("connect", vp), ("accept", vp), ("regMr", vp), ("regMrDmaBuf", vp),
                ("deregMr", vp), ("isend", vp), ("irecv", vp), ("iflush", vp), ("test", vp),
                ("closeSend", vp), ("closeRecv", vp), ("closeListen", vp)]


# A stand-in underlying net plugin: every entry point records that it ran.
FAKE_NET = r"""
#include <stddef.h>
#include <stdint.h>
#include <string.h>
typedef int R;
static int calls[17];
int fake_calls(int i) { return calls[i]; }
static R init(void* l) { calls[1]++; return 0; }
static R devices(int* n) { calls[2]++; *n = 3; return 0; }
static R props(int d, void* p) { calls[3]++; return d == 7 ? 4 : 0; }
static R listen_(int d, void* h, void** c) { calls[4]++; memcpy(h, "FAKE", 4); *c = (void*)0x10; return 0; }
static R connect_(int d, void* h, void** c) { calls[5]++; *c = (void*)0x20; return 0; }
static R accept_(void* l, void** c) { calls[6]++; *c = (void*)0x30; return 0; }
static R regmr(void* c, void* d, int s, int t, void** m) { calls[7]++; *m = (void*)0x40; return 0; }
static R regdma(void* c, void* d, size_t s, int t, uint64_t o, int fd, void** m) { calls[8]++; return 0; }
static R dereg(void* c, void* m) { calls[9]++; return 0; }
static R isend(void* c, void* d, int s, int t, void* m, void** r) { calls[10]++; *r = (void*)0x50; return 0; }
static R irecv(void* c, int n, void** d, int* s, int* t, void** m, void** r) { calls[11]++; *r = (void*)0x60; return 0; }
static R iflush(void* c, int n, void** d, int* s, void** m, void** r) { calls[12]++; return 0; }
static R test(void* r, int* done, int* s) { calls[13]++; *done = 1; return 0; }
static R cs(void* c) { calls[14]++; return 0; }
static R cr(void* c) { calls[15]++; return 0; }
static R cl(void* c) { calls[16]++; return 0; }
struct { const char* name; void* f[16]; } ncclNetPlugin_v6 = {"FAKE", {
  (void*)init, (void*)devices, (void*)props, (void*)listen_, (void*)connect_, (void*)accept_, (void*)regmr,
  (void*)regdma, (void*)dereg, (void*)isend, (void*)irecv, (void*)iflush, (void*)test, (void*)cs, (void*)cr,
  (void*)cl}};
"""

NET_DRIVER = r"""
import ctypes, json, sys
sys.path[:0] = [{root!r}, {tests!r}]
from test_collnet_plugin import NetV6, PLUGIN, LOGGER, vp
lib = ctypes.CDLL(PLUGIN)
t = NetV6.in_dll(lib, "ncclNetPlugin_v6")
F = lambda name, *types: ctypes.CFUNCTYPE(ctypes.c_int, *types)(getattr(t, name))
P = ctypes.POINTER
out = {{"name": t.name.decode(), "init": F("init", LOGGER)(LOGGER(lambda *a: None))}}
if out["init"] == 0:
    n = ctypes.c_int(); out["devices"] = [F("devices", P(ctypes.c_int))(ctypes.byref(n)), n.value]
    out["props_bad"] = F("getProperties", ctypes.c_int, vp)(7, None)
    h = (ctypes.c_char * 128)(); lc, sc, rc, mh, rq = vp(), vp(), vp(), vp(), vp()
    out["listen"] = F("listen", ctypes.c_int, vp, P(vp))(0, ctypes.cast(h, vp), ctypes.byref(lc))
    out["handle"] = bytes(h[:4]).decode()
    out["connect"] = F("connect", ctypes.c_int, vp, P(vp))(0, ctypes.cast(h, vp), ctypes.byref(sc))
    out["accept"] = F("accept", vp, P(vp))(lc, ctypes.byref(rc))
    out["comms"] = [lc.value, sc.value, rc.value]
    F("regMr", vp, vp, ctypes.c_int, ctypes.c_int, P(vp))(sc, None, 4, 1, ctypes.byref(mh))
    F("isend", vp, vp, ctypes.c_int, ctypes.c_int, vp, P(vp))(sc, None, 4, 0, mh, ctypes.byref(rq))
    d = ctypes.c_int(0); sz = ctypes.c_int(0)
    out["test"] = [F("test", vp, P(ctypes.c_int), P(ctypes.c_int))(rq, ctypes.byref(d), ctypes.byref(sz)), d.value]
    F("deregMr", vp, vp)(sc, mh)
    for nm in ("closeSend", "closeRecv", "closeListen"):
        F(nm, vp)(None)
    fake = ctypes.CDLL({fake!r})
    out["fake_calls"] = [fake.fake_calls(i) for i in range(17)]
print(json.dumps(out))
"""


def test_net_table_forwards_to_underlying_plugin(tmp_path):
    """ncclNetPlugin_v6 (reference: switchml_plugin.cc:37, NCCL_PLUGIN_SYMBOL
    beside the CollNet table) with SWITCHML_NET_PLUGIN set: every call is
    forwarded to that underlying plugin."""
    fake = tmp_path / "libfake_net.so"
    src = tmp_path / "fake_net.c"
    src.write_text(FAKE_NET)
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", str(fake), str(src)], check=True)
    code = NET_DRIVER.format(root=ROOT, tests=os.path.join(ROOT, "tests"), fake=str(fake))
    env = dict(os.environ, SWITCHML_NET_PLUGIN=str(fake))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["name"] == "SWITCHML"
    assert out["init"] == 0
    assert out["devices"] == [0, 3] and out["props_bad"] == 4
    assert out["listen"] == 0 and out["handle"] == "FAKE"
    assert out["connect"] == 0 and out["accept"] == 0 and out["comms"] == [0x10, 0x20, 0x30]
    assert out["test"] == [0, 1]
    calls = out["fake_calls"]
    for i in (1, 2, 3, 4, 5, 6, 7, 9, 10, 13, 14, 15, 16):
        assert calls[i] >= 1, (i, calls)


# The built-in TCP net (plugins/rccl_collnet/socket_net.h), driven the way
# RCCL's net transport drives a v6 net: listen -> handle to the peer ->
# connect / accept (non-blocking: NULL comm means "call again") -> regMr ->
# isend / irecv -> test until done -> close.
SOCKET_DRIVER = r"""
import ctypes, json, os, sys, time
import numpy as np
sys.path[:0] = [{root!r}, {tests!r}]
from test_collnet_plugin import NetV6, PLUGIN, LOGGER, vp
t = NetV6.in_dll(ctypes.CDLL(PLUGIN), "ncclNetPlugin_v6")
P = ctypes.POINTER
F = lambda name, *types: ctypes.CFUNCTYPE(ctypes.c_int, *types)(getattr(t, name))
init, devices = F("init", LOGGER), F("devices", P(ctypes.c_int))
props = F("getProperties", ctypes.c_int, vp)
listen = F("listen", ctypes.c_int, vp, P(vp)); connect = F("connect", ctypes.c_int, vp, P(vp))
accept = F("accept", vp, P(vp)); regmr = F("regMr", vp, vp, ctypes.c_int, ctypes.c_int, P(vp))
dereg = F("deregMr", vp, vp)
isend = F("isend", vp, vp, ctypes.c_int, ctypes.c_int, vp, P(vp))
irecv = F("irecv", vp, ctypes.c_int, P(vp), P(ctypes.c_int), P(ctypes.c_int), P(vp), P(vp))
iflush = F("iflush", vp, ctypes.c_int, P(vp), P(ctypes.c_int), P(vp), P(vp))
test = F("test", vp, P(ctypes.c_int), P(ctypes.c_int))
close_s, close_r, close_l = F("closeSend", vp), F("closeRecv", vp), F("closeListen", vp)
keep_logger = LOGGER(lambda *a: None)   # the library calls it later (warnings)
out = {{"init": init(keep_logger)}}
n = ctypes.c_int(); devices(ctypes.byref(n)); out["ndev"] = n.value
class Props(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("pciPath", ctypes.c_char_p), ("guid", ctypes.c_uint64),
                ("ptrSupport", ctypes.c_int), ("speed", ctypes.c_int), ("port", ctypes.c_int),
                ("latency", ctypes.c_float), ("maxComms", ctypes.c_int), ("maxRecvs", ctypes.c_int)]
pr = Props(); out["props"] = props(0, ctypes.cast(ctypes.pointer(pr), vp))
out["pname"], out["ptr"], out["maxRecvs"] = pr.name.decode(), pr.ptrSupport, pr.maxRecvs
out["pci_null"] = pr.pciPath is None

def pair():
    h = (ctypes.c_char * 128)(); lc, sc, rc = vp(), vp(), vp()
    assert listen(0, ctypes.cast(h, vp), ctypes.byref(lc)) == 0
    assert accept(lc, ctypes.byref(rc)) == 0 and not rc.value      # nobody connected yet: call again
    assert connect(0, ctypes.cast(h, vp), ctypes.byref(sc)) == 0 and sc.value
    for _ in range(10000):
        assert accept(lc, ctypes.byref(rc)) == 0
        if rc.value: break
        time.sleep(0.0005)
    assert rc.value
    return lc, sc, rc

def wait(req):
    d, sz = ctypes.c_int(0), ctypes.c_int(-1)
    while not d.value:
        rc = test(req, ctypes.byref(d), ctypes.byref(sz))
        if rc: return ("err", rc)
    return sz.value

lc, sc, rc = pair()
mh = vp(); out["regmr_host"] = regmr(sc, None, 0, 1, ctypes.byref(mh)); out["regmr_cuda"] = regmr(sc, None, 0, 2, ctypes.byref(vp()))
rng = np.random.default_rng(7)
sizes = [0, 1, 7, 4096, 65536 + 3, 8 << 20, 123457]
msgs = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
bufs = [np.full(s + 100, 0xAB, dtype=np.uint8) for s in sizes]
sreqs, rreqs = [], []
for i, (m, b) in enumerate(zip(msgs, bufs)):        # all posted before any test: FIFO matching
    q = vp(); assert isend(sc, m.ctypes.data_as(vp), m.size, i, mh, ctypes.byref(q)) == 0 and q.value; sreqs.append(q)
    q = vp(); d = (vp * 1)(b.ctypes.data); s = (ctypes.c_int * 1)(b.size); tg = (ctypes.c_int * 1)(i)
    assert irecv(rc, 1, d, s, tg, (vp * 1)(None), ctypes.byref(q)) == 0 and q.value; rreqs.append(q)
got = []
for i in range(len(sizes)):    # drive both sides like the proxy: poll every request
    done_s = done_r = None
    while done_s is None or done_r is None:
        for which, q in (("s", sreqs[i]), ("r", rreqs[i])):
            if (which == "s" and done_s is not None) or (which == "r" and done_r is not None): continue
            d, sz = ctypes.c_int(0), ctypes.c_int(-1)
            assert test(q, ctypes.byref(d), ctypes.byref(sz)) == 0
            if d.value:
                if which == "s": done_s = sz.value
                else: done_r = sz.value
    got.append([done_s, done_r])
out["sizes"] = got
out["payload_ok"] = all(bool(np.array_equal(b[:m.size], m)) and bool((b[m.size:] == 0xAB).all())
                        for m, b in zip(msgs, bufs))
fq = vp(); out["iflush"] = [iflush(rc, 1, (vp * 1)(None), (ctypes.c_int * 1)(0), (vp * 1)(None), ctypes.byref(fq)), fq.value]
# a receive smaller than the message: an error, not a silent truncation
big = np.zeros(64, np.uint8); small = np.zeros(16, np.uint8)
q = vp(); isend(sc, big.ctypes.data_as(vp), 64, 0, mh, ctypes.byref(q))
r2 = vp(); irecv(rc, 1, (vp * 1)(small.ctypes.data), (ctypes.c_int * 1)(16), (ctypes.c_int * 1)(0), (vp * 1)(None), ctypes.byref(r2))
out["truncated"] = wait(r2)
dereg(sc, mh)
out["close"] = [close_s(sc), close_r(rc), close_l(lc)]
# a connector with another handle's nonce is dropped, the right one accepted
h1 = (ctypes.c_char * 128)(); h2 = (ctypes.c_char * 128)(); l1, l2 = vp(), vp()
listen(0, ctypes.cast(h1, vp), ctypes.byref(l1)); listen(0, ctypes.cast(h2, vp), ctypes.byref(l2))
forged = bytearray(bytes(h2)); forged[8:14] = bytes(h1)[8:14]       # l1's address, l2's nonce
fh = (ctypes.c_char * 128).from_buffer_copy(bytes(forged)); s_bad, s_ok, r1 = vp(), vp(), vp()
connect(0, ctypes.cast(fh, vp), ctypes.byref(s_bad)); connect(0, ctypes.cast(h1, vp), ctypes.byref(s_ok))
for _ in range(10000):
    accept(l1, ctypes.byref(r1))
    if r1.value: break
    time.sleep(0.0005)
x = np.arange(10, dtype=np.uint8); y = np.zeros(10, np.uint8)
q1, q2 = vp(), vp()
isend(s_ok, x.ctypes.data_as(vp), 10, 0, None, ctypes.byref(q1))
irecv(r1, 1, (vp * 1)(y.ctypes.data), (ctypes.c_int * 1)(10), (ctypes.c_int * 1)(0), (vp * 1)(None), ctypes.byref(q2))
out["nonce_check"] = [wait(q1), wait(q2), bool((x == y).all())]
out["bad_handle"] = connect(0, ctypes.cast((ctypes.c_char * 128)(), vp), ctypes.byref(vp()))
print(json.dumps(out))
"""


def test_builtin_socket_net():
    """Without SWITCHML_NET_PLUGIN the library's own TCP net serves RCCL
    (so RCCL keeps the paired CollNet table): non-blocking accept, FIFO
    matching of posted sends and receives across sizes 0 B .. 8 MiB, receive
    sizes reported by test(), no bytes past the message touched, a
    too-small receive fails, a connection presenting another handle's nonce
    is dropped, host pointers only."""
    code = SOCKET_DRIVER.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    env = dict(os.environ)
    env.pop("SWITCHML_NET_PLUGIN", None)
    env["SWITCHML_NET_IFADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["init"] == 0 and out["ndev"] == 1 and out["props"] == 0
    assert out["pname"] == "SWITCHML" and out["ptr"] == 1 and out["maxRecvs"] == 1 and out["pci_null"]
    assert out["regmr_host"] == 0 and out["regmr_cuda"] != 0
    sizes = [0, 1, 7, 4096, 65536 + 3, 8 << 20, 123457]
    assert out["sizes"] == [[s, s] for s in sizes]
    assert out["payload_ok"]
    assert out["iflush"] == [0, None]
    assert out["truncated"] == ["err", 3]
    assert out["close"] == [0, 0, 0]
    assert out["nonce_check"] == [10, 10, True]
    assert out["bad_handle"] == 4


RESNET50_BUCKETS = [6_553_600, 6_553_600, 6_553_600, 5_896_232]   # 25 MiB DDP buckets of 25,557,032 params

CFG4_DRIVER = r"""
import json, sys
import numpy as np
import torch
sys.path[:0] = [{root!r}, {pkg!r}]
from oracle import oracle as O
from switchml_amd.collnet import CollNetComm, NCCL_FLOAT32
sizes = {sizes!r}
comm = CollNetComm()
xs = [O.splitmix_normal(50 + i, n) * np.float32(1e-3) for i, n in enumerate(sizes)]
refs = [O.dummy_allreduce(x, P=256, max_outstanding_packets=256, num_worker_threads=4, num_workers=8,
                          threaded=True) for x in xs]
out = {{"ptrSupport": comm.props.ptrSupport}}
# device buffers, not in place: RCCL's send / recv buffers
dsend = [torch.from_numpy(x).cuda() for x in xs]
drecv = [torch.empty_like(d) for d in dsend]
mhs = [comm.reg_mr(d.data_ptr(), 4 * d.numel(), 2) for d in dsend]
sz = comm.allreduce_buckets([(s.data_ptr(), r.data_ptr(), s.numel()) for s, r in zip(dsend, drecv)], NCCL_FLOAT32, mhs)
out["device_sizes"] = sz
out["device_ok"] = [bool(np.array_equal(r.cpu().numpy().view(np.uint32), ref.view(np.uint32)))
                    for r, ref in zip(drecv, refs)]
out["device_send_untouched"] = all(bool(np.array_equal(s.cpu().numpy(), x)) for s, x in zip(dsend, xs))
for m in mhs:
    comm.dereg_mr(m)
# pinned host buffers, in place (what the reference's NCCL_PTR_HOST plugin is handed)
hb = [torch.from_numpy(x.copy()).pin_memory() for x in xs]
sz = comm.allreduce_buckets([(h.data_ptr(), h.data_ptr(), h.numel()) for h in hb], NCCL_FLOAT32)
out["host_sizes"] = sz
out["host_ok"] = [bool(np.array_equal(h.numpy().view(np.uint32), ref.view(np.uint32))) for h, ref in zip(hb, refs)]
comm.close()
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_configs4_resnet50_buckets_through_plugin(cuda):
    """configs[4]: ResNet-50-sized gradient buckets (DDP's 25 MiB buckets:
    3 x 6,553,600 + 5,896,232 fp32; sizes not in the reference, so
    parity-unpinned as a workload) posted to the plugin's iallreduce and
    polled with test() — switchml_plugin.cc:293-387 — on device buffers
    (send != recv) and on pinned host buffers (in place), W = 8, T = 4,
    P = 256; every bucket bit-exact against the oracle's dummy packet loop."""
    code = CFG4_DRIVER.format(root=ROOT, pkg=os.path.join(ROOT, "p4app-switchml_amd"), sizes=RESNET50_BUCKETS)
    ini = ("[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\n"
           "max_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\n")
    env = dict(os.environ, SWITCHML_CONFIG_INI=ini, SWITCHML_COLLNET_LOOPBACK="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ptrSupport"] == 3
    assert out["device_sizes"] == [4 * n for n in RESNET50_BUCKETS]
    assert all(out["device_ok"]) and out["device_send_untouched"]
    assert out["host_sizes"] == [4 * n for n in RESNET50_BUCKETS]
    assert all(out["host_ok"])


@pytest.mark.gpu
def test_configs4_native_proxy_driver(cuda):
    """bin/collnet_bench: the CollNet table driven from native code in RCCL's
    proxy call order (dlopen, init, listen/connect, regMr, iallreduce x 4
    buckets, test until done) on device and pinned host buffers; every test()
    reports the bucket's byte size and both placements give the same bytes."""
    import json
    ini = ("[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\n"
           "max_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\n")
    env = dict(os.environ, SWITCHML_CONFIG_INI=ini, SWITCHML_COLLNET_LOOPBACK="1")
    exe = os.path.join(ROOT, "p4app-switchml_amd", "bin", "collnet_bench")
    r = subprocess.run([exe, "3", PLUGIN], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["placements_agree"] is True
    assert out["params"] == sum(RESNET50_BUCKETS)
