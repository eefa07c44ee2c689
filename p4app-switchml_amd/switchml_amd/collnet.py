"""ctypes driver of the RCCL CollNet plugin (librccl-net-switchml.so).

Calls the exported ncclCollNetPlugin_v6 table the way RCCL's proxy thread
does (init -> devices -> getProperties -> listen -> connect -> regMr ->
iallreduce -> test ... -> deregMr -> closeColl -> closeListen), so tests and
bench.py can run configs[4] — framework gradient buckets handed to the
plugin — without a multi-node CollNet topology (RCCL itself enables CollNet
only across nodes).  Reference: frameworks_integration/nccl_plugin/
switchml_plugin.cc:135-402.

Load torch (if used) before this module's library: torch bundles its own
libamdhip64.so.7 with the same SONAME as /opt/rocm's.
"""
from __future__ import annotations

import ctypes
import os

from . import _HERE

PLUGIN_PATH = os.path.join(_HERE, "librccl-net-switchml.so")

R = ctypes.c_int
vp = ctypes.c_void_p
LOGGER = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p)

# ncclDataType_t / ncclRedOp_t values (nccl.h)
NCCL_UINT8, NCCL_INT32, NCCL_FLOAT32, NCCL_FLOAT64 = 1, 2, 7, 8
NCCL_SUM, NCCL_MAX = 0, 2


class Props(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("pciPath", ctypes.c_char_p), ("guid", ctypes.c_uint64),
                ("ptrSupport", ctypes.c_int), ("speed", ctypes.c_int), ("port", ctypes.c_int),
                ("latency", ctypes.c_float), ("maxComms", ctypes.c_int), ("maxRecvs", ctypes.c_int)]


class CollNetV6(ctypes.Structure):
    """nccl/net_v6.h ncclCollNet_v6_t (plugins/rccl_collnet/collnet_abi.h)."""
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


class CollNetError(RuntimeError):
    pass


def _ok(rc, what):
    if rc != 0:
        raise CollNetError(f"{what} returned ncclResult_t {rc}")


class CollNetComm:
    """One CollNet communicator of `nranks` ranks (this process = `rank`),
    set up through the plugin table like RCCL's proxy does."""

    def __init__(self, nranks: int = 1, rank: int = 0, path: str = PLUGIN_PATH):
        self.lib = ctypes.CDLL(path)
        self.tbl = CollNetV6.in_dll(self.lib, "ncclCollNetPlugin_v6")
        self._logger = LOGGER(lambda *a: None)
        _ok(self.tbl.init(self._logger), "init")
        n = ctypes.c_int()
        _ok(self.tbl.devices(ctypes.byref(n)), "devices")
        self.props = Props()
        _ok(self.tbl.getProperties(0, ctypes.byref(self.props)), "getProperties")
        self._handle = (ctypes.c_char * 128)()
        self.lcomm = vp()
        _ok(self.tbl.listen(0, ctypes.cast(self._handle, vp), ctypes.byref(self.lcomm)), "listen")
        handles = (vp * nranks)(*([ctypes.cast(self._handle, vp).value] * nranks))
        self.coll = vp()
        _ok(self.tbl.connect(handles, nranks, rank, self.lcomm, ctypes.byref(self.coll)), "connect")

    def reg_mr(self, ptr: int, nbytes: int, type_: int = 1):
        mh = vp()
        _ok(self.tbl.regMr(self.coll, vp(ptr), nbytes, type_, ctypes.byref(mh)), "regMr")
        return mh

    def dereg_mr(self, mh):
        _ok(self.tbl.deregMr(self.coll, mh), "deregMr")

    def iallreduce(self, send: int, recv: int, count: int, dtype: int = NCCL_FLOAT32, mh=None):
        req = vp()
        _ok(self.tbl.iallreduce(self.coll, vp(send), vp(recv), count, dtype, NCCL_SUM, mh, mh, ctypes.byref(req)),
            "iallreduce")
        return req

    def test(self, req) -> tuple[bool, int]:
        done, size = ctypes.c_int(0), ctypes.c_int(0)
        _ok(self.tbl.test(req, ctypes.byref(done), ctypes.byref(size)), "test")
        return bool(done.value), size.value

    def wait(self, req) -> int:
        while True:
            done, size = self.test(req)
            if done:
                return size

    def allreduce_buckets(self, buckets, dtype: int = NCCL_FLOAT32, mhs=None) -> list[int]:
        """Post every bucket's iallreduce, then poll them (RCCL's proxy keeps
        several requests in flight); buckets = [(send_ptr, recv_ptr, count)].
        As with RCCL's proxy, the buffers must be ready when posted (their
        producing stream synchronized): the plugin's worker streams do not
        order after the caller's."""
        reqs = [self.iallreduce(s, r, c, dtype, None if mhs is None else mhs[i])
                for i, (s, r, c) in enumerate(buckets)]
        return [self.wait(q) for q in reqs]

    def close(self):
        if self.coll:
            _ok(self.tbl.closeColl(self.coll), "closeColl")
            self.coll = None
        if self.lcomm:
            _ok(self.tbl.closeListen(self.lcomm), "closeListen")
            self.lcomm = None
