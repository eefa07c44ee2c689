"""ctypes binding of include/switchml_client.h — the SwitchML Context
(Start / Stop / AllReduceAsync / AllReduce / WaitForAllJobs, Job status) of
the MI355X client library.  Mirrors the C++ API of
client_lib/src/context.h:76-155; used by tests and as the reference-shaped
entry point for Python callers (host numpy arrays or torch CUDA tensors).
"""
from __future__ import annotations

import ctypes

from . import lib as _kernel_lib

CREATED, STARTING, RUNNING, STOPPING, STOPPED = range(5)
JOB_INIT, JOB_QUEUED, JOB_RUNNING, JOB_FINISHED, JOB_FAILED = range(5)
FLOAT32, INT32 = 0, 1
SUM = 0

_bound = False


def _lib():
    global _bound
    L = _kernel_lib()
    if not _bound:
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.sml_context_start.restype = i32
        L.sml_context_start.argtypes = [ctypes.c_char_p]
        L.sml_context_stop.restype = i32
        L.sml_context_state.restype = i32
        L.sml_context_last_error.restype = ctypes.c_char_p
        L.sml_context_config.restype = ctypes.c_char_p
        L.sml_allreduce_async.restype = i32
        L.sml_allreduce_async.argtypes = [vp, vp, u64, i32, i32, ctypes.POINTER(vp)]
        L.sml_allreduce.restype = i32
        L.sml_allreduce.argtypes = [vp, vp, u64, i32, i32]
        L.sml_wait_for_all_jobs.restype = i32
        L.sml_job_wait.restype = i32
        L.sml_job_wait.argtypes = [vp]
        L.sml_job_status.restype = i32
        L.sml_job_status.argtypes = [vp]
        L.sml_job_id.restype = u64
        L.sml_job_id.argtypes = [vp]
        L.sml_job_release.argtypes = [vp]
        L.sml_context_stats.restype = i32
        L.sml_context_stats.argtypes = [vp]
        L.sml_ppp_per_ltu_calls.restype = i32
        L.sml_ppp_per_ltu_calls.argtypes = [ctypes.c_char_p]
        _bound = True
    return L


class ContextError(RuntimeError):
    pass


def _ok(rc, what):
    if rc != 0:
        raise ContextError(f"{what} failed ({rc}): {_lib().sml_context_last_error().decode()}")


def make_config(**kw) -> str:
    """INI text from keyword overrides, e.g. num_workers=2, mode='fused'."""
    general = {k: v for k, v in kw.items() if k in (
        "rank", "num_workers", "num_worker_threads", "max_outstanding_packets", "packet_numel",
        "backend", "scheduler", "prepostprocessor", "instant_job_completion")}
    dummy = {k: v for k, v in kw.items() if k in ("bandwidth", "process_packets", "fail_worker_thread",
                                                  "stall_worker_thread", "stall_ms")}
    hip = {k: v for k, v in kw.items() if k in ("device", "mode", "packet_ring", "burst_server", "batch_jobs",
                                                     "coalesce_us", "vcl")}
    xgmi = {k: v for k, v in kw.items() if k in ("session", "max_slice_numel", "timeout_ms", "push", "fail_setup")}
    unknown = set(kw) - set(general) - set(dummy) - set(hip) - set(xgmi)
    if unknown:
        raise KeyError(f"unknown config keys {sorted(unknown)}")

    def fmt(v):
        return ("true" if v else "false") if isinstance(v, bool) else str(v)
    out = "[general]\n" + "".join(f"{k} = {fmt(v)}\n" for k, v in general.items())
    out += "[backend.dummy]\n" + "".join(f"{k} = {fmt(v)}\n" for k, v in dummy.items())
    out += "[backend.hip]\n" + "".join(f"{k} = {fmt(v)}\n" for k, v in hip.items())
    out += "[backend.xgmi]\n" + "".join(f"{k} = {fmt(v)}\n" for k, v in xgmi.items())
    return out


def start(config_ini: str | None = None):
    _ok(_lib().sml_context_start(None if config_ini is None else config_ini.encode()), "sml_context_start")


def stop():
    _ok(_lib().sml_context_stop(), "sml_context_stop")


def state() -> int:
    return _lib().sml_context_state()


def config_text() -> str:
    return _lib().sml_context_config().decode()


def _ptr(t):
    if hasattr(t, "data_ptr"):          # torch tensor (host or device)
        return ctypes.c_void_p(t.data_ptr())
    return ctypes.c_void_p(t.ctypes.data)  # numpy array


def _dtype_of(t):
    s = str(t.dtype)
    if s.endswith("float32"):
        return FLOAT32
    if s.endswith("int32"):
        return INT32
    raise TypeError(f"unsupported dtype {t.dtype}")


class Job:
    def __init__(self, handle):
        self._h = handle

    @property
    def id(self) -> int:
        return int(_lib().sml_job_id(self._h))

    def status(self) -> int:
        return _lib().sml_job_status(self._h)

    def wait(self):
        _ok(_lib().sml_job_wait(self._h), "sml_job_wait")
        return self

    def __del__(self):
        if getattr(self, "_h", None):
            _lib().sml_job_release(self._h)
            self._h = None


def _ready(*tensors):
    """The Context takes plain pointers and runs on its own non-blocking HIP
    streams, so — like the reference's ProcessGroupSML, which synchronizes
    the producing stream before AllReduceAsync (ProcessGroupSML.cpp:137-151)
    — device (or pinned host) torch tensors are made ready first: the
    current stream's pending kernels may still write the input, or read a
    freed block the caching allocator has handed out again as the output.
    Every device involved is waited for: each CUDA tensor's own
    device, and for pinned host tensors the current device, whose stream is
    the one torch produces them on."""
    import torch
    devices = set()
    for t in tensors:
        if getattr(t, "is_cuda", False):
            devices.add(t.device.index if t.device.index is not None else torch.cuda.current_device())
        elif hasattr(t, "is_pinned") and t.is_pinned():
            devices.add(torch.cuda.current_device())
    for d in sorted(devices):
        torch.cuda.current_stream(d).synchronize()


def allreduce_async(inp, out=None, numel: int | None = None) -> Job:
    out = inp if out is None else out
    _ready(inp, out)
    n = inp.numel() if numel is None and hasattr(inp, "numel") and callable(inp.numel) else (
        inp.size if numel is None else numel)
    h = ctypes.c_void_p()
    _ok(_lib().sml_allreduce_async(_ptr(inp), _ptr(out), n, _dtype_of(inp), SUM, ctypes.byref(h)),
        "sml_allreduce_async")
    return Job(h)


def allreduce(inp, out=None):
    return allreduce_async(inp, out).wait()


def wait_for_all_jobs():
    _ok(_lib().sml_wait_for_all_jobs(), "sml_wait_for_all_jobs")


def stats() -> dict:
    arr = (ctypes.c_uint64 * 5)()
    _ok(_lib().sml_context_stats(ctypes.cast(arr, ctypes.c_void_p)), "sml_context_stats")
    return dict(zip(("jobs_submitted", "jobs_finished", "numel_submitted", "slices", "packets"), list(arr)))


def ppp_per_ltu_calls(name: str) -> bool:
    """Whether the prepostprocessor `name` takes per-packet PreprocessSingle /
    PostprocessSingle calls (sml_ppp_per_ltu_calls); ContextError for a name
    the factory rejects."""
    rc = _lib().sml_ppp_per_ltu_calls(name.encode())
    _ok(min(rc, 0), "sml_ppp_per_ltu_calls")
    return rc == 1
