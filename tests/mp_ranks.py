"""Rank processes for the multi-process tests (one process per rank).

* Rendezvous through a FileStore in a fresh directory (`init_method=file://`):
  no TCP port is picked by the parent and handed to the ranks later, so no
  other process can take it in between (the bind-close-reuse race of the
  old `_free_port()`).
* Every rank arms faulthandler: a crash prints its Python stack, and a rank
  still running at its deadline dumps the stacks of all its threads — the
  call it is blocked in — and exits, so a hang names itself instead of
  printing nothing.  The deadline is below the parent's, so the parent sees
  the death and reports it.
* A rank's result is flushed through the queue (put, close, join the feeder
  thread) before any teardown, so a crash in teardown cannot lose it.
* The parent (`collect`) stops waiting at the first failing or dead rank —
  its peers, blocked in a collective on it, would otherwise hold the test
  until the timeout — prints a heartbeat every 20 s (past pytest's capture)
  so a slow run is not mistaken for a hung one, and terminates the ranks still alive at the end."""
import faulthandler
import os
import queue
import shutil
import sys
import tempfile
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAPTURE_MANAGER = None   # set by conftest.py: pytest's capture manager


def heartbeat(msg: str) -> None:
    """One progress line on the real stderr, past pytest's output capture
    (captured output appears only when a test ends; a long test that prints
    nothing visible would look hung to whoever watches the run)."""
    line = f"[mp_ranks] {msg}\n"
    cm = CAPTURE_MANAGER
    if cm is not None:
        with cm.global_and_fixture_disabled():
            sys.stderr.write(line)
            sys.stderr.flush()
    else:
        sys.stderr.write(line)
        sys.stderr.flush()


def _failed(r) -> bool:
    return len(r) == 3 and (r[1] is None or r[1] is False)   # (rank, result-or-ok, error text)


def collect(q, procs, timeout=240, what="ranks"):
    """Return the list of per-rank result tuples (rank, ok_or_result, err),
    in arrival order.  Raises AssertionError naming the failing rank, a rank
    that exited without a result, or the ranks missing at the timeout."""
    res = []
    t0 = time.monotonic()
    last_beat = t0
    failed = None

    def take(r):
        nonlocal failed
        res.append(r)
        if _failed(r):
            failed = r
        return failed is not None

    try:
        while len(res) < len(procs):
            now = time.monotonic()
            if now - t0 > timeout:
                break
            try:
                r = q.get(timeout=min(2.0, max(0.1, timeout - (now - t0))))
            except queue.Empty:
                if now - last_beat >= 20:
                    heartbeat(f"{what}: {len(res)}/{len(procs)} reported after {now - t0:.0f} s")
                    last_beat = now
                done = {x[0] for x in res}
                dead = [i for i, p in enumerate(procs) if i not in done and p.exitcode not in (None, 0)]
                if dead:
                    # give a just-exited rank's queued result a moment to arrive
                    try:
                        if take(q.get(timeout=2.0)):
                            break
                        continue
                    except queue.Empty:
                        raise AssertionError(f"{what}: rank(s) {dead} exited with "
                                             f"{[procs[i].exitcode for i in dead]} and no result "
                                             "(its stack, if it hung or crashed, is on stderr above)")
                continue
            if take(r):
                break
    finally:
        for p in procs:
            p.join(timeout=30 if failed is None and len(res) == len(procs) else 3)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
                if p.is_alive():
                    p.kill()
                    p.join(timeout=5)
    if failed is not None:
        raise AssertionError(f"{what}: rank {failed[0]} failed: {failed[2]}")
    missing = sorted(set(range(len(procs))) - {x[0] for x in res})
    assert not missing, f"{what}: no result from rank(s) {missing} within {timeout} s"
    return res


def report(q, item):
    """Put one result and wait until the queue's feeder thread has written it
    to the pipe: what follows (teardown, interpreter exit) cannot lose it."""
    try:
        q.put(item)
        q.close()
        q.join_thread()
    except (ValueError, OSError):   # already reported and closed
        pass


def init_pg(backend, init, rank, world, device_id=None, timeout_s=120.0):
    """init_process_group over the FileStore `init`; a rank blocked on a
    failed peer raises after timeout_s instead of gloo's 30 / RCCL's 10 min."""
    import datetime

    import torch.distributed as dist
    kw = {"device_id": device_id} if device_id is not None else {}
    dist.init_process_group(backend, init_method=init, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return dist


def rank_entry(body, rank, world, init, q, deadline_s, args):
    """Target of every rank process: `body(rank, world, init, *args)` runs
    under faulthandler's deadline; its return value (or the traceback) is
    reported; the default process group, if the body left one, is destroyed
    only after that."""
    for p in (ROOT, os.path.join(ROOT, "p4app-switchml_amd"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    faulthandler.enable()
    faulthandler.dump_traceback_later(deadline_s, exit=True)
    try:
        item = (rank, body(rank, world, init, *args), "")
    except BaseException:  # noqa: BLE001 - reported to the parent
        item = (rank, None, traceback.format_exc()[-2000:])
    report(q, item)
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - the result is already out
        pass


def spawn(body, world, args=(), timeout=240, what="ranks", deadline=None):
    """Run `body` in `world` fresh spawned processes, rendezvous through a
    FileStore in a new temporary directory; return collect()'s results.
    `deadline`: seconds after which a rank still running dumps its stacks
    and exits (default: 20 s before the parent's `timeout`)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    d = tempfile.mkdtemp(prefix="sml_pg_")
    init = "file://" + os.path.join(d, "store")
    if deadline is None:
        deadline = max(20.0, timeout - 20.0)
    procs = [ctx.Process(target=rank_entry, args=(body, r, world, init, q, deadline, tuple(args)))
             for r in range(world)]
    try:
        for p in procs:
            p.start()
        return collect(q, procs, timeout=timeout, what=what)
    finally:
        shutil.rmtree(d, ignore_errors=True)
