"""The multi-process result collector (tests/mp_ranks.py), on CPU: a failing
rank ends the wait at once even while its peer blocks, a rank that dies
without a result is named, and healthy ranks all report."""
import os
import time

import pytest
import torch.multiprocessing as mp

from mp_ranks import collect, spawn


def _rank(rank, mode, q):
    if mode == "ok":
        q.put((rank, True, ""))
    elif mode == "fail":
        q.put((rank, None, "boom"))
    elif mode == "block":
        time.sleep(600)          # a peer stuck in a collective
    elif mode == "die":
        os._exit(3)


def _start(modes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, m, q)) for r, m in enumerate(modes)]
    for p in procs:
        p.start()
    return q, procs


def test_all_ranks_report():
    q, procs = _start(["ok", "ok", "ok"])
    res = collect(q, procs, timeout=60)
    assert sorted(r[0] for r in res) == [0, 1, 2]


def test_failure_ends_the_wait_while_a_peer_blocks():
    q, procs = _start(["block", "fail"])
    t0 = time.monotonic()
    with pytest.raises(AssertionError, match="rank 1 failed: boom"):
        collect(q, procs, timeout=120)
    assert time.monotonic() - t0 < 60
    assert not any(p.is_alive() for p in procs)


def test_dead_rank_without_result_is_named():
    q, procs = _start(["ok", "die"])
    with pytest.raises(AssertionError, match=r"rank\(s\) \[1\] exited with \[3\]"):
        collect(q, procs, timeout=120)


class _FakeQueue:
    """get() times out once, then yields the queued items (a result that
    arrives only after its rank has already exited)."""

    def __init__(self, items):
        self.items, self.first = list(items), True

    def get(self, timeout=None):
        import queue
        if self.first or not self.items:
            self.first = False
            raise queue.Empty
        return self.items.pop(0)


class _FakeProc:
    def __init__(self, exitcode):
        self.exitcode = exitcode

    def join(self, timeout=None):
        pass

    def is_alive(self):
        return self.exitcode is None

    def terminate(self):
        self.exitcode = -15


def test_failure_found_after_a_rank_died_ends_the_wait():
    """a failing result picked up in the dead-rank branch ends the
    wait like one from the main path (its peer, alive, is not waited for)."""
    q = _FakeQueue([(1, None, "late boom")])
    procs = [_FakeProc(None), _FakeProc(7)]
    t0 = time.monotonic()
    with pytest.raises(AssertionError, match="rank 1 failed: late boom"):
        collect(q, procs, timeout=30)
    assert time.monotonic() - t0 < 10


def _body_ok(rank, world, init):
    from mp_ranks import init_pg
    import torch
    dist = init_pg("gloo", init, rank, world)
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    return int(t.item())


def test_spawn_file_rendezvous():
    """Ranks meet through a FileStore in a fresh directory (no TCP port is
    chosen by the parent): gloo all_reduce over it."""
    res = spawn(_body_ok, 3, timeout=120)
    assert sorted(r[0] for r in res) == [0, 1, 2]
    assert all(r[1] == 6 for r in res)


def _body_hang(rank, world, init):
    if rank == 1:
        time.sleep(600)          # blocked past the rank deadline
    return True


def test_hung_rank_dumps_its_stack_and_is_named():
    """A rank still running at its deadline dumps every thread's stack
    (faulthandler) and exits: the parent names it within seconds of the
    deadline instead of waiting out its own timeout."""
    t0 = time.monotonic()
    with pytest.raises(AssertionError, match=r"rank\(s\) \[1\] exited with \[1\]"):
        spawn(_body_hang, 2, timeout=120, deadline=15)
    assert time.monotonic() - t0 < 60
