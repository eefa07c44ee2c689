"""The multi-process result collector (tests/mp_ranks.py), on CPU: a failing
rank ends the wait at once even while its peer blocks, a rank that dies
without a result is named, and healthy ranks all report."""
import os
import time

import pytest
import torch.multiprocessing as mp

from mp_ranks import collect


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
