"""Result collection for the multi-process tests (one process per rank).

A rank that fails reports at once and its peers are not waited for: they
are usually blocked in a collective on the failed rank and would otherwise
hold the test until its timeout, silently.  A rank that dies without
reporting (a crash, an abort) is noticed from its exit code.  While waiting,
a heartbeat line goes to stderr every 20 s so a slow run is not mistaken
for a hung one, and ranks still alive at the end are terminated."""
import queue
import sys
import time


def collect(q, procs, timeout=240, what="ranks"):
    """Return the list of per-rank result tuples (rank, ok_or_result, err),
    in arrival order.  Raises AssertionError naming the failing rank, a rank
    that exited without a result, or the ranks missing at the timeout."""
    res = []
    t0 = time.monotonic()
    last_beat = t0
    failed = None
    try:
        while len(res) < len(procs):
            now = time.monotonic()
            if now - t0 > timeout:
                break
            try:
                r = q.get(timeout=min(2.0, max(0.1, timeout - (now - t0))))
            except queue.Empty:
                if now - last_beat >= 20:
                    print(f"[mp_ranks] {what}: {len(res)}/{len(procs)} reported after {now - t0:.0f} s",
                          file=sys.stderr, flush=True)
                    last_beat = now
                done = {x[0] for x in res}
                dead = [i for i, p in enumerate(procs) if i not in done and p.exitcode not in (None, 0)]
                if dead:
                    # give a just-exited rank's queued result a moment to arrive
                    try:
                        res.append(q.get(timeout=2.0))
                        continue
                    except queue.Empty:
                        raise AssertionError(f"{what}: rank(s) {dead} exited with "
                                             f"{[procs[i].exitcode for i in dead]} and no result")
                continue
            res.append(r)
            if len(r) == 3 and (r[1] is None or r[1] is False):   # (rank, result-or-ok, error text)
                failed = r
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
