"""The CollNet plugin's cross-worker job order (plugins/rccl_collnet/
job_order.h): RCCL's proxy posts the CollNet chunks of its channels as each
channel's data arrives, so two workers interleave channels differently; the
switch pairs jobs by submission order, so worker 0's arrival order is logged
in shared memory and every other worker submits in that order.

CPU: job_order.cc compiled with a small driver; W worker processes get the
same calls — one sequence per "channel" — interleaved in a different random
order each, submit them through the log, and must all produce worker 0's
order; a segment left by a dead creator is replaced; a live one is refused;
a poisoned order is seen by every worker."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "p4app-switchml_amd", "plugins", "rccl_collnet")

DRIVER = r"""
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <random>
#include <string>
#include <vector>
#include "job_order.h"
using namespace sml_collnet;

// worker `rank`: channels c = 0..C-1, each with N calls (buf = c, seq = 0..N-1),
// arriving interleaved in a random order (per-channel order kept, as RCCL's
// proxy does); submit through the job order; print the submitted keys.
int worker(const char* session, int rank, int W, int C, int N, unsigned seed) {
    JobOrder order(session, rank, W, 20000);
    std::mt19937 rng(seed);
    std::vector<int> next(C, 0);
    std::deque<CallKey> pending;
    std::vector<CallKey> submitted;
    int arrived = 0;
    while ((int)submitted.size() < C * N) {
        if (arrived < C * N) {                       // one more call arrives
            int c;
            do c = rng() % C; while (next[c] == N);
            pending.push_back(CallKey{0, (uint32_t)c, (uint64_t)next[c]++, 1000 + c, 7, 0});
            arrived++;
        }
        if (order.leader()) {
            while (!pending.empty() && order.Append(pending.front())) {
                submitted.push_back(pending.front());
                pending.pop_front();
            }
        } else {
            CallKey k;
            while (order.Peek(&k)) {
                auto it = pending.begin();
                for (; it != pending.end(); ++it)
                    if (it->comm == k.comm && it->buf == k.buf && it->seq == k.seq) break;
                if (it == pending.end()) break;
                if (it->count != k.count) { fprintf(stderr, "count mismatch\n"); return 2; }
                submitted.push_back(*it);
                pending.erase(it);
                order.Consume();
            }
        }
        if (arrived == C * N && (int)submitted.size() < C * N) usleep(50);
    }
    std::string s;
    for (auto& k : submitted) s += std::to_string(k.buf) + ":" + std::to_string(k.seq) + ",";
    FILE* f = fopen((std::string(getenv("ORDER_OUT")) + "/r" + std::to_string(rank)).c_str(), "w");
    fprintf(f, "%s\n", s.c_str());
    fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    const std::string mode = argv[1];
    const char* session = argv[2];
    if (mode == "order") {
        int W = atoi(argv[3]), C = atoi(argv[4]), N = atoi(argv[5]);
        std::vector<pid_t> kids;
        for (int r = W - 1; r >= 0; r--) {          // followers start first: they must wait for worker 0
            pid_t p = fork();
            if (p == 0) { fflush(stdout); _exit(worker(session, r, W, C, N, 1234 + 77 * r)); }
            kids.push_back(p);
        }
        int bad = 0;
        for (pid_t p : kids) { int st; waitpid(p, &st, 0); bad |= !WIFEXITED(st) || WEXITSTATUS(st); }
        return bad;
    }
    if (mode == "leader") {                          // create, report, exit without cleanup (a crash)
        JobOrder* o = new JobOrder(session, 0, 2, 5000);
        printf("created\n");
        fflush(stdout);
        if (argc > 3) { sleep(atoi(argv[3])); }
        _exit(0);
        (void)o;
    }
    if (mode == "poison") {
        pid_t p = fork();
        if (p == 0) { JobOrder o(session, 1, 2, 20000); while (!o.Poisoned()) usleep(100); printf("follower saw poison\n"); fflush(stdout); _exit(0); }
        JobOrder o(session, 0, 2, 20000);
        o.Poison();
        int st; waitpid(p, &st, 0);
        return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
    }
    if (mode == "reconnect") {
        // worker 1 closes its communicator and reconnects at once, while
        // worker 0 still holds the first one open; then worker 0 closes and
        // reconnects in the same process.  Worker 1 must follow the SECOND
        // order (keys of communicator 1), not the first one's log.
        pid_t p = fork();
        if (p == 0) {
            {
                JobOrder a(session, 1, 2, 20000);
                CallKey k;
                while (!a.Peek(&k)) usleep(100);
                a.Consume();
            }
            CallKey k;
            {
                JobOrder b(session, 1, 2, 20000);
                while (!b.Peek(&k)) usleep(100);
                b.Consume();
            }
            printf("follower second order starts with comm %u\n", k.comm);
            fflush(stdout);
            _exit(k.comm == 1 ? 0 : 5);
        }
        {
            JobOrder a(session, 0, 2, 20000);
            a.Append(CallKey{0, 0, 0, 1, 7, 0});
            usleep(300000);                          // still open while worker 1 reconnects
        }
        JobOrder b(session, 0, 2, 20000);            // same process, same session
        b.Append(CallKey{1, 0, 0, 1, 7, 0});
        int st;
        waitpid(p, &st, 0);
        return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
    }
    if (mode == "late_detach") {
        // ADVICE r4: worker 1 detaches from communicator A AFTER worker 0 has
        // closed A and created B under the same session.  Only worker 0
        // removes the name, so B's segment survives and a fresh worker 1
        // joins B; when worker 0 closes B, the name is gone.
        int to_child[2], to_parent[2];
        if (pipe(to_child) || pipe(to_parent)) return 9;
        char c;
        pid_t p = fork();
        if (p == 0) {
            {
                JobOrder a(session, 1, 2, 20000);
                if (write(to_parent[1], "a", 1) != 1) _exit(8);
                if (read(to_child[0], &c, 1) != 1) _exit(8);     // B exists now
            }                                                // late detach from A
            if (write(to_parent[1], "d", 1) != 1) _exit(8);
            _exit(0);
        }
        int st;
        {
            JobOrder a(session, 0, 2, 20000);
            if (read(to_parent[0], &c, 1) != 1) return 7;   // worker 1 attached to A
        }
        JobOrder* b = new JobOrder(session, 0, 2, 20000);
        if (write(to_child[1], "b", 1) != 1) return 7;
        if (read(to_parent[0], &c, 1) != 1) return 7;       // worker 1 detached from A
        waitpid(p, &st, 0);
        pid_t q = fork();
        if (q == 0) {
            try { { JobOrder j(session, 1, 2, 2000); printf("joined B\n"); fflush(stdout); } _exit(0); }
            catch (const std::exception& e) { printf("lost B: %s\n", e.what()); fflush(stdout); _exit(6); }
        }
        waitpid(q, &st, 0);
        delete b;
        return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
    }
    if (mode == "churn") {
        // ADVICE r4 under load: K communicators in a row under one session.
        // Worker 1 takes communicator k's key, says so, and closes at once;
        // worker 0 closes comm k on that word and creates comm k + 1 — so
        // worker 1's detach of k (possibly the last one, which removes the
        // name) races worker 0's replacement of the name by k + 1.  Every
        // communicator must deliver its own key; no segment in use may be lost.
        const int K = atoi(argv[3]);
        int up[2];
        if (pipe(up)) return 9;
        pid_t p = fork();
        if (p == 0) {
            for (int k = 0; k < K; k++) {
                CallKey got{};
                try {
                    JobOrder b(session, 1, 2, 20000);
                    while (!b.Peek(&got)) usleep(10);
                    b.Consume();
                    if (write(up[1], "c", 1) != 1) _exit(8);
                } catch (const std::exception& e) {
                    printf("follower %d: %s\n", k, e.what());
                    fflush(stdout);
                    _exit(4);
                }
                if (got.comm != (uint32_t)k) {
                    printf("follower %d got comm %u\n", k, got.comm);
                    fflush(stdout);
                    _exit(5);
                }
            }
            _exit(0);
        }
        char c;
        for (int k = 0; k < K; k++) {
            JobOrder a(session, 0, 2, 20000);
            a.Append(CallKey{(uint32_t)k, 0, 0, 1, 7, 0});
            if (read(up[0], &c, 1) != 1) return 7;
        }
        int st;
        waitpid(p, &st, 0);
        printf("churn done\n");
        return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
    }
    try {                                            // "join": a second leader for the session
        JobOrder o(session, 0, 2, 2000);
        printf("joined\n");
    } catch (const std::exception& e) {
        printf("refused: %s\n", e.what());
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("joborder")
    src = d / "driver.cc"
    src.write_text(DRIVER)
    exe = d / "driver"
    subprocess.run(["g++", "-O1", "-std=c++17", f"-I{SRC}", "-o", str(exe), str(src),
                    os.path.join(SRC, "job_order.cc"), "-lpthread", "-lrt"], check=True)
    return str(exe)


@pytest.mark.parametrize("W,C,N", [(2, 2, 500), (4, 3, 300), (8, 2, 200)])
def test_every_worker_submits_worker0_order(driver, tmp_path, W, C, N):
    session = f"test-{os.getpid()}-{W}-{C}"
    r = subprocess.run([driver, "order", session, str(W), str(C), str(N)], capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, ORDER_OUT=str(tmp_path)))
    assert r.returncode == 0, r.stderr
    seqs = {str(w): (tmp_path / f"r{w}").read_text().strip() for w in range(W)}
    assert len(set(seqs.values())) == 1, "workers submitted in different orders"
    keys = seqs["0"].strip(",").split(",")
    assert len(keys) == C * N
    for c in range(C):                               # each channel's calls stay in order
        s = [int(k.split(":")[1]) for k in keys if k.split(":")[0] == str(c)]
        assert s == list(range(N))
    assert not os.path.exists(f"/dev/shm/switchml-collnet-{session}")


def test_stale_segment_replaced_live_one_refused(driver):
    session = f"stale-{os.getpid()}"
    path = f"/dev/shm/switchml-collnet-{session}"
    r = subprocess.run([driver, "leader", session], capture_output=True, text=True, timeout=60)
    assert "created" in r.stdout and os.path.exists(path)          # left behind by a "crashed" creator
    r = subprocess.run([driver, "join", session], capture_output=True, text=True, timeout=60)
    assert "joined" in r.stdout, r.stdout + r.stderr               # dead creator: replaced
    os.unlink(path) if os.path.exists(path) else None
    live = subprocess.Popen([driver, "leader", session, "20"], stdout=subprocess.PIPE, text=True)
    try:
        assert live.stdout.readline().strip() == "created"
        r = subprocess.run([driver, "join", session], capture_output=True, text=True, timeout=60)
        assert r.stdout.startswith("refused") and "in use" in r.stdout
    finally:
        live.kill()
        live.wait()
        if os.path.exists(path):
            os.unlink(path)


def test_poison_reaches_every_worker(driver):
    r = subprocess.run([driver, "poison", f"poison-{os.getpid()}"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "follower saw poison" in r.stdout


def test_reconnect_same_session(driver):
    """a communicator closed and reconnected under the same
    session — worker 1 first, while worker 0 still holds the old order — gets
    the new order: worker 0 removes the name on close, a full segment (all
    its workers attached) is an old communicator's and is not joined, and
    worker 0's own old segment never blocks it."""
    session = f"reconnect-{os.getpid()}"
    r = subprocess.run([driver, "reconnect", session], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "starts with comm 1" in r.stdout
    assert not os.path.exists(f"/dev/shm/switchml-collnet-{session}")


def test_late_detach_keeps_the_new_segment(driver):
    """a worker that detaches from an old communicator after
    worker 0 has reconnected under the same session never removes the new
    communicator's segment (worker 0 alone owns the name)."""
    session = f"late-{os.getpid()}"
    r = subprocess.run([driver, "late_detach", session], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "joined B" in r.stdout, r.stdout + r.stderr
    assert not os.path.exists(f"/dev/shm/switchml-collnet-{session}")


def test_churned_sessions_keep_every_communicator(driver):
    """ADVICE r4 under load: 300 communicators in a row under one session,
    each worker closing and reconnecting as fast as it can, the last
    detach of one interleaving with worker 0's creation of the next: every
    communicator delivers its own key, and the name is gone at the end.
    (The check-then-unlink window itself is too narrow to hit on demand —
    the round-4 code passes this too; the flock in unlink_if_named closes it
    by construction.)"""
    session = f"churn-{os.getpid()}"
    r = subprocess.run([driver, "churn", session, "300"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "churn done" in r.stdout, r.stdout + r.stderr
    assert not os.path.exists(f"/dev/shm/switchml-collnet-{session}")


def test_unsized_segment_is_not_mapped(driver):
    """a follower that opens worker 0's segment between its O_EXCL
    create and its ftruncate sees 0 bytes; mapping and reading it would raise
    SIGBUS.  An empty segment of the session's name (what that window looks
    like) is waited out by a follower and replaced by worker 0."""
    session = f"unsized-{os.getpid()}"
    path = f"/dev/shm/switchml-collnet-{session}"
    open(path, "wb").close()                         # 0 bytes, like a segment not yet sized
    try:
        r = subprocess.run([driver, "join", session], capture_output=True, text=True, timeout=60)
        assert "joined" in r.stdout, r.stdout + r.stderr
    finally:
        if os.path.exists(path):
            os.unlink(path)
