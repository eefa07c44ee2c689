"""The driver's N > 1 bench command, observed by the GPU suite (VERDICT r4
#2): `bench.py --gpus 2 --steps 4 --warmup 2` as a fresh child process on a
one-GPU box, under SML_BENCH_REHEARSE=1 — both ranks on cuda:0, each an RCCL
host of its own, so every collective runs in RCCL's kernels as on a node
(bench.py main).  The line must parse and carry: n_gpus 2, the nccl (RCCL)
backend, the headline's self-check against the committed digests, every
switch path verified bit for bit (p4/exponents.p4:48-54,
p4/processor.p4:48-54 via the oracle digests and the cross-path equality),
both N > 1 readings, and a timed region that fits inside the child's wall
time."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from mp_ranks import heartbeat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def run_child(cmd, env, out_dir, timeout, what):
    """Run `cmd` in its own session with stdout / stderr to files; heartbeat
    every 20 s; kill the whole process group at the timeout.  Returns
    (returncode, stdout text, stderr tail, wall seconds)."""
    out_p, err_p = os.path.join(out_dir, "stdout"), os.path.join(out_dir, "stderr")
    t0 = time.monotonic()
    with open(out_p, "w") as fo, open(err_p, "w") as fe:
        p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=fo, stderr=fe, start_new_session=True)
        last = t0
        while p.poll() is None:
            now = time.monotonic()
            if now - t0 > timeout:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                break
            if now - last >= 20:
                heartbeat(f"{what}: running for {now - t0:.0f} s")
                last = now
            time.sleep(0.5)
    wall = time.monotonic() - t0
    with open(out_p) as f:
        out = f.read()
    with open(err_p, errors="replace") as f:
        err = f.read()[-3000:]
    return p.returncode, out, err, wall


def rendezvous_port():
    """A --master-port for the driver-form launch, chosen BELOW the kernel's
    ephemeral range (/proc/sys/net/ipv4/ip_local_port_range): no outgoing
    connection (RCCL's, the TCP net's, the store clients') is ever given such
    a port, so between this pick and torchrun's bind only another explicit
    listener could take it — not the bind-0-close-reuse race.
    Checked free (bindable) at pick time; random within [lo - 12000, lo)."""
    import random
    import socket
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        lo = 32768
    top = max(lo, 2048)
    cands = list(range(max(1025, top - 12000), top))
    random.SystemRandom().shuffle(cands)
    for port in cands[:200]:
        with socket.socket() as s:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
        return port
    raise RuntimeError("no free port below the ephemeral range")


def assert_two_readings(line, n, nb=4):
    """the same keys at every N — value = weak_256MiB_value
    (256 MiB per GPU), strong_1GiB_value (configs[3]'s 1 GiB job over the N
    GPUs), each with its own roofline and self-check — and `scaling` "weak"
    at every N."""
    assert line["scaling"] == "weak"
    assert line["value"] == line["weak_256MiB_value"] > 0
    assert set(line["config"]["readings"]) == {"value", "weak_256MiB_value", "strong_1GiB_value"}
    for key, blk in (("weak_256MiB_value", "weak_256MiB"), ("strong_1GiB_value", "strong_1GiB")):
        b = line[blk]
        assert line[key] == b["value"] > 0 and b["n_gpus"] == n
        assert b["self_check"] is True and b["buckets_checked_min_over_ranks"] == nb, (blk, b)
        assert b["roofline"]["bound"] == "hbm" and 0 < b["roofline"]["frac"] < 1.0
    assert line["weak_256MiB"]["numel_per_gpu"] == 67_108_864
    assert line["strong_1GiB"]["job_numel"] == 268_435_456
    assert line["strong_1GiB"]["numel_per_gpu"] == 268_435_456 // n
    assert line["strong_1GiB"]["scaling"] == "strong" and line["weak_256MiB"]["scaling"] == "weak"


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("launcher,n", [("bench", 2), ("driver", 2), ("driver", 4)])
def test_bench_n2_rehearsal_line(cuda, tmp_path, launcher, n):
    """launcher "bench": `bench.py --gpus 2` starts its ranks itself;
    "driver": the driver's own form, `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
    bench.py --gpus 2 ...` (RANK / LOCAL_RANK / MASTER_* from torchrun)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    env["SML_BENCH_REHEARSE"] = "1"
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "4", "--warmup", "2"]
    if launcher == "bench":
        cmd = [sys.executable, "-u", *args]
    else:
        cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(rendezvous_port()), *args]
    rc, out, err, wall = run_child(cmd, env, str(tmp_path), 800, f"bench.py --gpus {n} (rehearsal, {launcher})")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, f"no JSON line (rc {rc}); stderr tail:\n{err}"
    line = json.loads(lines[-1])
    assert rc == 0, (rc, line.get("failures"), line.get("diagnostic_failures"), err[-1500:])
    assert line["n_gpus"] == n and line["steps"] == 4 and line["warmup"] == 2
    assert line["config"]["process_group"]["backend"] == "nccl"
    assert line["config"]["process_group"]["rehearsal"]
    assert line["self_check"] is True and line["self_check_detail"]["buckets_checked_min_over_ranks"] == 4
    for k in bench.SWITCH_PATHS:
        assert line[k].get("verified") is True, (k, line[k])
        assert line[k]["workers"] == n
    assert line["p2p_switch"]["bit_equal_to_switchsim"] and line["xgmi_switch"]["bit_equal_to_switchsim"]
    assert line["ms_per_step"] * line["steps"] / 1e3 < wall
    assert_two_readings(line, n)
    # rehearsal-only fields are labelled, never reported as measured against xGMI
    assert line["rehearsal_note"]
    for k in (*bench.SWITCH_PATHS, "rccl_fp32_allreduce"):
        f = line.get(k, {})
        assert f.get("frac_of_xgmi_bound") is None and f.get("rehearsal_note"), (k, f)
    assert line["switchsim"]["phases_note"] and line["configs4_plugin"]["rehearsal_note"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_n1_line(cuda, tmp_path):
    """The driver's N = 1 line keeps its contract: the metric and unit of
    BASELINE.json, the headline's self-check against the committed digests,
    `roofline` (hbm bound, 8 TB/s peak, frac = achieved / peak, PMC traffic
    within 0.1 % of the algorithmic bytes) and `cpu_baseline` (the oracle's
    port of the reference path on the host cores) — with a short CPU sample
    (--cpu-seconds 2) to keep the test brief; `--graph-steps` exercised too
    (a graph of 4 steps over the 4 cycled buckets: the self-check covers
    every bucket the replays write)."""
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    quick = ["--no-cpu-baseline", "--no-side", "--no-rccl-collnet"]
    for extra in ([], ["--graph-steps", "4"] + quick, ["--buckets", "1"] + quick):
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "4",
               "--cpu-seconds", "2"] + extra
        rc, out, err, wall = run_child(cmd, env, str(tmp_path), 500, "bench.py --gpus 1")
        lines = [l for l in out.splitlines() if l.startswith("{")]
        assert lines, (rc, err[-1500:])
        line = json.loads(lines[-1])
        assert rc == 0, (rc, line.get("failures"), line.get("diagnostic_failures"), err[-800:])
        assert line["metric"] == base["metric"] and line["unit"] == "GB/s" and line["n_gpus"] == 1
        assert line["self_check"] is True and line["higher_is_better"] is True
        nb = line["config"]["buckets_cycled"]
        assert line["self_check_detail"]["buckets_checked_min_over_ranks"] == nb == (1 if "--buckets" in extra else 4)
        assert line["ms_per_step"] * line["steps"] / 1e3 < wall
        r = line["roofline"]
        assert r["bound"] == "hbm" and r["peak"] == bench.HBM_PEAK_GBPS and r["unit"] == "GB/s"
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3 and 0.3 < r["frac"] < 1.0
        n, P = line["config"]["numel_per_gpu"], line["config"]["packet_numel"]
        assert abs(r["traffic"] / (8 * n + -(-n // P)) - 1) < 1e-3
        assert_two_readings(line, 1, nb)
        assert "rehearsal_note" not in line
        if not extra:
            cb = line["cpu_baseline"]
            assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["unit"].startswith("GB/s")
        elif "--graph-steps" in extra:
            assert "hipGraph" in line["config"]["launch"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_rehearsal_survives_a_failed_first_contact(cuda, tmp_path):
    """DESIGN §6, first contact: one rank's in-node switch fails right after
    joining its session (SML_BENCH_INJECT=xgmi_switch:1 ->
    backend.xgmi.fail_setup), as a worker that cannot map a peer's plane on
    the driver's first 8-GPU run would.  The ranks agree on the failure
    collectively and move on: the line is printed, exit 0 (a path that could
    not run is diagnostic), xgmi_switch reports its error and failed phase,
    the other three switch paths are verified, and nothing waited out a
    barrier timeout (the session was poisoned)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    env["SML_BENCH_REHEARSE"] = "1"
    env["SML_BENCH_INJECT"] = "xgmi_switch:1"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
           "--switch-numel", "4194304", "--job-numel", "0", "--no-plugin", "--no-rccl-collnet",
           "--exchange-timeout", "150"]
    rc, out, err, wall = run_child(cmd, env, str(tmp_path), 500, "bench.py --gpus 2 (injected xgmi setup failure)")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, f"no JSON line (rc {rc}); stderr tail:\n{err}"
    line = json.loads(lines[-1])
    assert rc == 0, (rc, line.get("failures"), line.get("diagnostic_failures"), err[-1500:])
    assert "xgmi_switch" in line, (line.get("switchsim"), line.get("diagnostic_failures"), err[-2000:])
    x = line["xgmi_switch"]
    assert x["failed_phase"] == "setup" and ("injected setup failure" in x["error"] or "another rank" in x["error"]), x
    for k in ("switchsim", "p2p_switch", "xgmi_switch_push"):
        assert line[k].get("verified") is True, (k, line[k])
    assert any(d.startswith("xgmi_switch:") for d in line["diagnostic_failures"]), line["diagnostic_failures"]
    assert wall < 150, wall


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("dying", [0, 1])
def test_bench_line_survives_a_dead_rank(cuda, tmp_path, dying):
    """DESIGN §6, first contact: a rank that DIES in the diagnostic phase (a
    fault on its first peer access; here SML_BENCH_INJECT=die:<rank>,
    os._exit(7) at the phase's start).  The driver's launcher,
    torch.distributed.run, then SIGTERMs the surviving ranks; bench.term_guard
    takes the signal on its own thread and the rank holding the store's token
    prints the line — rank 0, or rank 1 when rank 0 is the one that died —
    with the measured, self-checked headline and a "terminated" diagnostic.
    The run's exit status is the failure's (non-zero), but the line is there."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    env["SML_BENCH_REHEARSE"] = "1"
    env["SML_BENCH_INJECT"] = f"die:{dying}"
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2", "--job-numel", "0",
            "--switch-numel", "4194304", "--no-rccl-collnet", "--exchange-timeout", "200"]
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(rendezvous_port()), *args]
    rc, out, err, wall = run_child(cmd, env, str(tmp_path), 500, f"bench.py --gpus 2 (rank {dying} dies)")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (rc, lines, err[-2000:])
    line = json.loads(lines[0])
    assert rc != 0
    assert line["self_check"] is True and line["value"] > 0 and line["n_gpus"] == 2
    term = [d for d in line.get("diagnostic_failures", []) if d.startswith("terminated")]
    assert term, (line.get("diagnostic_failures"), err[-2000:])
    assert ("printed by rank 1" in term[0]) == (dying == 0), term
    assert wall < 150, wall      # SIGTERM answered at once, not after the watchdog or the SIGKILL grace


def test_rendezvous_port_is_below_the_ephemeral_range():
    """the driver-form rehearsal's --master-port is never an
    ephemeral port (no outgoing connection can be handed it between the pick
    and torchrun's bind) and is free when picked."""
    import socket
    with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
        lo = int(f.read().split()[0])
    for _ in range(5):
        p = rendezvous_port()
        assert 1024 < p < max(lo, 2048), (p, lo)
        with socket.socket() as s:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind(("127.0.0.1", p))
