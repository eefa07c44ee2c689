#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X:
"fp32->int32 quantize+pack GB/s (device-resident), 256 MiB bucket, 1/2/4/8 GPU".

One step = one pass of the hot path (CpuExponentQuantizerPPP's
PreprocessSingle over a whole job slice: per-packet exponent, fp32->int32
scale+round, big-endian pack — ppp.cc:69-156) over fp32 data already resident
in HBM, as one launch of the fused HIP kernel sml_quantize_pack (K1) per GPU.
Exponents are the loopback's (the dummy backend returns them unchanged, so
the local exponent is the global one: W = 1).

Every N (1 by default; `--gpus N` starts the N ranks itself when WORLD_SIZE
is unset, or they come from torch.distributed.run) reports the SAME two
readings, each with its own timed region, self-check and roofline, so a
1/2/4/8 curve compares each reading with itself:
  value = weak_256MiB_value   the step is K1 over a 256 MiB bucket (configs[2]'s
              bucket) on EVERY GPU, 4 buckets cycled; `scaling` "weak" at every N
  strong_1GiB_value   the step is configs[3] — ONE 1 GiB job split over the N
              GPUs by the FIFO rule (fifo_scheduler.cc:93-109, slice g -> GPU
              g; the whole job on one GPU at N = 1); strong scaling
The path has no exchange step at W = 1, so no collective runs in either timed
region.  At N > 1, first-class fields beside them time the switch simulation
with W = N real workers (each holding its own 1 GiB bucket):
  switchsim   K2 -> RCCL int8 MAX -> K3 -> RCCL int32 SUM -> K4 (ring, xGMI)
  p2p_switch  K2 -> RCCL int8 MAX -> K3 -> K6 over the peers' HBM (hipIpc,
              xGMI) on this rank's block shard -> RCCL all_gather (fp32)
  xgmi_switch the client's Context::AllReduce with backend = xgmi (the
              native in-node switch: shm rendezvous, exponent max over the
              peers' planes, K3, K6 on this rank's shard, gather)
  xgmi_switch_push  the same in its push form (backend.xgmi.push: K3 writes
              each shard into its owner's inbox over xGMI, K6 reads local HBM)
each checked (bit-equal to each other, and within the quantization bound of
an fp32 all-reduce of the same buckets) and set against its xGMI bound; and
configs4_plugin: the ResNet-50 buckets through the CollNet plugin table on an
N-rank communicator over the xgmi backend (device and pinned host buffers).
The exit status is 1 when the headline's own check fails (the timed planes
differ from the committed digests), when the headline cannot be measured, or
when ANY switch path (switchsim, p2p_switch, xgmi_switch, xgmi_switch_push)
RAN and gave wrong bits — not within the quantization bound, timed calls that
differ from the first, or a peer-memory path not bit-equal to switchsim: wrong
bits are a correctness failure wherever they come from (--lenient-switch
demotes the peer-memory paths' mismatch to a diagnostic, for bring-up only).
A field that could not run or timed out (switch paths, plugin,
rccl_collnet) is reported in the line under "diagnostic_failures" and in its
own field, so one path that cannot start cannot void the measured headline.

Units: value / roofline.achieved = ALGORITHMIC bytes per second: 4N read
(fp32 in) + 4N written (int32 payload) + B written (int8 exponents),
B = ceil(N/256) per slice — see DESIGN.md §4.  input_GBps = 4N / t alongside.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBPS = 153.0   # per xGMI link and direction; 7 links per GPU, one to each peer of an 8-GPU node
CFG3_JOB_NUMEL = 268_435_456   # configs[3]: 1 GiB fp32 (also allreduce_benchmark's default tensor-numel, main.cc:101)
METRIC = "fp32→int32 quantize+pack GB/s (device-resident), 256 MiB bucket, 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="untimed launches of the same step for this long before the warmup steps "
                         "(HBM/fabric clocks ramp under load: profiles/r01/bench_warmup_sweep.jsonl)")
    ap.add_argument("--numel", type=int, default=64 * 1024 * 1024, help="fp32 elements per GPU at N=1 (256 MiB)")
    ap.add_argument("--packet-numel", type=int, default=256)
    ap.add_argument("--job-numel", type=int, default=CFG3_JOB_NUMEL,
                    help="the strong_1GiB reading (at every N, beside the weak headline): one job of this many "
                         "fp32 elements split over the ranks by the FIFO rule (default configs[3]'s 268435456 = "
                         "1 GiB; 0 = skip the reading)")
    ap.add_argument("--strong-steps", type=int, default=200,
                    help="timed steps of the strong_1GiB reading (fixed, so its value does not carry the first "
                         "launch's latency at N = 8's 128 MiB slices the way 20 steps would)")
    ap.add_argument("--strong-warmup", type=int, default=100)
    ap.add_argument("--switch-numel", type=int, default=CFG3_JOB_NUMEL,
                    help="N > 1: fp32 elements per worker for the switchsim / p2p_switch fields (0 = skip them)")
    ap.add_argument("--exchange-timeout", type=float, default=300.0,
                    help="N > 1: seconds the switch / plugin phase may take before the run reports what it has "
                         "measured, with a failure, and exits 1 (a hang would otherwise print nothing)")
    ap.add_argument("--lenient-switch", action="store_true",
                    help="N > 1, bring-up only: a peer-memory switch path (p2p_switch, xgmi_switch, "
                         "xgmi_switch_push) that runs and gives wrong bits is reported under diagnostic_failures "
                         "instead of failing the run (default: wrong bits from any path fail the run)")
    ap.add_argument("--no-plugin", action="store_true",
                    help="N > 1: skip the configs4_plugin field (ResNet-50 buckets through the CollNet table per rank)")
    ap.add_argument("--buckets", type=int, default=4,
                    help="distinct input buckets (and output planes) the timed steps cycle through: 4 (default) "
                         "streams 2 GiB past the 256 MiB Infinity Cache, so the headline is an HBM-proper rate; "
                         "1 = one resident bucket (HBM + Infinity Cache; reported as side.resident)")
    ap.add_argument("--grid-limit", type=int, default=0, help="workgroups per launch (0 = one per 4 tiles)")
    ap.add_argument("--xcd-chunk", type=int, default=64,
                    help="workgroups per contiguous run on one XCD (0 = plain blockIdx order)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side", action="store_true", help="skip the cold-HBM and 1 GiB single-GPU side fields")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--extra", action="store_true", help="also time dequantize / fused round trip / copy / plugin")
    ap.add_argument("--no-rccl-collnet", action="store_true",
                    help="skip the rccl_collnet field (RCCL's own all_reduce dispatched into the CollNet plugin, "
                         "run by rank 0 in fresh child processes at the end)")
    ap.add_argument("--graph-steps", type=int, default=1,
                    help="capture this many steps per hipGraph replay (1 = eager launches)")
    return ap.parse_args(argv)


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes with
    torch.distributed.run (one per GPU) as CHILD processes and exit with their
    status.  --standalone: the launcher's own store binds an OS-chosen port on
    127.0.0.1 and hands it to the ranks (no port picked here and bound later,
    which another process could take in between).  Runs before anything
    touches the GPU (no exec from a GPU-initialised process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", f"--nproc-per-node={n}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def load_traffic(numel, P, key="quantize_pack"):
    """HBM bytes per launch from the PMC passes (profiles/pmc_traffic.json,
    written by profiles/collect_pmc.py from separate rocprofv3 --pmc runs):
    the entry `key` when its size matches, and for the cycling pattern also
    the per-GPU FIFO slice sizes of configs[3] (`quantize_pack_cold_slices`,
    the N > 1 lines)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        k = d.get(key, {})
        if k.get("numel") == numel and k.get("packet_numel") == P:
            return k.get("hbm_bytes_per_launch")
        if key == "quantize_pack_cold":
            for e in d.get("quantize_pack_cold_slices", []):
                if e.get("numel") == numel and e.get("packet_numel") == P:
                    return e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def host_cores():
    """CPU threads this process may run on: its affinity mask, capped by the
    cgroup CPU quota (cgroup v2 cpu.max) when one is set — on the GPU box the
    mask lists every core of the machine while the lease's quota is its share
    — and the share the box announces (OMP_NUM_THREADS)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, round(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    return aff, quota, share


BENCH_SEED0 = 4242   # bucket b of a run holds bench_bucket(4242 + b, ...) (tests/golden/make_bench_digests.py)
DIGESTS_BENCH = os.path.join(ROOT, "tests", "golden", "digests_bench.json")


def _u64(c):
    """A 64-bit constant as the int64 with the same bits (torch has no uint64 arithmetic)."""
    c &= (1 << 64) - 1
    return c - (1 << 64) if c >= 1 << 63 else c


def _lsr(torch, z, s):
    """Logical right shift of int64 bit patterns."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def bench_bucket(torch, seed, off, n, device):
    """Gradient-like fp32 from integer arithmetic only, elements [off, off+n)
    of a job: the same bits on every host and device.  Restates oracle.py's
    splitmix_grad (a signed 24-bit mantissa from splitmix64, scaled by
    2^-(24+k), k in 0..15 varying per 256-block, so block exponents differ)
    over the GLOBAL element index, so a rank's FIFO slice of a job is exactly
    that slice of the job; int64 products wrap like the uint64 ones."""
    out = torch.empty(n, dtype=torch.float32, device=device)
    step = 1 << 25
    for a in range(0, n, step):          # bounded temporaries
        m = min(step, n - a)
        i = torch.arange(off + a, off + a + m, dtype=torch.int64, device=device)
        z = i * _u64(0xBF58476D1CE4E5B9) + _u64(seed * 0x9E3779B97F4A7C15)
        z = (z ^ _lsr(torch, z, 31)) * _u64(0x94D049BB133111EB)
        z = z ^ _lsr(torch, z, 29)
        mant = _lsr(torch, z, 40) - (1 << 23)                       # [-2^23, 2^23)
        k = ((i >> 8) * 7 + (z & 1)) % 16
        scale = ((127 - 24 - k).to(torch.int32) << 23).view(torch.float32)   # 2^-(24+k), exact
        out[a:a + m] = mant.to(torch.float32) * scale
    return out


def planes_sha256(torch, exps, payload, numel, P):
    """SHA-256 of an exponent plane and the first numel words of a payload
    plane (host copies; outside any timed region)."""
    import hashlib
    e = exps.cpu().numpy().tobytes()
    q = payload[:numel].cpu().numpy().tobytes()
    return {"exps": hashlib.sha256(e).hexdigest(), "payload": hashlib.sha256(q).hexdigest()}


def expected_digests(job_numel, world, rank, N, P, nb):
    """The committed digests of this rank's buckets, or None when the run's
    shape has none (other packet size / bucket size / bucket count)."""
    try:
        with open(DIGESTS_BENCH) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if P != d["packet_numel"] or nb > d["buckets"]:
        return None
    if job_numel == 0 and N == d["bucket_numel"]:
        return d["bucket_T1"][:nb]
    if job_numel == d["job_numel"] and f"T{world}" in d["job"]:
        return [d["job"][f"T{world}"][b][rank] for b in range(nb)]
    return None


def cpu_baseline(numel, P, budget_s):
    """The oracle's restatement of the reference CPU path (per-packet
    PreprocessSingle calls in DummyWorkerThread order, b = mop/T ring) on this
    host's cores, over the same 256 MiB bucket, repeated for ~budget_s.

    `value` is the reference's DEFAULT build, VCL=1 (client_lib/Makefile:26,
    113-120): its 16-element vector loops restated with SSE2 intrinsics — the
    instruction set that build targets (no -m flags) — with one worker thread
    per usable core (the affinity mask capped by the cgroup CPU quota).  One
    thread per core of the whole affinity mask, the lease's announced share
    (OMP_NUM_THREADS), the reference's default 4 worker threads, 1 thread, and
    the scalar VCL=0 path (roundf per element) are reported beside it."""
    import numpy as np
    from oracle import oracle as O

    aff, quota, share = host_cores()
    cores = min(aff, quota) if quota else aff
    x = O.splitmix_normal(42, numel)
    out = np.empty_like(x)
    alg = 8 * numel + O.num_blocks(numel, P)

    def run(T, deadline_s, min_reps, vcl):
        rates, t_end, reps = [], time.perf_counter() + deadline_s, 0
        while reps < min_reps or time.perf_counter() < t_end:
            t0 = time.perf_counter()
            O.dummy_allreduce(x, P=P, max_outstanding_packets=max(256, 4 * T), num_worker_threads=T,
                              num_workers=1, threaded=T > 1, mode=O.MODE_PREPROCESS, out=out, vcl=vcl)
            rates.append(alg / (time.perf_counter() - t0) / 1e9)
            reps += 1
        return float(np.median(rates)), reps

    multi, repsT = run(cores, budget_s * 0.3, 3, True)
    at_aff = run(aff, budget_s * 0.1, 2, True)[0] if aff != cores else multi
    sh = run(share, budget_s * 0.1, 3, True)[0] if share and share not in (cores, aff) else (
        multi if share == cores else at_aff if share == aff else None)
    four = run(4, budget_s * 0.1, 3, True)[0] if cores > 4 else None
    single = run(1, budget_s * 0.1, 2, True)[0]
    s_multi = run(cores, budget_s * 0.2, 3, False)[0]
    s_single = run(1, budget_s * 0.1, 2, False)[0]
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), model)
    except OSError:
        pass
    # the baseline is the reference path at its BEST measured thread count
    # (a conservative GPU/CPU ratio): all usable cores, or the lease's share
    best_T, best = max(((cores, multi), (aff, at_aff), (share or cores, sh if sh is not None else multi)),
                       key=lambda tv: tv[1])
    return {
        "value": round(best, 3),
        "unit": "GB/s (8N+B algorithmic bytes, same as value)",
        "cores": best_T,
        "kind": "port",
        "sample": (f"oracle/sml_oracle.c restatement of CpuExponentQuantizerPPP as the reference builds it by "
                   f"default (VCL=1, vector loops in SSE2), driven in DummyWorkerThread order, PreprocessSingle "
                   f"only (exponent + quantize + BE pack into the b-packet ring), the full {numel * 4 >> 20} MiB "
                   f"bucket, packet_numel {P}; value = best of {cores} worker threads (affinity mask {aff} CPUs, "
                   f"cgroup quota {quota} CPUs; {repsT} reps, median): {multi:.3f} GB/s, {aff} threads: "
                   f"{at_aff:.3f}, the lease's share of {share} threads: {sh}; 1 thread: {single:.3f} GB/s; scalar "
                   f"VCL=0 build: {s_multi:.3f} GB/s on {cores} threads, {s_single:.3f} on 1; host CPU {model}"),
        "all_cores_threads": cores,
        "all_cores_value": round(multi, 3),
        "cores_source": "min(len(os.sched_getaffinity(0)), cgroup cpu.max quota)",
        "affinity_cpus": aff,
        "cgroup_quota_cpus": quota,
        "affinity_threads_value": round(at_aff, 3),
        "lease_share_threads": share,
        "lease_share_value": None if sh is None else round(sh, 3),
        "single_thread_value": round(single, 3),
        "ref_default_4_threads_value": None if four is None else round(four, 3),
        "vcl0_scalar_value": round(s_multi, 3),
        "vcl0_scalar_single_thread_value": round(s_single, 3),
        "cpu_model": model,
        "input_GBps": round(multi * 4 * numel / alg, 3),
    }


class Fail(RuntimeError):
    """A check of the run failed: the line is still printed, the exit status is 1."""


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
        world = 1
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    on_term = {"emit": None}
    if world > 1:
        term_guard(on_term)

    import torch
    import torch.distributed as dist
    import switchml_amd as sw

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SML_BENCH_REHEARSE=1: rehearse the N>1 path on a 1-GPU box — all ranks
    # on device local % device_count, still over RCCL: every rank is an RCCL
    # host of its own (NCCL_HOSTID), the ranks linked by the SwitchML
    # library's TCP net (switchml_amd.rccl_collnet.same_gpu_rccl_env), so the
    # reductions run in the same RCCL kernels as on a node.  SML_BENCH_REHEARSE
    # =gloo keeps the old host-reduction rehearsal.  Never used for numbers.
    rehearse_mode = os.environ.get("SML_BENCH_REHEARSE", "")
    rehearse = rehearse_mode in ("1", "gloo")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if rehearse else local
    if world > 1:
        if rehearse_mode == "gloo":
            dist.init_process_group("gloo")
        else:
            if rehearse:
                from switchml_amd.rccl_collnet import same_gpu_rccl_env
                os.environ.update(same_gpu_rccl_env(rank, "bench" + os.environ.get("MASTER_PORT", "0")))
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
    pg = {"backend": dist.get_backend() if world > 1 else None,
          "rehearsal": ("ranks share one GPU: " + ("gloo" if rehearse_mode == "gloo" else
                                                   "RCCL, one RCCL host per rank (NCCL_HOSTID), SwitchML TCP net"))
          if rehearse else None}
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    sw.lib()
    if args.grid_limit:
        sw.set_grid_limit(args.grid_limit)
    sw.set_xcd_chunk(args.xcd_chunk)

    P = args.packet_numel
    if args.graph_steps > 1:
        # hipGraph capture needs a non-default stream: the whole run (launchers,
        # capture, replays, the timing events) moves to one
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    stream = torch.cuda.current_stream()
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    nb = max(1, args.buckets)

    # The headline, `value` = weak_256MiB_value at every N: every GPU runs K1
    # over its own 256 MiB buckets (the metric's bucket; N = 1 is configs[2]'s).
    hl = k1_reading(sw, torch, dist, world, rank, dev, stream, 0, args.numel, P, nb, args.steps, args.warmup,
                    args.settle_ms, args.graph_steps)
    # (the second reading, strong_1GiB_value, runs once the line can be
    # printed without it: below, under the N > 1 watchdog)
    st = None
    N, B, alg_bytes = hl["numel_per_gpu"], hl["num_blocks_per_gpu"], hl["alg_bytes_per_gpu"]
    elapsed, kern_ms_max = hl["elapsed_s"], hl["kernel_ms"]

    failures = []
    if not hl["ok"]:
        failures.append(f"self_check ({hl['name']}): " + hl["check_note"])
    diag_failures = []          # diagnostic fields: reported, not fatal (module docstring)
    side, fields, extra = {}, {}, {}

    emit_lock, emitted = threading.Lock(), [False]
    # N > 1: the launcher's store (torch.distributed.run hosts it in its
    # agent, so it outlives any rank) holds a one-shot token; whichever rank
    # takes it prints the line
    store = dist.distributed_c10d._get_default_store() if world > 1 else None

    def take_token():
        """Every printing path takes it (rank 0's normal end and watchdog
        too), so a rank SIGTERMed after rank 0 printed stays silent."""
        if store is None:
            return True
        try:
            import datetime
            store.set_timeout(datetime.timedelta(seconds=20))   # the end of the run: never wait long
            return int(store.add("sml_bench_line_token", 1)) == 1
        except Exception:  # noqa: BLE001 - no store: rank 0 alone prints
            return rank == 0

    def emit(any_rank=False):
        """The run's one JSON line, from whatever has been measured so far —
        exactly once, whichever of the normal end, the watchdog or the
        launcher's SIGTERM (term_guard) comes first.  Rank 0 prints it; on
        SIGTERM (another rank died) any surviving rank may, the store's token
        deciding which — so a fault that kills rank 0 itself on its first
        peer access does not lose the line (every rank holds the same
        all-reduced readings and switch fields; only `side.topology` is
        rank 0's)."""
        if rank != 0 and not any_rank:
            return
        with emit_lock:
            if emitted[0]:
                return
            emitted[0] = True
            if take_token():
                emit_line()

    def emit_line():
        ms_per_step = elapsed * 1e3 / args.steps
        value = hl["total_alg"] / (elapsed / args.steps) / 1e9
        achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
        workload = (f"configs[2]-sized bucket: {N * 4 >> 20} MiB fp32 on EVERY GPU ({world} GPU(s), weak scaling), "
                    "fused exponent+quantize+BE pack (sml_quantize_pack, K1), loopback exponents (W=1); `value` "
                    "= weak_256MiB_value at every N; strong_1GiB_value = configs[3]'s 1 GiB job split over the N GPUs")
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32->i32",
            "data": ("synthetic gradient-like fp32 generated on device from integers only (bench_bucket: "
                     "splitmix64 24-bit mantissas x 2^-(24..39), seed 4242 + bucket, global element index); "
                     "every GPU holds its own copy of the same 4 buckets"),
            "config": {
                "workload": workload,
                "job_numel": world * N,
                "numel_per_gpu": N,
                "packet_numel": P,
                "num_blocks_per_gpu": B,
                "parallelism": f"shard{world} (every GPU its own buckets, no data-path collective)",
                "bytes_per_step_per_gpu": alg_bytes,
                "buckets_cycled": nb,
                "xcd_chunk": args.xcd_chunk,
                "launch": "eager" if args.graph_steps <= 1 else f"hipGraph replay, {args.graph_steps} steps per graph",
                "process_group": pg,
            },
            "input_GBps": round(4 * world * N / (elapsed / args.steps) / 1e9, 2),
            "kernel_ms": round(kern_ms_max, 5),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic(N, P, "quantize_pack" if nb == 1 else "quantize_pack_cold"),
                "kernel": f"sml::k_quantize_pack<{P},aligned,fused,BE,half-away> (K1: 2-slice wave tiles, sc1 nt payload stores at >= 64 MiB)",
            },
            "self_check": hl["ok"],
            "self_check_detail": {"what": hl["check_note"], "buckets_checked_min_over_ranks": hl["checked"]},
        }
        if nb > 1:
            line["roofline"]["note"] = (f"steps cycle {nb} distinct buckets + planes ({nb * (8 * N + B) >> 20} MiB "
                                        "per GPU, past the 256 MiB Infinity Cache): an HBM-proper rate")
        if "frac" in side.get("resident", {}):
            line["roofline"]["frac_resident"] = side["resident"]["frac"]
            line["roofline"]["traffic_resident"] = load_traffic(args.numel, P, "quantize_pack")
        rd = readings(hl, st, world, nb, P)
        line["config"]["readings"] = rd.pop("readings")
        line.update(rd)
        line["value"] = rd["weak_256MiB_value"]     # the same number, by construction
        if st is not None and rehearse:
            line["strong_1GiB"]["rehearsal_note"] = REHEARSAL_NOTE
        if rehearse:
            line["rehearsal_note"] = ("value / weak_256MiB_value / strong_1GiB_value: " + REHEARSAL_NOTE)
        line.update(fields)
        if side:
            line["side"] = side
        if extra:
            line["extra"] = extra
        if "cpu_baseline" in side_cpu:
            line["cpu_baseline"] = side_cpu["cpu_baseline"]
        if failures:
            line["failures"] = failures
        if diag_failures:
            line["diagnostic_failures"] = diag_failures
        print(json.dumps(line), flush=True)

    side_cpu = {}

    def on_sigterm():
        diag_failures.append("terminated: SIGTERM from the launcher (another rank failed or the run was stopped) "
                             "during the multi-GPU diagnostic phase; the fields above are what was measured"
                             + ("" if rank == 0 else f" (line printed by rank {rank})"))
        emit(any_rank=True)
    on_term["emit"] = on_sigterm

    def guarded(key, fn):
        """A side measurement: its failure is reported, never the headline's."""
        try:
            side[key] = fn()
        except Exception as e:  # noqa: BLE001 - reported in the line
            side[key] = {"error": repr(e)[:300]}
            diag_failures.append(f"side.{key}: {side[key]['error']}")

    watchdog = None
    if world > 1:
        # The multi-GPU phase (the strong reading, side fields, switch paths,
        # plugin over the in-node switch) is where a hang could happen; past the deadline the
        # run reports what it has, with the timeout, and every rank exits
        # (1 only if the headline's own check failed).
        def on_timeout():
            diag_failures.append(f"timeout: the multi-GPU diagnostic phase exceeded {args.exchange_timeout:g} s")
            try:
                # where every thread of this rank is stuck (to stderr; the
                # driver's record keeps it): the call a hang sits in
                import faulthandler
                sys.stderr.write(f"[bench rank {rank}] watchdog: stacks at the timeout\n")
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
            except Exception:  # noqa: BLE001 - diagnostics only
                pass
            try:
                emit()
            finally:
                os._exit(1 if failures else 0)
        watchdog = threading.Timer(args.exchange_timeout, on_timeout)
        watchdog.daemon = True
        watchdog.start()
    # The second named reading at every N, strong_1GiB_value: configs[3]'s one
    # 1 GiB job split over the N GPUs by the FIFO rule (at N = 1 the whole job
    # on one GPU), its own timed region, self-check and roofline.  At N > 1 it
    # runs under the watchdog: a hang in its barriers cannot swallow the
    # headline measured above.
    if args.job_numel:
        st = k1_reading(sw, torch, dist, world, rank, dev, stream, args.job_numel, 0, P, nb, args.strong_steps,
                        args.strong_warmup, args.settle_ms, 1)
        if not st["ok"]:
            failures.append(f"self_check ({st['name']}): " + st["check_note"])
    if world == 1 and not args.no_side:
        if nb > 1:
            guarded("resident", lambda: bucket_measure(sw, torch, args.numel, P, stream, nbuf=1))
        else:
            guarded("cold_hbm", lambda: bucket_measure(sw, torch, args.numel, P, stream, nbuf=4))
        guarded("copy_ceiling", lambda: copy_ceiling(sw, torch, args.numel, stream, nbuf=nb, k1_ms=kern_ms_max))
    if world > 1 and not args.no_side:
        if rank == 0:
            # what the peer-to-peer paths rely on: every pair of the node's GPUs can map each other
            guarded("topology", lambda: {
                "devices": ndev, "name": torch.cuda.get_device_name(dev),
                "peer_access": [[i == j or torch.cuda.can_device_access_peer(i, j) for j in range(ndev)]
                                for i in range(ndev)]})
    if world > 1 and os.environ.get("SML_BENCH_INJECT", "") == f"die:{rank}":
        # tests only: this rank dies at the start of the diagnostic phase, as
        # one that faults on its first peer access would (the launcher then
        # SIGTERMs the others: term_guard)
        sys.stderr.write(f"[bench rank {rank}] SML_BENCH_INJECT: dying\n")
        sys.stderr.flush()
        os._exit(7)
    if world > 1 and args.switch_numel:
        try:
            fields.update(exchange_measure(sw, torch, dist, args.switch_numel, P, world, rank, dev,
                                           rehearsal=pg["rehearsal"]))
        except Exception as e:  # noqa: BLE001 - recorded as a diagnostic failure below
            fields["switchsim"] = {"error": repr(e)[:400]}
        fatal, diag = switch_verdicts(fields, lenient=args.lenient_switch)
        failures.extend(fatal)
        diag_failures.extend(diag)
    if world > 1 and not args.no_plugin:
        # configs[4] on every GPU at once: each rank hands the ResNet-50 buckets
        # to its own plugin instance, on an N-rank communicator whose backend
        # is the in-node switch (a real cross-rank SwitchML all-reduce)
        try:
            fields["configs4_plugin"] = plugin_measure_ranks(torch, dist, dev, world)
            if rehearse:
                fields["configs4_plugin"]["rehearsal_note"] = (
                    "rehearsal: the N ranks' plugins share one GPU (peer planes in the same HBM, no xGMI); "
                    "times are not an N-GPU measurement")
            if not fields["configs4_plugin"]["placements_agree_all_ranks"]:
                diag_failures.append("configs4_plugin: device and pinned-host results differ")
        except Exception as e:  # noqa: BLE001
            fields["configs4_plugin"] = {"error": repr(e)[:400]}
            diag_failures.append(f"configs4_plugin: {fields['configs4_plugin']['error']}")
    if watchdog is not None:
        watchdog.cancel()
    if args.extra and rank == 0:
        extra.update(extra_measurements(sw, torch, torch.randn(args.numel, device=dev, generator=gen), P, stream))
    if world > 1:
        dist.destroy_process_group()
    if not args.no_rccl_collnet and rank == 0:
        # RCCL itself calling the plugin's CollNet table, in fresh processes
        # (their own RCCL communicator and xgmi session); not part of the
        # headline, and its failure is reported in the field, not fatal
        torch.cuda.empty_cache()
        fields["rccl_collnet"] = rccl_collnet_field(world, same_gpu=world == 1 or rehearse)
        if not fields["rccl_collnet"].get("ok", False):
            diag_failures.append("rccl_collnet: " + fields["rccl_collnet"].get("error", "not ok"))
    if world == 1 and not args.no_cpu_baseline:
        try:
            side_cpu["cpu_baseline"] = cpu_baseline(N, P, args.cpu_seconds)
        except Exception as e:  # noqa: BLE001 - reported; the headline stands
            diag_failures.append(f"cpu_baseline: {repr(e)[:300]}")
    emit()
    if failures:
        sys.exit(1)


def term_guard(on_term):
    """N > 1: keep rank 0's line when the launcher stops the ranks.

    torch.distributed.run stops every rank with SIGTERM (SIGKILL 30 s later)
    as soon as ONE rank fails — a rank that faults on its first peer-memory
    access on a real node (first contact) would otherwise take the
    measured and checked headline down with it, unprinted.  SIGTERM is
    blocked in this thread before torch, RCCL or HIP start theirs (so all of
    them inherit the mask) and taken by one daemon thread in sigwait, which
    runs on_term["emit"] (rank 0's line with a "terminated" diagnostic, once
    the headline exists) and exits 1.  Every blocking wait of the main thread
    (collectives, device syncs, ctypes calls) releases the GIL, so the thread
    runs while the main thread is stuck in one."""
    import signal
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM})

    def waiter():
        signal.sigwait({signal.SIGTERM})
        try:
            if on_term["emit"] is not None:
                on_term["emit"]()
        finally:
            os._exit(1)
    threading.Thread(target=waiter, name="sigterm-guard", daemon=True).start()


REHEARSAL_NOTE = ("rehearsal: the ranks share ONE GPU (SML_BENCH_REHEARSE), so these rates are one device's "
                  "throughput split between the ranks, not N GPUs'; never a measurement of the N-GPU node")


def k1_reading(sw, torch, dist, world, rank, dev, stream, job_numel, numel, P, nb, steps, warmup, settle_ms,
               graph_steps=1):
    """One timed K1 reading on every rank.

    job_numel = 0: every rank quantizes its own `numel`-element buckets (the
    weak reading: the same per-GPU work at every N).  job_numel > 0: ONE job
    of that many elements split over the ranks by the FIFO rule
    (fifo_scheduler.cc:93-109, slice g -> GPU g: the strong reading).  Either
    way `nb` distinct buckets + planes are cycled step after step (past the
    256 MiB Infinity Cache: HBM proper), bucket b = elements [off, off + N) of
    bench_bucket(4242 + b, .) — integer-exact, so the planes the TIMED
    launches leave are hashed afterwards and compared with the oracle's
    digests (tests/golden/digests_bench.json).

    Timed region: `steps` back-to-back launches on `stream`, bracketed by a
    barrier and a device sync on both sides (wall clock -> value; MAX over
    ranks) and by two HIP events on the launch stream itself (-> average
    launch duration for the roofline; includes the inter-launch gaps, so it
    is conservative against rocprofv3's per-dispatch durations)."""
    off = 0
    if job_numel:
        off, N = sw.fifo_slice(job_numel, world, rank)
        total_alg = sum(8 * n + sw.num_blocks(n, P)
                        for n in (sw.fifo_slice(job_numel, world, r)[1] for r in range(world)))
    else:
        N = numel
        total_alg = world * (8 * N + sw.num_blocks(N, P))
    B = sw.num_blocks(N, P)
    xs = [bench_bucket(torch, BENCH_SEED0 + b, off, N, dev) for b in range(nb)]
    pls = [torch.empty(B * P, dtype=torch.int32, device=dev) for _ in range(nb)]
    exs = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nb)]
    cyc = [0]
    # one prepared C call per step (arguments checked once: the first step's
    # launch is not delayed by the Python wrapper)
    launchers = [sw.quantize_pack_launcher(xs[i], P, 1, pls[i], exps_out=exs[i], stream=stream) for i in range(nb)]

    def launch():
        i = cyc[0]
        cyc[0] = (i + 1) % nb
        launchers[i]()

    step, per_call = launch, 1
    if graph_steps > 1:
        # G consecutive steps captured into one hipGraph (G kernel nodes);
        # each replay still runs exactly G full steps.  The captured steps
        # cycle the buckets from bucket 0, so every replay covers every
        # bucket only when G is a multiple of their number.
        if graph_steps % nb:
            sys.exit(f"bench.py: --graph-steps {graph_steps} must be a multiple of --buckets {nb} "
                     "(each replay repeats the same captured steps)")
        if steps % graph_steps or warmup % graph_steps:
            sys.exit("bench.py: --steps and --warmup must be multiples of --graph-steps")
        launch()
        torch.cuda.synchronize()
        cyc[0] = 0
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for _ in range(graph_steps):
                launch()
        step, per_call = graph.replay, graph_steps

    settle(step, settle_ms)
    for _ in range(warmup // per_call):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # one untimed pass through the timing code itself (events, syncs,
    # barriers), so lazy first-use costs of those calls stay out of the region
    for _ in range(2):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0.record(stream)
        step()
        ev1.record(stream)
        torch.cuda.synchronize()
        _ = ev0.elapsed_time(ev1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps // per_call):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    # The closing barrier brackets the region but its own latency (a
    # collective, tens of us at N = 8) is not a step: each rank stops its
    # clock at its device sync and the MAX over ranks below is the job's time.
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_ms = ev0.elapsed_time(ev1) / steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(t[0]), float(t[1])

    # self-check: the planes the TIMED launches left (the last launch on each
    # bucket, the kernel instance and knobs of this run) against the oracle's digests
    want = expected_digests(job_numel, world, rank, N, P, nb)
    if want is None:
        ok, check_note, checked = True, "no committed digest for this shape: not checked", 0
    else:
        got = [planes_sha256(torch, exs[b], pls[b], N, P) for b in range(nb)]
        bad = [b for b in range(nb) if got[b] != want[b]]
        ok, checked = not bad, nb
        check_note = ("timed exponent + BE payload planes of every bucket == tests/golden/digests_bench.json"
                      if ok else f"buckets {bad} differ from tests/golden/digests_bench.json")
    ok_t = torch.tensor([int(ok), checked], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
    del xs, pls, exs, launchers
    return {"name": "strong_1GiB" if job_numel else "weak_256MiB", "job_numel": job_numel or world * N,
            "numel_per_gpu": N, "num_blocks_per_gpu": B, "alg_bytes_per_gpu": 8 * N + B, "total_alg": total_alg,
            "steps": steps, "warmup": warmup, "elapsed_s": elapsed, "kernel_ms": kern_ms_max,
            "ok": bool(ok_t[0].item()), "checked": int(ok_t[1].item()), "check_note": check_note}


def reading_block(r, world, nb, P, scaling):
    """A reading's own sub-object: rate, scaling, timing, self-check and its
    roofline (algorithmic bytes of rank 0's slice / HIP-event kernel time, max
    over ranks; PMC traffic from profiles/pmc_traffic.json at that size)."""
    ms = r["elapsed_s"] * 1e3 / r["steps"]
    ach = r["alg_bytes_per_gpu"] / (r["kernel_ms"] * 1e-3) / 1e9
    return {
        "value": round(r["total_alg"] / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "scaling": scaling,
        "n_gpus": world, "job_numel": r["job_numel"], "numel_per_gpu": r["numel_per_gpu"],
        "buckets_cycled": nb, "steps": r["steps"], "warmup": r["warmup"], "ms_per_step": round(ms, 5),
        "kernel_ms": round(r["kernel_ms"], 5),
        "self_check": r["ok"], "buckets_checked_min_over_ranks": r["checked"],
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBPS, 4),
                     "traffic": load_traffic(r["numel_per_gpu"], P, "quantize_pack" if nb == 1 else "quantize_pack_cold"),
                     "note": "per GPU: algorithmic bytes of rank 0's slice / HIP-event kernel time, max over ranks"},
    }


def readings(hl, st, world, nb, P=256):
    """The two named readings every line carries at every N,
    so a 1/2/4/8 curve compares each reading with ITSELF at N = 1:
      weak_256MiB_value   256 MiB buckets on EVERY GPU (4 cycled) — `value`
      strong_1GiB_value   configs[3]'s 1 GiB job split over the N GPUs (at
                          N = 1 the whole job on one GPU)
    `hl` / `st` are k1_reading results (st None: the strong reading skipped)."""
    out = {"weak_256MiB_value": None, "weak_256MiB": reading_block(hl, world, nb, P, "weak"),
           "readings": {
               "value": "= weak_256MiB_value (the same reading at every N; scaling weak)",
               "weak_256MiB_value": "weak scaling: every GPU quantizes its own 256 MiB buckets (4 cycled)",
               "strong_1GiB_value": "strong scaling: configs[3]'s one 1 GiB job split over the N GPUs "
                                    "(FIFO rule; the whole job on one GPU at N = 1)"}}
    out["weak_256MiB_value"] = out["weak_256MiB"]["value"]
    out["strong_1GiB_value"] = None
    if st is not None:
        out["strong_1GiB"] = reading_block(st, world, nb, P, "strong")
        out["strong_1GiB_value"] = out["strong_1GiB"]["value"]
    return out


SWITCH_PATHS = ("switchsim", "p2p_switch", "xgmi_switch", "xgmi_switch_push")


def switch_verdicts(fields, lenient=False):
    """(fatal, diagnostic) failure lines for the N > 1 switch fields.  A path
    that could not run (an error, a timeout, missing) is diagnostic.  A path
    that RAN and was not verified — outside the quantization bound, timed
    calls differing from the first, or (peer-memory paths) not bit-equal to
    switchsim — is fatal, for every path: wrong bits are a correctness
    failure.  `lenient` (bring-up only) demotes the peer-memory paths'
    mismatch to a diagnostic; switchsim's stays fatal."""
    fatal, diag = [], []
    for k in SWITCH_PATHS:
        f = fields.get(k, {})
        if "error" in f or "verified" not in f:
            diag.append(f"{k}: {f.get('error', 'not run')}")
        elif not f["verified"]:
            (diag if lenient and k != "switchsim" else fatal).append(
                f"{k}: not verified (within bound {f.get('within_quantization_bound')}, bit-equal "
                f"{f.get('bit_equal_to_switchsim', f.get('bit_equal_to_other_paths'))}, timed calls equal "
                f"{f.get('timed_calls_equal_first')})")
    return fatal, diag


def rccl_collnet_field(world, same_gpu=False, timeout=120.0):
    """RCCL's own torch.distributed all_reduce with the SwitchML plugin
    library loaded (switchml_amd/rccl_collnet.py): W worker processes, each
    its own CollNet "node" (NCCL_HOSTID), NCCL_COLLNET_ENABLE=1; RCCL's p2p
    traffic runs over the library's TCP net.  The CollNet table declines RCCL
    7.2 (its CollNet AllReduce does not reduce or hangs: DESIGN.md §9 F2), so
    RCCL falls back to its own algorithms over that net; the plugin driven by
    hand (the in-node xgmi switch behind it) is checked on the same data.
    Two workers at every N (GPUs 0 and 1 when the node has them; at N = 1
    they share the GPU): the field shows RCCL running over the plugin's net
    and the table's decision, and is kept short so the driver's N = 8 run is
    not spent on it.  Reported: correctness of RCCL's all-reduce over the
    net, the plugin's call counters, configs[4] timing."""
    try:
        from switchml_amd import rccl_collnet as R
        W = 2
        t0 = time.time()
        rep = R.launch(W, same_gpu=same_gpu, numel=1 << 22, iters=5, timeout=timeout)
        ranks = [r for r in rep["ranks"] if r]
        out = {"workers": W, "same_gpu": same_gpu, "ok": rep["ok"], "seconds": round(time.time() - t0, 1),
               "net": "SWITCHML TCP net (librccl-net-switchml.so)",
               "collnet_declined": rep["collnet_declined"],
               "collnet_dispatched_by_rccl": rep["collnet_dispatched_by_rccl"],
               "iallreduce_calls": rep["iallreduce_calls"], "returncodes": rep["returncodes"]}
        if ranks:
            out["rccl_int_allreduce_equals_exact_sum"] = all(r["int_exact"] for r in ranks)
            out["plugin_by_hand_equals_exact_sum"] = all(r.get("hand_int_exact", False) for r in ranks)
            out["plugin_by_hand_equals_rccl_on_ints"] = all(r["int_equal_direct"] for r in ranks)
            out["normal_within_quantization_bound"] = all(r["normal_within_bound"] for r in ranks)
            if all("configs4_ms_per_iter" in r for r in ranks):
                out["configs4_rccl_over_net_ms_per_iteration_max_over_ranks"] = round(
                    max(r["configs4_ms_per_iter"] for r in ranks), 3)
        if "tails" in rep:
            out["tails"] = [t[-4:] for t in rep["tails"]]
        return out
    except Exception as e:  # noqa: BLE001 - reported in the field
        return {"ok": False, "error": repr(e)[:400]}


def settle(step, settle_ms):
    """Clock settle: the first ~20-40 ms of streaming after idle run ~4 %
    slower; run the same step untimed for settle_ms first."""
    import torch
    t_settle = time.perf_counter() + settle_ms * 1e-3
    while time.perf_counter() < t_settle:
        for _ in range(10):
            step()
        torch.cuda.synchronize()


def time_launches(torch, fn, stream, reps, warm=3):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def bucket_measure(sw, torch, N, P, stream, nbuf=4, reps=200):
    """K1 with the steps cycling through nbuf distinct 256 MiB buckets and
    output planes.  nbuf = 4 (nbuf x 512 MiB >> the 256 MiB Infinity Cache):
    every launch streams from / to HBM proper (the headline's own setting).
    nbuf = 1: one bucket re-read every step, partly served by the Infinity
    Cache — reported as side.resident, labelled so."""
    B = sw.num_blocks(N, P)
    g = torch.Generator(device=stream.device)
    g.manual_seed(4242)
    xs = [torch.randn(N, device=stream.device, generator=g) for _ in range(nbuf)]
    pls = [torch.empty(B * P, dtype=torch.int32, device=stream.device) for _ in range(nbuf)]
    exs = [torch.empty(B, dtype=torch.int8, device=stream.device) for _ in range(nbuf)]
    i = [0]

    def fn():
        k = i[0]
        i[0] = (k + 1) % nbuf
        sw.quantize_pack(xs[k], P, 1, payload=pls[k], exps_out=exs[k], stream=stream)

    settle(fn, 30.0)
    t = time_launches(torch, fn, stream, reps)
    alg = 8 * N + B
    note = ("K1 cycling distinct buckets and planes: HBM-proper rate (no Infinity Cache reuse)" if nbuf > 1 else
            "K1 re-reading ONE resident bucket: HBM + Infinity Cache (part of the bucket is served by the "
            "256 MiB MALL), not an HBM fraction")
    return {"buckets": nbuf, "bucket_MiB": N * 4 >> 20, "kernel_ms": round(t * 1e3, 5),
            "achieved_GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4),
            "note": note}


def copy_ceiling(sw, torch, N, stream, nbuf=4, reps=200, k1_ms=None):
    """The practical HBM ceiling for K1's access pattern: sml_stream_copy (the
    same 1024-element tiles, XCD order, non-temporal 16-B loads and K1's store
    policy for a plane of this size — non-temporal at >= 64 MiB — no
    arithmetic) moving the same 4N read + 4N written bytes, its steps cycling
    the same number of distinct buckets as the headline."""
    g = torch.Generator(device=stream.device)
    g.manual_seed(99)
    xs = [torch.randn(N, device=stream.device, generator=g) for _ in range(nbuf)]
    ys = [torch.empty_like(x) for x in xs]
    i = [0]

    def fn():
        k = i[0]
        i[0] = (k + 1) % nbuf
        sw.stream_copy(xs[k], ys[k], stream=stream)

    settle(fn, 30.0)
    t = time_launches(torch, fn, stream, reps)
    out = {"buckets": nbuf, "kernel_ms": round(t * 1e3, 5), "GBps": round(8 * N / t / 1e9, 1),
           "frac_of_peak": round(8 * N / t / 1e9 / HBM_PEAK_GBPS, 4)}
    if k1_ms:
        out["k1_time_over_copy_time"] = round(k1_ms / (t * 1e3), 4)
    out["note"] = ("a plain copy of the same bytes in K1's tile shape and store policy, steps cycling the same buckets: "
                   "what the HBM delivers to this access pattern")
    return out


def exchange_measure(sw, torch, dist, n, P, world, rank, dev, reps=5, rehearsal=None):
    """The switch simulation with W = world real workers, each holding its
    own n-element fp32 bucket (distinct per rank).  Two exchange paths:
      switchsim   ring all-reduces (RCCL) of the int8 exponents (MAX) and the
                  host-order int32 payload (SUM, wrapping)
      p2p_switch  the payload summed at the reader from the peers' planes
                  mapped over xGMI (K6), fp32 shards all-gathered
      xgmi_switch the same switch natively in the client runtime
                  (Context::AllReduce, backend = xgmi), pull and push forms
    Verified: the two outputs are bit-identical, and both are within the
    quantization bound of an fp32 all-reduce of the same buckets.  Timed:
    max over ranks of the mean of `reps` calls.  xGMI bound: each GPU moves
    2(W-1)/W x 4n bytes over its W-1 links to the other W-1 GPUs."""
    from switchml_amd.switchsim import SwitchSimAllReduce
    from switchml_amd.p2pswitch import PeerSwitchAllReduce

    W = world
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = torch.randn(n, device=dev, generator=g) * float(2.0 ** (rank % 4 - 1))
    B = sw.num_blocks(n, P)
    bound_s = 2 * (W - 1) / W * 4 * n / ((W - 1) * XGMI_LINK_GBPS * 1e9)

    # reference sum (fp32, RCCL) and the per-element tolerance from the global exponents
    ref = x.clone()
    dist.all_reduce(ref)
    ge = sw.exponents(x, P)
    dist.all_reduce(ge, op=dist.ReduceOp.MAX)
    scale = torch.pow(2.0, ge.float()).repeat_interleave(P)[:n]
    tol = scale * (W * W * 2.0 ** -32 + W * W * 2.0 ** -23)
    del ge

    res, outs = {}, {}
    # calibration: RCCL's own fp32 all-reduce of the same buckets on this node
    # (what the switch paths compete with; same xGMI links)
    try:
        y = x.clone()
        dist.all_reduce(y)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(y)
        torch.cuda.synchronize()
        tt = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt[0])
        res["rccl_fp32_allreduce"] = {"ms_per_allreduce": round(t * 1e3, 3),
                                      "busbw_GBps": round(2 * (W - 1) / W * 4 * n / t / 1e9, 2),
                                      "frac_of_xgmi_bound": round(bound_s / t, 4)}
        del y
    except Exception as e:  # noqa: BLE001 - calibration only
        res["rccl_fp32_allreduce"] = {"error": repr(e)[:300]}

    def phase_ms(ar, call):
        """One more call with the instance's phase marks on: per-phase
        milliseconds, max over ranks (diagnostic; syncs between phases)."""
        ar.phases = {}
        call()
        ph, ar.phases = ar.phases, None
        keys = list(ph)
        d = torch.tensor([ph[b] - ph[a] for a, b in zip(keys, keys[1:])], dtype=torch.float64, device=dev)
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
        return {k: round(float(v) * 1e3, 3) for k, v in zip(keys[1:], d.tolist())}

    def agreed(fn):
        """Run fn on this rank, then learn (one all_reduce MIN) whether it
        succeeded on EVERY rank: a path that fails on one rank — its first
        contact with a peer's HBM over xGMI on a real node — is then skipped
        by all of them together, instead of leaving the others blocked in a
        collective that rank will never join (first contact).
        Returns (ok on all ranks, fn's value, this rank's exception)."""
        val, err = None, None
        try:
            val = fn()
        except Exception as e:  # noqa: BLE001 - reported in the path's field
            err = e
        t = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item()), val, err

    def failed(pipe, what, err):
        return {"error": (repr(err)[:400] if err is not None else f"{what} failed on another rank"),
                "failed_phase": what, "pipeline": pipe}

    def run_path(name, pipe, setup, call, teardown, local_teardown, with_phases):
        """One switch path through agreed phases: setup, a first call checked
        against the fp32 all-reduce, `reps` timed calls (each keeping its
        result), optional phase marks, teardown; every timed call must equal
        the first (planes are reused call after call)."""
        ok, ar, err = agreed(setup)
        if not ok:
            if ar is not None:
                # set up here but not on another rank: undo it locally (a
                # collective teardown would wait for the rank that failed)
                try:
                    local_teardown(ar)
                except Exception:  # noqa: BLE001 - the path already failed
                    pass
            res[name] = failed(pipe, "setup", err)
            return
        out = torch.empty_like(x)

        def first():
            call(ar, out)
            torch.cuda.synchronize()
            e = (out - ref).abs()
            return bool((e <= tol).all().item()), float(e.max().item())
        ok, v, err = agreed(first)
        if not ok:
            try:
                teardown(ar)
            except Exception:  # noqa: BLE001
                pass
            res[name] = failed(pipe, "first call", err)
            return
        within, max_err = v
        touts = [torch.empty_like(x) for _ in range(reps)]   # every timed call keeps its result
        dist.barrier()
        t0, terr = time.perf_counter(), None
        try:
            for i in range(reps):
                call(ar, touts[i])
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 - agreed just below, with the time
            terr = e
        tt = torch.tensor([(time.perf_counter() - t0) / reps, 1.0 if terr is not None else 0.0],
                          dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        phases = None
        if with_phases and not float(tt[1]):
            try:
                phases = phase_ms(ar, lambda: call(ar, out))
            except Exception as e:  # noqa: BLE001 - diagnostic only
                phases = {"error": repr(e)[:200]}
        try:
            teardown(ar)
        except Exception as e:  # noqa: BLE001
            terr = terr or e
        if float(tt[1]):
            res[name] = failed(pipe, "timed calls", terr)
            return
        t = float(tt[0])
        same = all(bool(torch.equal(o, out)) for o in touts)
        del touts
        ok_t = torch.tensor([int(within), int(same)], dtype=torch.int32, device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        outs[name] = out
        res[name] = {"workers": W, "numel_per_worker": n, "packet_numel": P,
                     "ms_per_allreduce": round(t * 1e3, 3), "algbw_GBps": round(4 * n / t / 1e9, 2),
                     "busbw_GBps": round(2 * (W - 1) / W * 4 * n / t / 1e9, 2),
                     "xgmi_bound_ms": round(bound_s * 1e3, 3),
                     "frac_of_xgmi_bound": round(bound_s / t, 4),
                     "within_quantization_bound": bool(ok_t[0].item()),
                     "timed_calls_equal_first": bool(ok_t[1].item()),
                     "max_abs_err_vs_fp32_allreduce": max_err, "pipeline": pipe}
        if with_phases:
            res[name]["phases_ms"] = phases

    def torch_teardown(ar):
        if hasattr(ar, "close"):
            ar.close()

    for name, cls, pipe in (
            ("switchsim", SwitchSimAllReduce,
             "K2 exps -> all_reduce(int8, MAX) -> K3 LE payload -> all_reduce(int32, SUM) -> K4"),
            ("p2p_switch", PeerSwitchAllReduce,
             "K2 exps -> all_reduce(int8, MAX) -> K3 BE payload -> K6 over the peers' planes (hipIpc, xGMI) "
             "on this rank's block shard -> all_gather(fp32)")):
        run_path(name, pipe, lambda cls=cls: cls(n, P, dev), lambda ar, o: ar(x, o), torch_teardown,
                 lambda ar: getattr(ar, "_unmap", lambda: None)(), True)
    # the native in-node switch: the client's Context with backend = xgmi
    # (C++ runtime, no torch.distributed in the data path: a failure there is
    # a barrier timeout or a poisoned session, never a hang), in its pull form
    # (K6 reads the peers' planes over xGMI) and its push form (K3 writes
    # each shard into its owner's inbox over xGMI; backend.xgmi.push)
    from switchml_amd import client as C
    for name, push in (("xgmi_switch", False), ("xgmi_switch_push", True)):
        pipe = ("Context::AllReduce, backend xgmi: K2 -> int8 max over the peers' exponent planes -> " +
                ("K3 writing each shard into its owner's inbox (hipIpc, xGMI) -> K6 on this worker's shard over "
                 "the local inbox" if push else
                 "K3 BE -> K6 on this worker's shard over the peers' planes (hipIpc, xGMI)") +
                " -> gather of the W shards")
        session = [f"bench-xgmi-{os.getpid()}-{int(time.time() * 1e3)}-{int(push)}" if rank == 0 else None]
        dist.broadcast_object_list(session, src=0)

        # SML_BENCH_INJECT=<path>:<rank> (tests only): that rank's worker fails
        # right after joining the session (backend.xgmi.fail_setup) — what a
        # failed first mapping of a peer's plane looks like to the run
        inject = os.environ.get("SML_BENCH_INJECT", "") == f"{name}:{rank}"

        def xgmi_setup(push=push, sess=session[0], inject=inject):
            if C.state() == C.RUNNING:
                C.stop()
            C.start(C.make_config(backend="xgmi", rank=rank, num_workers=W, num_worker_threads=1, packet_numel=P,
                                  max_outstanding_packets=256, mode="bulk", bandwidth=0, device=dev.index,
                                  session=sess, max_slice_numel=64 << 20, push=push, timeout_ms=60000,
                                  fail_setup=inject))
            return C

        def xgmi_teardown(_c):
            if C.state() == C.RUNNING:
                C.stop()
        run_path(name, pipe, xgmi_setup, lambda c, o: c.allreduce(x, o), xgmi_teardown, xgmi_teardown, False)
    # the three paths compute the same switch: bit-equal outputs
    paths = ("switchsim", "p2p_switch", "xgmi_switch", "xgmi_switch_push")
    names = [k for k in paths if k in outs]
    eqs = {}
    for k in names:
        if k == "switchsim" or "switchsim" not in outs:
            continue
        eq = torch.tensor([int(torch.equal(outs["switchsim"], outs[k]))], dtype=torch.int32, device=dev)
        dist.all_reduce(eq, op=dist.ReduceOp.MIN)
        eqs[k] = bool(eq.item())
    for name in paths:
        r = res[name]
        if "error" not in r:
            same = all(eqs.values()) if name == "switchsim" else eqs.get(name)
            r["bit_equal_to_switchsim" if name != "switchsim" else "bit_equal_to_other_paths"] = same
            # switchsim is the reference the other paths are checked against:
            # its own verdict does not depend on theirs (a peer-memory path's
            # mismatch is that path's failure)
            r["verified"] = bool(r["within_quantization_bound"] and r["timed_calls_equal_first"]
                                 and (name == "switchsim" or same))
        r["xgmi_link_GBps_assumed"] = XGMI_LINK_GBPS
    res["p2p_switch"]["status"] = "experimental (first cross-GPU run is the driver's multi-GPU bench)"
    label_rehearsal(res, rehearsal)
    return res


def label_rehearsal(res, rehearsal):
    """Fields a rehearsal (ranks sharing one GPU) cannot measure, marked so
    (VERDICT r5 #3): no xGMI link is crossed, so `frac_of_xgmi_bound` is
    null; the collectives ran over the SwitchML library's TCP net (or gloo),
    so rates and `phases_ms` time that net, not xGMI.  No-op on a node."""
    if not rehearsal:
        return res
    for k, r in res.items():
        if not isinstance(r, dict) or "error" in r:
            continue
        if "frac_of_xgmi_bound" in r:
            r["frac_of_xgmi_bound"] = None
        r["rehearsal_note"] = ("rehearsal (" + rehearsal + "): no xGMI link was crossed, so frac_of_xgmi_bound is "
                               "null; ms / GB/s time one shared GPU and, for the collectives, the TCP net")
        if "phases_ms" in r:
            r["phases_note"] = ("rehearsal: the all_reduce / all_gather phases ran over the SwitchML TCP net "
                                "between ranks on one GPU, not xGMI")
    return res


def extra_measurements(sw, torch, x, P, stream, reps=20):
    """Side measurements (not the headline): dequantize, fused loopback round
    trip, and a plain device copy as the practical HBM ceiling."""
    N = x.numel()
    B = sw.num_blocks(N, P)
    payload = torch.empty(B * P, dtype=torch.int32, device=x.device)
    exps = torch.empty(B, dtype=torch.int8, device=x.device)
    sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=stream)
    out = torch.empty_like(x)
    res = {}

    def timeit(fn, warm=3):
        return time_launches(torch, fn, stream, reps, warm)

    t = timeit(lambda: sw.dequantize(payload, exps, N, P, 1, out=out, stream=stream))
    res["dequantize_GBps"] = round((8 * N + B) / t / 1e9, 1)
    t = timeit(lambda: sw.roundtrip_loopback(x, P, 1, out=out, stream=stream))
    res["roundtrip_fused_GBps"] = round(8 * N / t / 1e9, 1)
    t = timeit(lambda: out.copy_(x))
    res["torch_copy_GBps"] = round(8 * N / t / 1e9, 1)
    # a FIFO slice that starts 4 bytes past a 16-B boundary (unaligned path)
    xm = x[1:]
    pm = torch.empty(sw.num_blocks(N - 1, P) * P, dtype=torch.int32, device=x.device)
    em = torch.empty(sw.num_blocks(N - 1, P), dtype=torch.int8, device=x.device)
    t = timeit(lambda: sw.quantize_pack(xm, P, 1, payload=pm, exps_out=em, stream=stream))
    res["quantize_pack_unaligned_slice_GBps"] = round((8 * (N - 1) + em.numel()) / t / 1e9, 1)
    del xm, pm, em
    # the other halves of the switch-sim pipeline: K2 (exponents only) and K3 (given global exponents)
    t = timeit(lambda: sw.exponents(x, P, out=exps, stream=stream))
    res["exponents_only_GBps"] = round((4 * N + B) / t / 1e9, 1)
    t = timeit(lambda: sw.quantize_pack(x, P, 1, global_exps=exps, payload=payload, stream=stream))
    res["quantize_global_exps_GBps"] = round((8 * N + B) / t / 1e9, 1)
    # other packet sizes: 64 (DPDK's other LTU), 1024 (RDMA message LTU)
    for Pq in (64, 1024):
        Bq = sw.num_blocks(N, Pq)
        eq = torch.empty(Bq, dtype=torch.int8, device=x.device)
        t = timeit(lambda: sw.quantize_pack(x, Pq, 1, payload=payload, exps_out=eq, stream=stream))
        res[f"quantize_pack_P{Pq}_GBps"] = round((8 * N + Bq) / t / 1e9, 1)
        t = timeit(lambda: sw.dequantize(payload, eq, N, Pq, 1, out=out, stream=stream))
        res[f"dequantize_P{Pq}_GBps"] = round((8 * N + Bq) / t / 1e9, 1)
    sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=stream)
    t = timeit(lambda: sw.loopback_aggregate(payload, 2, stream=stream))
    res["loopback_x2_GBps"] = round(8 * N / t / 1e9, 1)
    t = timeit(lambda: sw.bswap_i32(payload, out=payload, stream=stream))
    res["bswap_int32_GBps"] = round(8 * N / t / 1e9, 1)
    res.update(host_inclusive(sw, torch, x, N, P))
    # DPDK frames (F3): fused quantize straight into Eth/IP/UDP/SwitchML frames
    fp = sw.frame_params(max_outstanding_pkts=64)
    fbytes = (B + min(B, 64)) * sw.frame_bytes(P)
    frames = torch.empty(fbytes, dtype=torch.uint8, device=x.device)
    t = timeit(lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=64, frames=frames, stream=stream))
    res["frames_device_GBps"] = round((4 * N + fbytes) / t / 1e9, 1)
    # receive side: the same frames (W = 1 loopback) back to fp32; the rx
    # bitmap reset (rte_bitmap_reset per slice) is inside the timed call
    rx = sw.RxSlice(N, P, 64, device=x.device, out=out)

    def rx_once():
        rx.reset(stream)
        sw.dequantize_frames(frames, fbytes // sw.frame_bytes(P), rx, num_workers=1, stream=stream)
    with torch.cuda.stream(stream):
        t = timeit(rx_once)
    res["frames_rx_device_GBps"] = round((4 * N + fbytes) / t / 1e9, 1)
    del frames, rx
    # the same two calls cycling 4 frame sets (and rx outputs): a stream of
    # received frames, past the Infinity Cache, as the headline cycles buckets
    fsets = [torch.empty(fbytes, dtype=torch.uint8, device=x.device) for _ in range(4)]
    rxs = [sw.RxSlice(N, P, 64, device=x.device) for _ in range(4)]
    k = [0]

    def tx_cycle():
        sw.quantize_pack_frames(x, fp, P, 1, batch_max=64, frames=fsets[k[0] % 4], stream=stream)
        k[0] += 1

    def rx_cycle():
        r = rxs[k[0] % 4]
        r.reset(stream)
        sw.dequantize_frames(fsets[k[0] % 4], fbytes // sw.frame_bytes(P), r, num_workers=1, stream=stream)
        k[0] += 1
    # warm calls cover every set twice: a set's first use pays first-touch
    # costs (~130 us once), which 3 warm calls over 4 sets left in the timed
    # loop (+6 %, tools/debug/rx_bench_method_probe.py, profiles/r05)
    t = timeit(tx_cycle, warm=8)
    res["frames_device_4sets_GBps"] = round((4 * N + fbytes) / t / 1e9, 1)
    with torch.cuda.stream(stream):
        t = timeit(rx_cycle, warm=8)
    res["frames_rx_device_4sets_GBps"] = round((4 * N + fbytes) / t / 1e9, 1)
    del fsets, rxs
    # INT32 job slices over the same wire format: B frames (no extra batch),
    # payload = htonl of the words; and the receive side back to int32
    xi = x.view(torch.int32)
    fbytes_i = B * sw.frame_bytes(P)
    iframes = torch.empty(fbytes_i, dtype=torch.uint8, device=x.device)
    t = timeit(lambda: sw.pack_frames_int32(xi, fp, P, frames=iframes, stream=stream))
    res["frames_int32_device_GBps"] = round((4 * N + fbytes_i) / t / 1e9, 1)
    rxi = sw.RxSliceInt32(N, P, device=x.device)

    def rxi_once():
        rxi.reset(stream)
        sw.unpack_frames_int32(iframes, B, rxi, stream=stream)
    with torch.cuda.stream(stream):
        t = timeit(rxi_once)
    res["frames_int32_rx_device_GBps"] = round((4 * N + fbytes_i) / t / 1e9, 1)
    res["frames_int32_round_trip_exact"] = bool(torch.equal(rxi.out, xi))
    del iframes, rxi
    # the same two on 4 cycled frame sets and outputs (cold, as the FLOAT32 4-set rates)
    ifsets = [torch.empty(fbytes_i, dtype=torch.uint8, device=x.device) for _ in range(4)]
    rxis = [sw.RxSliceInt32(N, P, device=x.device) for _ in range(4)]
    k[0] = 0

    def itx_cycle():
        sw.pack_frames_int32(xi, fp, P, frames=ifsets[k[0] % 4], stream=stream)
        k[0] += 1

    def irx_cycle():
        r = rxis[k[0] % 4]
        r.reset(stream)
        sw.unpack_frames_int32(ifsets[k[0] % 4], B, r, stream=stream)
        k[0] += 1
    t = timeit(itx_cycle, warm=8)
    res["frames_int32_device_4sets_GBps"] = round((4 * N + fbytes_i) / t / 1e9, 1)
    with torch.cuda.stream(stream):
        t = timeit(irx_cycle, warm=8)
    res["frames_int32_rx_device_4sets_GBps"] = round((4 * N + fbytes_i) / t / 1e9, 1)
    res["frames_int32_4sets_exact"] = all(bool(torch.equal(r.out, xi)) for r in rxis)
    del ifsets, rxis
    hframes = torch.empty(fbytes, dtype=torch.uint8).pin_memory()
    t = timeit(lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=64, frames=hframes, stream=stream))
    res["frames_to_pinned_host_input_GBps"] = round(4 * N / t / 1e9, 2)
    # the receive side from a NIC's rx ring: returned frames in pinned host
    # memory, read by the rx kernels over PCIe, fp32 out in HBM (output bytes / s)
    hrx = sw.RxSlice(N, P, 64, device=x.device)

    def hrx_once():
        hrx.reset(stream)
        sw.dequantize_frames(hframes, fbytes // sw.frame_bytes(P), hrx, num_workers=1, stream=stream)
    with torch.cuda.stream(stream):
        t = timeit(hrx_once)
    res["frames_rx_from_pinned_host_output_GBps"] = round(4 * N / t / 1e9, 2)
    res["frames_rx_from_pinned_host_exact"] = bool(torch.equal(hrx.out.view(torch.int32),
                                                               sw.roundtrip_loopback(x, P, 1).view(torch.int32)))
    del hframes, hrx
    hi = torch.empty(fbytes_i, dtype=torch.uint8).pin_memory()
    sw.pack_frames_int32(xi, fp, P, frames=hi, stream=stream)
    hrxi = sw.RxSliceInt32(N, P, device=x.device)

    def hrxi_once():
        hrxi.reset(stream)
        sw.unpack_frames_int32(hi, B, hrxi, stream=stream)
    with torch.cuda.stream(stream):
        t = timeit(hrxi_once)
    res["frames_int32_rx_from_pinned_host_output_GBps"] = round(4 * N / t / 1e9, 2)
    res["frames_int32_rx_from_pinned_host_exact"] = bool(torch.equal(hrxi.out, xi))
    del hi, hrxi
    # K6: the switch's aggregation over W worker planes fused with the
    # dequantize (the peer-to-peer switch's compute; planes local here)
    sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=stream)
    planes = [payload] + [payload.clone() for _ in range(7)]
    eplanes = [exps] * 8
    for W in (2, 4, 8):
        t = timeit(lambda: sw.switch_aggregate(planes[:W], eplanes[:W], N, P, out=out, stream=stream))
        res[f"switch_aggregate_W{W}_GBps"] = round((W * (4 * B * P + B) + 4 * N) / t / 1e9, 1)
    agg = torch.empty_like(payload)
    t = timeit(lambda: sw.switch_aggregate(planes, None, N, P, payload_out=agg, stream=stream))
    res["switch_payload_sum_W8_GBps"] = round(9 * 4 * B * P / t / 1e9, 1)
    del planes, agg
    t = timeit(lambda: sw.stream_copy(x, out, stream=stream))
    res["nt_tile_copy_GBps"] = round(8 * N / t / 1e9, 1)
    del out
    res["configs4_plugin"] = plugin_buckets(torch, x.device)
    return res


RESNET50_BUCKETS = [6_553_600, 6_553_600, 6_553_600, 5_896_232]   # DDP 25 MiB buckets of 25,557,032 fp32


def plugin_measure_ranks(torch, dist, dev, world):
    """configs[4] at N GPUs: every rank hands the ResNet-50 buckets to its
    CollNet plugin instance at once, on an N-rank communicator whose backend
    is the in-node switch (general.backend = xgmi): a real SwitchML
    all-reduce across the N GPUs over xGMI.  Reported: max-over-ranks ms per
    iteration, device and pinned host buffers (the H<->D-inclusive rate), and
    aggregate elements/s = N x params / t."""
    rank = dist.get_rank()
    session = [f"bench-cfg4-{os.getpid()}-{int(time.time() * 1e3)}" if rank == 0 else None]
    dist.broadcast_object_list(session, src=0)
    ini = ("[general]\nbackend = xgmi\nrank = %d\nnum_workers = %d\nnum_worker_threads = 4\npacket_numel = 256\n"
           "max_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = bulk\ndevice = %d\n"
           "[backend.xgmi]\nsession = %s\n" % (rank, world, dev.index, session[0]))
    dist.barrier()
    # a failure on one rank (its first xGMI contact) is agreed on by all of
    # them in the one collective that follows, instead of leaving the others
    # waiting in it (the plugin's own exchange fails by its barrier timeout)
    r, err = None, None
    try:
        r = plugin_buckets(torch, dev, ini=ini, nranks=world, rank=rank)
    except Exception as e:  # noqa: BLE001 - agreed below, reported by the caller
        err = e
    t = torch.tensor([r["device"]["ms_per_iteration"] if r else 0.0, r["pinned_host"]["ms_per_iteration"] if r else 0.0,
                      0.0 if (r and r["placements_agree"]) else 1.0, 1.0 if r is None else 0.0],
                     dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if float(t[3]):
        raise RuntimeError(repr(err)[:300] if err is not None else "configs4_plugin failed on another rank")
    out = {k: r[k] for k in ("buckets", "params", "num_workers", "num_worker_threads", "packet_numel", "backend")}
    out["ranks"] = world
    for i, name in enumerate(("device", "pinned_host")):
        ms = float(t[i])
        out[name] = {"ms_per_iteration_max_over_ranks": round(ms, 4),
                     "aggregate_elements_per_s": round(world * r["params"] / (ms * 1e-3), 1),
                     "aggregate_fp32_GBps": round(world * 4 * r["params"] / (ms * 1e-3) / 1e9, 2)}
    out["placements_agree_all_ranks"] = float(t[2]) == 0.0
    out["note"] = ("CollNet iallreduce/test on an N-rank communicator, backend xgmi (the in-node switch: "
                   "exponent max, K3, K6 over the peers' planes, gather); pinned_host = H<->D-inclusive rate")
    return out


def plugin_buckets(torch, dev, iters=10, ini=None, nranks=1, rank=0):
    """configs[4]: ResNet-50-sized gradient buckets handed to the RCCL CollNet
    plugin's iallreduce and polled with test() (switchml_plugin.cc:293-387),
    all four buckets in flight per iteration, as RCCL's proxy posts them.
    Placements: device buffers (ptrSupport CUDA: the HIP quantizer works in
    place in HBM) and pinned host buffers (what the reference's HOST-only
    plugin is handed; read and written by the kernels over PCIe).
    Backend: the loopback (W = 8, T = 4, fused round trip) unless `ini`
    names another (the in-node switch at N > 1)."""
    import numpy as np
    if ini is None:
        ini = ("[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\nmax_outstanding_packets = 256\n"
               "[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\n")
        os.environ["SWITCHML_COLLNET_LOOPBACK"] = "1"
    os.environ["SWITCHML_CONFIG_INI"] = ini
    from switchml_amd import client as C
    from switchml_amd.collnet import CollNetComm, NCCL_FLOAT32
    if C.state() == C.RUNNING:
        C.stop()
    comm = CollNetComm(nranks=nranks, rank=rank)
    g = torch.Generator(device=dev)
    g.manual_seed(7 + rank)
    dsend = [torch.randn(n, device=dev, generator=g) * 1e-3 for n in RESNET50_BUCKETS]
    drecv = [torch.empty_like(d) for d in dsend]
    hsend = [d.cpu().pin_memory() for d in dsend]
    hrecv = [torch.empty_like(h).pin_memory() for h in hsend]
    total = sum(RESNET50_BUCKETS)
    cfg = C.config_text()
    res = {"buckets": RESNET50_BUCKETS, "params": total,
           "num_workers": int(cfg.split("num_workers = ")[1].split()[0]),
           "num_worker_threads": int(cfg.split("num_worker_threads = ")[1].split()[0]),
           "packet_numel": 256, "backend": cfg.split("backend = ")[1].split()[0],
           "mode": cfg.split("mode = ")[1].split()[0]}
    for name, snd, rcv in (("device", dsend, drecv), ("pinned_host", hsend, hrecv)):
        jobs = [(s.data_ptr(), r.data_ptr(), s.numel()) for s, r in zip(snd, rcv)]
        comm.allreduce_buckets(jobs, NCCL_FLOAT32)
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            comm.allreduce_buckets(jobs, NCCL_FLOAT32)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        res[name] = {"ms_per_iteration": round(t * 1e3, 4), "elements_per_s": round(total / t, 1),
                     "fp32_GBps": round(4 * total / t / 1e9, 2)}
    res["placements_agree"] = all(bool(torch.equal(r.cpu(), h)) for r, h in zip(drecv, hrecv))
    comm.close()
    C.stop()
    return res


def host_inclusive(sw, torch, x, N, P, chunk=8 * 1024 * 1024, reps=5):
    """The path as the reference runs it: the bucket starts in (pinned) host
    memory — a DPDK mbuf / RDMA buffer — and the packets end there.  Timed:
    H2D of the fp32 bucket, K1 quantize+pack, D2H of payload + exponents.
    'serial' = one stream; 'pipelined' = chunks of `chunk` elements on three
    streams (H2D / kernel / D2H overlap; PCIe is full duplex).  Rates are fp32
    input bytes per second (4N / t)."""
    dev = x.device
    hx = torch.empty(N, dtype=torch.float32, pin_memory=True)
    hx.copy_(x.cpu())
    B = sw.num_blocks(N, P)
    hp = torch.empty(B * P, dtype=torch.int32, pin_memory=True)
    he = torch.empty(B, dtype=torch.int8, pin_memory=True)
    dx = torch.empty_like(x)
    dp = torch.empty(B * P, dtype=torch.int32, device=dev)
    de = torch.empty(B, dtype=torch.int8, device=dev)
    s0 = torch.cuda.current_stream()

    def serial():
        dx.copy_(hx, non_blocking=True)
        sw.quantize_pack(dx, P, 1, payload=dp, exps_out=de, stream=s0)
        hp.copy_(dp, non_blocking=True)
        he.copy_(de, non_blocking=True)

    sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    assert chunk % P == 0 and N % chunk == 0

    def pipelined():
        for c in range(N // chunk):
            lo, hi = c * chunk, (c + 1) * chunk
            blo, bhi = lo // P, hi // P
            with torch.cuda.stream(sa):
                dx[lo:hi].copy_(hx[lo:hi], non_blocking=True)
                e1 = torch.cuda.Event()
                e1.record(sa)
            sb.wait_event(e1)
            sw.quantize_pack(dx[lo:hi], P, 1, payload=dp[lo:hi], exps_out=de[blo:bhi], stream=sb)
            e2 = torch.cuda.Event()
            e2.record(sb)
            sc.wait_event(e2)
            with torch.cuda.stream(sc):
                hp[lo:hi].copy_(dp[lo:hi], non_blocking=True)
                he[blo:bhi].copy_(de[blo:bhi], non_blocking=True)

    dring = [torch.empty(chunk, dtype=torch.float32, device=dev) for _ in range(2)]
    copy_done = [torch.cuda.Event() for _ in range(2)]
    kern_done = [torch.cuda.Event() for _ in range(2)]

    def hybrid():
        # input over PCIe by the copy engine (H2D, chunked into a 2-slot HBM
        # ring), output by the kernel's own stores straight into the pinned
        # host planes (D2H direction): the two PCIe directions overlap.
        for c in range(N // chunk):
            lo, hi = c * chunk, (c + 1) * chunk
            blo, bhi = lo // P, hi // P
            r = c % 2
            with torch.cuda.stream(sa):
                if c >= 2:
                    sa.wait_event(kern_done[r])
                dring[r].copy_(hx[lo:hi], non_blocking=True)
                copy_done[r].record(sa)
            sb.wait_event(copy_done[r])
            sw.quantize_pack(dring[r], P, 1, payload=hp[lo:hi], exps_out=he[blo:bhi], stream=sb)
            kern_done[r].record(sb)

    def zero_copy():
        # K1 reads the pinned host bucket and writes the pinned host planes
        # directly over PCIe (host memory is device-accessible under HIP's
        # unified addressing): one pass, both PCIe directions at once.
        sw.quantize_pack(hx, P, 1, payload=hp, exps_out=he, stream=s0)

    ref_head = sw.quantize_pack(x[: 4 * P], P, 1)[0]
    ref_tail = sw.quantize_pack(x[N - 4 * P:], P, 1)[0]
    ref_e = sw.exponents(x, P)
    out = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined), ("hybrid", hybrid), ("zero_copy", zero_copy)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        out[f"host_inclusive_{name}_input_GBps"] = round(4 * N / t / 1e9, 2)
        if name != "serial":   # every variant leaves the same planes in hp / he
            tail = slice(N - 4 * P, N)
            ok_v = bool(torch.equal(hp[: 4 * P].to(dev), ref_head)) and bool(torch.equal(hp[tail].to(dev), ref_tail))
            ok_v = ok_v and bool(torch.equal(he.to(dev), ref_e))
            out["host_inclusive_check"] = out.get("host_inclusive_check", True) and ok_v
        hp.zero_()
        he.zero_()
    return out


if __name__ == "__main__":
    main()
