#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X:
"fp32->int32 quantize+pack GB/s (device-resident), 256 MiB bucket, 1/2/4/8 GPU".

One step = one pass of the hot path (CpuExponentQuantizerPPP's
PreprocessSingle over a whole job slice: per-packet exponent, fp32->int32
scale+round, big-endian pack — ppp.cc:69-156) over one 256 MiB fp32 bucket
that is already resident in HBM, as one launch of the fused HIP kernel
sml_quantize_pack (K1).  Exponents are the loopback's (the dummy backend
returns them unchanged, so the local exponent is the global one: W = 1).

Multi-GPU (launched by torch.distributed.run): "sharding mode" — every rank
owns its own 256 MiB slice of a G x 256 MiB job (FifoScheduler slicing,
fifo_scheduler.cc:93-109, slice g -> GPU g); the path has no exchange step
at W = 1, so there is no collective in the timed region (weak scaling).
value = all ranks' algorithmic bytes / max-over-ranks time.

Units: value / roofline.achieved = ALGORITHMIC bytes per second: 4N read
(fp32 in) + 4N written (int32 payload) + B written (int8 exponents),
B = N/256 — see DESIGN.md §4.  input_GBps = 4N / t is reported alongside.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="untimed launches of the same step for this long before the warmup steps "
                         "(HBM/fabric clocks ramp under load: profiles/r01/bench_warmup_sweep.jsonl)")
    ap.add_argument("--numel", type=int, default=64 * 1024 * 1024, help="fp32 elements per GPU (256 MiB)")
    ap.add_argument("--packet-numel", type=int, default=256)
    ap.add_argument("--job-numel", type=int, default=0,
                    help="strong scaling: one job of this many fp32 elements split over the ranks by the FIFO "
                         "rule (configs[3]: 268435456 = 1 GiB); 0 = --numel per GPU (weak scaling, default)")
    ap.add_argument("--grid-limit", type=int, default=0, help="workgroups per launch (0 = one per 4 tiles)")
    ap.add_argument("--xcd-chunk", type=int, default=64,
                    help="workgroups per contiguous run on one XCD (0 = plain blockIdx order)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--extra", action="store_true", help="also time dequantize / fused round trip / copy")
    ap.add_argument("--p2p", action="store_true",
                    help="N > 1: also time the peer-to-peer switch (K6 over the peers' HBM, hipIpc)")
    ap.add_argument("--graph-steps", type=int, default=1,
                    help="capture this many steps per hipGraph replay (1 = eager launches)")
    return ap.parse_args()


def load_traffic(numel, P):
    """HBM bytes per launch from the PMC passes (profiles/pmc_traffic.json,
    written by profiles/collect_pmc.py from separate rocprofv3 --pmc runs)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        k = d.get("quantize_pack", {})
        if k.get("numel") == numel and k.get("packet_numel") == P:
            return k.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(numel, P, budget_s):
    """The oracle's restatement of the reference CPU path (per-packet
    PreprocessSingle calls in DummyWorkerThread order, b = mop/T ring) on this
    host's cores, over the same 256 MiB bucket, repeated for ~budget_s.

    `value` is the reference's DEFAULT build, VCL=1 (client_lib/Makefile:26,
    113-120): its 16-element vector loops restated with SSE2 intrinsics — the
    instruction set that build targets (no -m flags) — on all cores used.  The
    scalar VCL=0 path (roundf per element) is reported beside it."""
    import numpy as np
    from oracle import oracle as O

    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    cores = max(1, min(cores, 16))
    x = O.splitmix_normal(42, numel)
    out = np.empty_like(x)
    alg = 8 * numel + O.num_blocks(numel, P)

    def run(T, deadline_s, min_reps, vcl):
        rates, t_end, reps = [], time.perf_counter() + deadline_s, 0
        while reps < min_reps or time.perf_counter() < t_end:
            t0 = time.perf_counter()
            O.dummy_allreduce(x, P=P, max_outstanding_packets=256, num_worker_threads=T,
                              num_workers=1, threaded=T > 1, mode=O.MODE_PREPROCESS, out=out, vcl=vcl)
            rates.append(alg / (time.perf_counter() - t0) / 1e9)
            reps += 1
        return float(np.median(rates)), reps

    multi, repsT = run(cores, budget_s * 0.35, 3, True)
    four, reps4 = run(4, budget_s * 0.1, 3, True) if cores > 4 else (None, 0)
    single, reps1 = run(1, budget_s * 0.1, 2, True)
    s_multi, s_repsT = run(cores, budget_s * 0.25, 3, False)
    s_single, s_reps1 = run(1, budget_s * 0.2, 2, False)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), model)
    except OSError:
        pass
    return {
        "value": round(multi, 3),
        "unit": "GB/s (8N+B algorithmic bytes, same as value)",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle/sml_oracle.c restatement of CpuExponentQuantizerPPP as the reference builds it by "
                   f"default (VCL=1, vector loops in SSE2), driven in DummyWorkerThread order, PreprocessSingle "
                   f"only (exponent + quantize + BE pack into the b-packet ring), the full {numel * 4 >> 20} MiB "
                   f"bucket, packet_numel {P}, max_outstanding_packets 256; {cores} worker threads x {repsT} reps "
                   f"(median); 1 thread: {single:.3f} GB/s; scalar VCL=0 build: {s_multi:.3f} GB/s on {cores} "
                   f"threads, {s_single:.3f} on 1; host CPU {model}"),
        "single_thread_value": round(single, 3),
        "ref_default_4_threads_value": None if four is None else round(four, 3),
        "vcl0_scalar_value": round(s_multi, 3),
        "vcl0_scalar_single_thread_value": round(s_single, 3),
        "cpu_model": model,
        "input_GBps": round(multi * 4 * numel / alg, 3),
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import switchml_amd as sw

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SML_BENCH_REHEARSE=1: rehearse the N>1 path on a 1-GPU box (all ranks on
    # device local % device_count, gloo instead of RCCL).  Never used for numbers.
    rehearse = os.environ.get("SML_BENCH_REHEARSE") == "1"
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if rehearse else local
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    sw.lib()
    if args.grid_limit:
        sw.set_grid_limit(args.grid_limit)
    sw.set_xcd_chunk(args.xcd_chunk)

    P = args.packet_numel
    if args.job_numel:
        # configs[3]: one job sharded over the ranks, slice g -> GPU g (fifo_scheduler.cc:93-109)
        N = sw.fifo_slice(args.job_numel, world, rank)[1]
        total_alg = sum(8 * n + sw.num_blocks(n, P)
                        for n in (sw.fifo_slice(args.job_numel, world, r)[1] for r in range(world)))
    else:
        N = args.numel
        total_alg = world * (8 * N + sw.num_blocks(N, P))
    B = sw.num_blocks(N, P)
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    x = torch.randn(N, dtype=torch.float32, device=dev, generator=gen)
    payload = torch.empty(B * P, dtype=torch.int32, device=dev)
    exps = torch.empty(B, dtype=torch.int8, device=dev)
    stream = torch.cuda.current_stream()
    alg_bytes = 8 * N + B

    def launch():
        sw.quantize_pack(x, P, 1, payload=payload, exps_out=exps, stream=torch.cuda.current_stream())

    step, per_call = launch, 1
    if args.graph_steps > 1:
        # G consecutive steps captured into one hipGraph (G kernel nodes, the
        # same launch each time): the Python/ctypes launch path leaves the
        # timed loop; each replay still runs exactly G full steps.
        launch()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(args.graph_steps):
                launch()
        step, per_call = graph.replay, args.graph_steps
        assert args.steps % per_call == 0 and args.warmup % per_call == 0, "steps/warmup must be multiples of --graph-steps"

    # Clock settle: the first ~20-40 ms of streaming after idle run ~4 % slower
    # (warmup 10 -> 78-79 us per launch, >= 500 -> 76 us); run the same step
    # untimed for settle_ms first so the K timed steps see steady-state clocks
    # whatever W the caller passes.
    t_settle = time.perf_counter() + args.settle_ms * 1e-3
    while time.perf_counter() < t_settle:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup // per_call):
        step()
    torch.cuda.synchronize()

    # Timed region: K back-to-back launches on `stream`, bracketed by a barrier
    # and a device sync on both sides (wall clock -> value), and by two HIP
    # events recorded on the launch stream itself (-> average launch duration
    # for the roofline; includes the inter-launch gaps, so it is conservative
    # against rocprofv3's per-dispatch durations).  Per-launch event pairs
    # were measured to add ~4 us per launch and are not used.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps // per_call):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(t[0]), float(t[1])

    # sanity: the timed output is the HIP kernel's and it is deterministic
    ok = bool(torch.equal(exps[:4].cpu(), sw.exponents(x[:4 * P], P).cpu()))

    extra = {}
    if world > 1 or args.extra:
        # Switch-sim mode (not the headline): W = world workers all-reduce their
        # buckets through K2 -> RCCL int8 MAX -> K3 -> RCCL int32 SUM -> K4.
        try:
            extra["switchsim"] = switchsim_measure(sw, torch, dist, x, N, P, world, dev)
        except Exception as e:  # reported, never fatal to the headline line
            extra["switchsim"] = {"error": repr(e)[:300]}
        if args.p2p and world > 1:
            # peer-to-peer switch (opt-in): K6 reads the peers' planes over xGMI
            try:
                from switchml_amd.p2pswitch import PeerSwitchAllReduce
                extra["p2p_switch"] = switchsim_measure(
                    sw, torch, dist, x, N, P, world, dev, cls=PeerSwitchAllReduce,
                    pipeline="K2 exps -> all_reduce(int8, MAX) -> K3 BE payload -> K6 over peers' planes "
                             "(hipIpc, xGMI) on this rank's block shard -> all_gather(fp32)")
            except Exception as e:
                extra["p2p_switch"] = {"error": repr(e)[:300]}
    if args.extra and rank == 0:
        extra.update(extra_measurements(sw, torch, x, payload, exps, N, P, stream))

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = total_alg / (elapsed / args.steps) / 1e9
        achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
        line = {
            "metric": "fp32→int32 quantize+pack GB/s (device-resident), 256 MiB bucket, 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if args.job_numel else "weak",
            "vs_baseline": None,
            "dtype": "f32->i32",
            "data": "synthetic N(0,1) fp32 (torch.randn on device, seed 42+rank)",
            "config": {
                "workload": (f"configs[3]-style job: {args.job_numel * 4 >> 20} MiB fp32 sharded over {world} GPU(s) "
                             "by the FIFO rule, fused exponent+quantize+BE pack (sml_quantize_pack, K1), loopback "
                             "exponents (W=1)") if args.job_numel else
                            ("configs[2]-sized bucket: 256 MiB fp32 per GPU, fused exponent+quantize+BE pack "
                             "(sml_quantize_pack, K1), loopback exponents (W=1)"),
                "numel_per_gpu": N,
                "packet_numel": P,
                "num_blocks_per_gpu": B,
                "parallelism": f"shard{world} (FIFO slices, no data-path collective)",
                "bytes_per_step_per_gpu": alg_bytes,
                "xcd_chunk": args.xcd_chunk,
                "launch": "eager" if args.graph_steps <= 1 else f"hipGraph replay, {args.graph_steps} steps per graph",
            },
            "input_GBps": round(4 * (args.job_numel or world * N) / (elapsed / args.steps) / 1e9, 2),
            "kernel_ms": round(kern_ms_max, 5),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic(N, P),
                "kernel": f"sml::k_quantize_pack<{P},aligned,fused,BE,half-away>",
            },
            "self_check": ok,
        }
        if extra:
            line["extra"] = extra
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(N, P, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def switchsim_measure(sw, torch, dist, x, N, P, world, dev, reps=5, cls=None,
                      pipeline="K2 exps -> all_reduce(int8, MAX) -> K3 LE payload -> all_reduce(int32, SUM) -> K4"):
    """Time a switch-sim all-reduce of the same 256 MiB bucket per GPU
    (switchml_amd/switchsim.py, or the peer-to-peer switch); max over ranks.
    algbw = 4N / t."""
    from switchml_amd.switchsim import SwitchSimAllReduce
    if world == 1 and not dist.is_initialized():
        return {"note": "single rank: no exchange to time"}
    ar = (cls or SwitchSimAllReduce)(N, P, dev)
    out = torch.empty_like(x)
    ar(x, out)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        ar(x, out)
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t = float(t[0])
    if hasattr(ar, "close"):
        ar.close()
    return {"workers": world, "ms_per_allreduce": round(t * 1e3, 3), "algbw_GBps": round(4 * N / t / 1e9, 2),
            "pipeline": pipeline}


def extra_measurements(sw, torch, x, payload, exps, N, P, stream, reps=20):
    """Side measurements (not the headline): dequantize, fused loopback round
    trip, and a plain device copy as the practical HBM ceiling."""
    out = torch.empty_like(x)
    res = {}

    def timeit(fn):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e-3

    B = exps.numel()
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
        rx.state.zero_()
        sw.dequantize_frames(frames, fbytes // sw.frame_bytes(P), rx, num_workers=1, stream=stream)
    with torch.cuda.stream(stream):
        t = timeit(rx_once)
    res["frames_rx_device_GBps"] = round((4 * N + fbytes) / t / 1e9, 1)
    del frames, rx
    hframes = torch.empty(fbytes, dtype=torch.uint8).pin_memory()
    t = timeit(lambda: sw.quantize_pack_frames(x, fp, P, 1, batch_max=64, frames=hframes, stream=stream))
    res["frames_to_pinned_host_input_GBps"] = round(4 * N / t / 1e9, 2)
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
        evs = []
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
            evs.append(e2)

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
