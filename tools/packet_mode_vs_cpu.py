#!/usr/bin/env python3
"""The per-packet path against the reference's CPU per-packet loop, same job,
same box.

GPU: bin/allreduce_benchmark in packet mode — the loopback backend driving
the HIP PPP through its per-LTU interface (PreprocessSingle/PostprocessSingle
semantics, one exchange burst per ring pass: csrc/client/loopback_backend.cc
run_packet_loop) — 64 MiB fp32, T = 4 worker threads, W = 2, device ring and
pinned host ring.
CPU: the oracle's restatement of the reference's DummyWorkerThread loop with
the reference's default build (VCL=1), T = 4 threads, the same job (pre +
ProcessPacket + post for every packet: the whole round trip), and the
preprocess-only rate bench.py's cpu_baseline reports as
ref_default_4_threads_value.  Rates in the bench's unit: (8N + B) / t.

Usage: python tools/packet_mode_vs_cpu.py OUT.json"""
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def median(v):
    v = sorted(v)
    return v[len(v) // 2]


def gpu_packet_mode(numel, T, W, jobs=7):
    """packet: HBM ring, one exchange launch per ring pass (ProcessPacket +
    post + pre); packet_pinned_ring: the ring in pinned host memory (a NIC's
    mbuf pool: ProcessPacket on the CPU, one exchange launch per pass, read
    and written over PCIe, host sync per burst)."""
    import tempfile
    exe = os.path.join(ROOT, "p4app-switchml_amd", "bin", "allreduce_benchmark")
    res = {}
    with tempfile.NamedTemporaryFile("w", suffix=".cfg", delete=False) as f:
        f.write("[backend.hip]\npacket_ring = pinned\n")
        pinned_cfg = f.name
    with tempfile.NamedTemporaryFile("w", suffix=".cfg", delete=False) as f:
        f.write("[backend.hip]\npacket_ring = pinned\nburst_server = true\n")
        server_cfg = f.name
    for name, mode, extra in (("packet", "packet", []), ("packet_pinned_ring", "packet", ["--config", pinned_cfg]),
                              ("packet_pinned_ring_burst_server", "packet", ["--config", server_cfg]),
                              ("bulk", "bulk", []), ("fused", "fused", [])):
        r = subprocess.run([exe, "--tensor-numel", str(numel), "--tensor-type", "float", "--num-workers", str(W),
                            "--num-worker-threads", str(T), "--bandwidth", "0", "--device", "gpu", "--mode", mode,
                            "--num-jobs", str(jobs), "--num-warmup-jobs", "2", "--verify", "true"] + extra,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "Data verified successfully" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
        ns = [int(m) for m in re.findall(r"Duration: #(\d+)# ns", r.stdout)]
        res[name] = {"median_ms": median(ns) / 1e6, "jobs": len(ns)}
    os.unlink(pinned_cfg)
    os.unlink(server_cfg)
    return res


def cpu_reference(numel, T, W, P=256, reps=5):
    import numpy as np
    from oracle import oracle as O
    x = O.splitmix_normal(42, numel)
    out = np.empty_like(x)
    res = {}
    for name, mode in (("roundtrip", O.MODE_ROUNDTRIP), ("preprocess_only", O.MODE_PREPROCESS)):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            O.dummy_allreduce(x, P=P, max_outstanding_packets=256, num_worker_threads=T, num_workers=W,
                              threaded=T > 1, mode=mode, out=out, vcl=True)
            ts.append(time.perf_counter() - t0)
        res[name] = {"median_ms": median(ts) * 1e3}
    return res


def main():
    numel, T, W, P = 16 * 1024 * 1024, 4, 2, 256
    alg = 8 * numel + (numel + P - 1) // P
    g = gpu_packet_mode(numel, T, W)
    c = cpu_reference(numel, T, W)
    for d in (g, c):
        for k, v in d.items():
            v["GBps_8N_plus_B"] = round(alg / (v["median_ms"] * 1e-3) / 1e9, 2)
    out = {"job": f"{numel * 4 >> 20} MiB fp32, T={T} worker threads, W={W}, P={P}, max_outstanding_packets=256",
           "gpu_allreduce_benchmark": g, "cpu_reference_vcl1_T4": c,
           "packet_mode_vs_cpu_roundtrip": round(c["roundtrip"]["median_ms"] / g["packet"]["median_ms"], 3),
           "packet_mode_vs_cpu_preprocess_only": round(c["preprocess_only"]["median_ms"] / g["packet"]["median_ms"], 3),
           "pinned_ring_vs_cpu_roundtrip": round(c["roundtrip"]["median_ms"] /
                                                 g["packet_pinned_ring"]["median_ms"], 3),
           "pinned_ring_burst_server_vs_cpu_roundtrip": round(c["roundtrip"]["median_ms"] /
                                                              g["packet_pinned_ring_burst_server"]["median_ms"], 3),
           "note": ("GPU packet mode = the whole all-reduce (per-packet ProcessPacket + post + pre through the "
                    "HIP PPP's exchange bursts: PostprocessReuseBurst, one launch per pass over the b-slot ring; "
                    "device ring, and a pinned host ring like a NIC's mbuf pool); CPU = the oracle's restatement "
                    "of the reference's VCL=1 per-packet loop on this host, same job")}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
