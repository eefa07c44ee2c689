"""bench.py's self-check: the timed buckets come from an
integer-exact generator restated in bench.py (bench_bucket), and the planes
the timed K1 launches leave are compared with oracle digests committed in
tests/golden/digests_bench.json (made by tests/golden/make_bench_digests.py).
CPU: the restatement equals oracle.splitmix_grad (any seed, any offset), and
the committed N = 1 digest of bucket 0 is the oracle's.  GPU: the same
generator on the device, and K1 over the first bench bucket hashing to the
committed digest."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402

DIGESTS = os.path.join(ROOT, "tests", "golden", "digests_bench.json")


@pytest.mark.parametrize("seed,off,n", [(4242, 0, 100_000), (4245, 123_457, 70_001), (0, 1 << 33, 5000),
                                        (2 ** 40 + 3, 67_108_864 - 777, 2000)])
def test_bench_generator_is_oracle_splitmix_grad(seed, off, n):
    import torch
    got = bench.bench_bucket(torch, seed, off, n, "cpu").numpy()
    if off < (1 << 32):
        ref = O.splitmix_grad(seed, off + n)[off:]
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    # restated in numpy at the global index directly (offsets past what fits in memory)
    i = np.arange(off, off + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed * 0x9E3779B97F4A7C15 % 2 ** 64) + i * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(31))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(29))
    mant = (z >> np.uint64(40)).astype(np.int64) - (1 << 23)
    k = ((i >> np.uint64(8)) * np.uint64(7) + (z & np.uint64(1))) % np.uint64(16)
    ref2 = np.ldexp(mant.astype(np.float32), -(24 + k.astype(np.int32))).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), ref2.view(np.uint32))


def test_bench_digests_shape_and_bucket0():
    with open(DIGESTS) as f:
        d = json.load(f)
    assert d["packet_numel"] == 256 and d["buckets"] == 4 and d["seed0"] == bench.BENCH_SEED0
    assert len(d["bucket_T1"]) == 4
    assert sorted(d["job"]) == ["T1", "T2", "T4", "T8"]
    for G in (1, 2, 4, 8):
        assert [len(r) for r in d["job"][f"T{G}"]] == [G] * 4
    # T = 4 slice 0 of the job IS the N = 1 bucket (same seed, elements [0, 2^26))
    assert d["job"]["T4"][0][0] == d["bucket_T1"][0]
    x = O.splitmix_grad(d["seed0"], d["bucket_numel"])
    e, q = O.exponents(x, 256), O.quantize(x, 256, 1)
    assert hashlib.sha256(e.tobytes()).hexdigest() == d["bucket_T1"][0]["exps"]
    assert hashlib.sha256(q.tobytes()).hexdigest() == d["bucket_T1"][0]["payload"]
    assert bench.expected_digests(0, 1, 0, d["bucket_numel"], 256, 4) == d["bucket_T1"]
    assert bench.expected_digests(d["job_numel"], 8, 5, 0, 256, 4) == [d["job"]["T8"][b][5] for b in range(4)]
    assert bench.expected_digests(0, 1, 0, d["bucket_numel"], 64, 4) is None
    # the headline at N > 1: every GPU holds the same 4 buckets -> bucket_T1 on every rank
    assert bench.expected_digests(0, 8, 7, d["bucket_numel"], 256, 4) == d["bucket_T1"]
    # the strong reading at N = 1: the whole 1 GiB job on one GPU
    assert bench.expected_digests(d["job_numel"], 1, 0, d["job_numel"], 256, 4) == [d["job"]["T1"][b][0]
                                                                                   for b in range(4)]


@pytest.mark.gpu
def test_bench_bucket_on_gpu_hashes_to_digest(cuda):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
    import switchml_amd as sw
    with open(DIGESTS) as f:
        d = json.load(f)
    small = bench.bench_bucket(torch, 4243, 1000, 300_000, cuda).cpu().numpy()
    assert np.array_equal(small.view(np.uint32), O.splitmix_grad(4243, 301_000)[1000:].view(np.uint32))
    N = d["bucket_numel"]
    for b in (0, 3):
        x = bench.bench_bucket(torch, d["seed0"] + b, 0, N, cuda)
        B = sw.num_blocks(N, 256)
        pl = torch.empty(B * 256, dtype=torch.int32, device=cuda)
        ex = torch.empty(B, dtype=torch.int8, device=cuda)
        sw.quantize_pack(x, 256, 1, payload=pl, exps_out=ex)
        torch.cuda.synchronize()
        assert bench.planes_sha256(torch, ex, pl, N, 256) == d["bucket_T1"][b]


def test_switch_verdicts_wrong_bits_fatal_for_every_path():
    """bench.py's N > 1 switch checks: a path that RAN and is
    not verified fails the run, whichever path it is; a path that could not
    run (error, timeout, missing) is diagnostic; --lenient-switch demotes
    only the peer-memory paths' mismatch."""
    ok = {"verified": True, "within_quantization_bound": True, "timed_calls_equal_first": True}
    bad = {"verified": False, "within_quantization_bound": True, "timed_calls_equal_first": True,
           "bit_equal_to_switchsim": False}
    fields = {"switchsim": ok, "p2p_switch": bad, "xgmi_switch": {"error": "boom"}, "xgmi_switch_push": ok}
    fatal, diag = bench.switch_verdicts(fields)
    assert len(fatal) == 1 and fatal[0].startswith("p2p_switch: not verified") and len(diag) == 1
    assert diag[0].startswith("xgmi_switch: ") and "boom" in diag[0]
    for k in ("xgmi_switch", "xgmi_switch_push"):
        f2 = dict(fields, p2p_switch=ok, **{k: dict(bad, timed_calls_equal_first=False)})
        fatal, diag = bench.switch_verdicts(f2)
        assert [x.split(":")[0] for x in fatal] == [k]
    fatal, diag = bench.switch_verdicts(fields, lenient=True)
    assert fatal == [] and len(diag) == 2
    fatal, _ = bench.switch_verdicts(dict(fields, switchsim=dict(bad, bit_equal_to_other_paths=False)),
                                     lenient=True)
    assert len(fatal) == 1 and fatal[0].startswith("switchsim")
    fatal, diag = bench.switch_verdicts({})
    assert fatal == [] and len(diag) == 4
    fatal, diag = bench.switch_verdicts({k: ok for k in bench.SWITCH_PATHS})
    assert fatal == [] and diag == []


def _reading(name, job_numel, world, n, elapsed_s, kernel_ms, steps=20, ok=True):
    """A synthetic k1_reading result (bench.py) of rank 0's slice `n`."""
    B = -(-n // 256)
    slices = ([n] * world if job_numel == 0 else
              [-(-job_numel // world) if g < job_numel % world else job_numel // world for g in range(world)])
    return {"name": name, "job_numel": job_numel or world * n, "numel_per_gpu": n, "num_blocks_per_gpu": B,
            "alg_bytes_per_gpu": 8 * n + B, "total_alg": sum(8 * m + -(-m // 256) for m in slices),
            "steps": steps, "warmup": 10, "elapsed_s": elapsed_s, "kernel_ms": kernel_ms, "ok": ok,
            "checked": 4, "check_note": "x"}


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_every_line_names_the_same_two_readings(world):
    """every line at every N carries weak_256MiB_value (=
    value) and strong_1GiB_value, each with its own roofline, and
    config.readings says which is which; `scaling` is "weak" at every N (the
    headline is the same reading at every N)."""
    n = 67_108_864
    hl = _reading("weak_256MiB", 0, world, n, 20 * 0.0825e-3, 0.0818)
    sn = 268_435_456 // world
    st = _reading("strong_1GiB", 268_435_456, world, sn, 200 * 0.0825e-3 * sn / n, 0.0818 * sn / n, steps=200)
    r = bench.readings(hl, st, world, 4, 256)
    assert set(r) == {"weak_256MiB_value", "weak_256MiB", "strong_1GiB_value", "strong_1GiB", "readings"}
    assert set(r["readings"]) == {"value", "weak_256MiB_value", "strong_1GiB_value"}
    w, s = r["weak_256MiB"], r["strong_1GiB"]
    assert w["scaling"] == "weak" and s["scaling"] == "strong" and w["n_gpus"] == s["n_gpus"] == world
    assert r["weak_256MiB_value"] == w["value"] and r["strong_1GiB_value"] == s["value"]
    # weak: world x (8n + B) per step; strong: the whole 1 GiB job per step
    assert abs(w["value"] - world * (8 * n + n // 256) / 0.0825e-3 / 1e9) < 0.01
    assert abs(s["value"] - (8 * 268_435_456 + 268_435_456 // 256) / (0.0825e-3 * sn / n) / 1e9) < 0.5
    for blk in (w, s):
        rf = blk["roofline"]
        assert rf["bound"] == "hbm" and rf["peak"] == bench.HBM_PEAK_GBPS and rf["unit"] == "GB/s"
        assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 and 0.7 < rf["frac"] < 1.0
    assert s["job_numel"] == 268_435_456 and s["numel_per_gpu"] == sn and s["steps"] == 200
    # the strong reading skipped (--job-numel 0): the key is still there, null
    r0 = bench.readings(hl, None, world, 4, 256)
    assert r0["strong_1GiB_value"] is None and "strong_1GiB" not in r0


def test_rehearsal_fields_are_labelled_not_measured():
    """when the ranks share one GPU no fraction of the xGMI
    bound is reported (null, with a note), and phases say they timed the TCP
    net; on a node (rehearsal None) the fields are untouched."""
    def res():
        return {"switchsim": {"frac_of_xgmi_bound": 2.10, "busbw_GBps": 300.0, "phases_ms": {"payload_sum": 208.0}},
                "xgmi_switch": {"frac_of_xgmi_bound": 1.91},
                "rccl_fp32_allreduce": {"frac_of_xgmi_bound": 0.4},
                "p2p_switch": {"error": "boom"}}
    r = bench.label_rehearsal(res(), "ranks share one GPU: RCCL")
    for k in ("switchsim", "xgmi_switch", "rccl_fp32_allreduce"):
        assert r[k]["frac_of_xgmi_bound"] is None and "rehearsal" in r[k]["rehearsal_note"]
    assert "TCP net" in r["switchsim"]["phases_note"] and "phases_note" not in r["xgmi_switch"]
    assert r["p2p_switch"] == {"error": "boom"}
    assert bench.label_rehearsal(res(), None) == res()


def test_roofline_traffic_covers_the_n_gt1_slices():
    """The N > 1 lines' roofline.traffic: profiles/pmc_traffic.json holds
    K1's PMC bytes per launch at the headline bucket and at configs[3]'s
    per-GPU FIFO slices for N = 2 / 8 (N = 4's slice is the headline
    bucket), each within 0.1 % of the algorithmic bytes."""
    for n in (67_108_864, 268_435_456, 134_217_728, 33_554_432):   # headline; strong slices at N = 1, 2, 8
        t = bench.load_traffic(n, 256, "quantize_pack_cold")
        assert t is not None, n
        alg = 8 * n + n // 256
        assert abs(t / alg - 1) < 1e-3, (n, t / alg)
    assert bench.load_traffic(12345, 256, "quantize_pack_cold") is None


def _scale_report():
    import importlib.util
    spec = importlib.util.spec_from_file_location("scale_report", os.path.join(ROOT, "tools", "scale_report.py"))
    sr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sr)
    return sr


def test_scale_report_tabulates_bench_lines(tmp_path):
    """tools/scale_report.py finds bench lines in JSON files and text logs and
    tabulates them (used on the driver's scaling run)."""
    sr = _scale_report()
    one = {"metric": "m", "n_gpus": 1, "value": 6500.0, "roofline": {"frac": 0.82}, "ms_per_step": 0.082,
           "self_check": True, "scaling": "weak", "weak_256MiB_value": 6500.0, "strong_1GiB_value": 6700.0,
           "strong_1GiB": {"roofline": {"frac": 0.84}, "self_check": True}}
    two = {"metric": "m", "n_gpus": 2, "value": 12000.0, "roofline": {"frac": 0.8}, "ms_per_step": 0.09,
           "self_check": True, "scaling": "weak", "weak_256MiB_value": 12000.0, "strong_1GiB_value": 13000.0,
           "strong_1GiB": {"roofline": {"frac": 0.81}, "self_check": True},
           "switchsim": {"ms_per_allreduce": 5.0, "busbw_GBps": 200.0, "frac_of_xgmi_bound": 0.4, "verified": True,
                         "phases_ms": {"k2": 0.1, "payload_sum": 4.0}}}
    (tmp_path / "scale.json").write_text(json.dumps({"runs": [two, one]}))
    (tmp_path / "log.txt").write_text("banner\nrank0 " + json.dumps(two) + "\n")
    got = list(sr.load(str(tmp_path / "scale.json"))) + list(sr.load(str(tmp_path / "log.txt")))
    assert [b["n_gpus"] for b in got] == [2, 1, 2]
    rep = sr.report(got[:2])
    assert "| 2 | switchsim | 5.000 |" in rep and "payload_sum 4.00" in rep
    assert "| 2 | 0.923 | 0.923 | 0.970 |" in rep      # 12000 / (2 x 6500) twice; 13000 / (2 x 6700)


def test_scale_report_efficiency_is_per_reading():
    """each reading's efficiency is against the SAME reading at
    N = 1 — a strong 1 GiB rate is never divided by the weak 256 MiB rate."""
    sr = _scale_report()
    mk = lambda n, w, s: {"metric": "m", "n_gpus": n, "value": w, "weak_256MiB_value": w,  # noqa: E731
                          "strong_1GiB_value": s}
    lines = [mk(1, 6500.0, 6700.0), mk(2, 13000.0, 13400.0), mk(4, 25350.0, 24120.0), mk(8, 51350.0, 42880.0)]
    eff = sr.efficiency(lines)
    assert eff["value"] == eff["weak_256MiB_value"]
    assert [round(eff["weak_256MiB_value"][n], 4) for n in (1, 2, 4, 8)] == [1.0, 1.0, 0.975, 0.9875]
    assert [round(eff["strong_1GiB_value"][n], 4) for n in (1, 2, 4, 8)] == [1.0, 1.0, 0.9, 0.8]
    # an N = 1 line without the strong reading: no strong efficiency at all (not a mixed one)
    lines[0]["strong_1GiB_value"] = None
    assert sr.efficiency(lines)["strong_1GiB_value"] == {}
    assert sr.efficiency(lines[1:]) == {"value": {}, "weak_256MiB_value": {}, "strong_1GiB_value": {}}


def test_term_guard_prints_the_line_when_the_launcher_stops_the_ranks(tmp_path):
    """N > 1 (first contact): torch.distributed.run SIGTERMs every
    rank once one rank fails; bench.term_guard takes the signal on its own
    thread while the main thread is blocked (here in a sleep, on a node in a
    collective or a device sync), prints rank 0's line once and exits 1.
    Before the line exists (on_term["emit"] unset) it just exits 1."""
    import subprocess
    prog = tmp_path / "p.py"
    prog.write_text(
        "import os, sys, threading, time, signal\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        "on = {'emit': None}\n"
        "bench.term_guard(on)\n"
        "if sys.argv[1] == 'line':\n"
        "    on['emit'] = lambda: print('{\"metric\": \"m\", \"terminated\": true}', flush=True)\n"
        "threading.Timer(0.5, lambda: os.kill(os.getpid(), signal.SIGTERM)).start()\n"
        "time.sleep(30)\n"
        "print('not reached', flush=True)\n")
    for mode, want in (("line", '{"metric": "m", "terminated": true}'), ("early", "")):
        p = subprocess.run([sys.executable, str(prog), mode], capture_output=True, text=True, timeout=60)
        assert p.returncode == 1, (p.returncode, p.stderr[-500:])
        assert p.stdout.strip() == want, p.stdout
