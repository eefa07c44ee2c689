"""Generate tests/golden/digests.json — SHA-256 digests of the oracle's
planes at the full BASELINE sizes ("SHA-256 of (BE payload
plane, exponent plane, dequant output) for 64 MiB and 256 MiB").

The GPU tests (tests/test_golden_digests.py) recompute the same planes with
the HIP kernels and compare digests, so the full-size configurations are
pinned bit for bit without the oracle on the GPU box; the CPU tests recompute
them with the oracle to keep the fixture and the oracle in step.

Inputs are integer-exact generators (identical bytes on every host):
  randbits  the reference's own random-float recipe on glibc rand()
            (allreduce_benchmark/main.cc:197-205), O.c_ref_random_floats
  pattern   float(i) * (-1)^i (allreduce_benchmark/main.cc:207-212)
  grad      O.splitmix_grad: 24-bit mantissas scaled by 2^-(24..39)

Planes per slice (FIFO slices of fifo_scheduler.cc:93-109; blocks restart
at every slice start): exps (int8[B]), payload (BE int32[B*P] = wire bytes),
out = dequantize(loopback_xW(payload), exps) (float32[numel]).  Digests run
over the slices in order.  NaN outputs — the 0/0 of a zero scale, when
W * 2^e overflows float (e = 127, W >= 2) — are canonicalized to 0x7fc00000
before hashing: x86 divides to the negative default NaN 0xffc00000, gfx950
to the positive one; that sign is the one non-bit-exact case.

Run: python tests/golden/make_digests.py   (rewrites digests.json,
digests_ext.json and digests_switch.json, ~2 min; --ext-only rewrites only
digests_ext.json, --switch-only digests_ext.json and digests_switch.json)
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

CASES = [
    # name, generator, seed, numel, P, W, T
    ("cfg2_randbits_T1", "randbits", 1, 16_777_216, 256, 1, 1),
    ("cfg2_grad_T4", "grad", 42, 16_777_216, 256, 1, 4),
    ("cfg2_pattern_W2", "pattern", 0, 16_777_216, 256, 2, 1),
    ("cfg3_grad_W2", "grad", 43, 67_108_864, 256, 2, 1),
    ("cfg3_randbits_W8_T4", "randbits", 7, 67_108_864, 256, 8, 4),
    ("rdma_grad_P1024_W3", "grad", 44, 16_777_216 + 1000, 1024, 3, 1),
    # configs[3]: the 1 GiB job (allreduce_benchmark's default tensor-numel,
    # main.cc:101) split into 8 FIFO slices, slice g = GPU g's shard
    ("cfg3_job_1GiB_randbits_T8", "randbits", 11, 268_435_456, 256, 1, 8),
]

# configs[3]'s switch simulation: W = 8 workers, each with its own 64 MiB
# bucket (rank r: generator seed + r, scaled by 2^(r % 4 - 1) so the per-block
# exponents differ between workers).  The switch (p4/exponents.p4:48-54 signed
# int8 max, p4/processor.p4:48-54 wrapping bit<32> sum) sees every worker's
# packets; digests of the global exponent plane, the aggregated BE payload
# plane and the dequantized sum every worker ends with.
SWITCH_CASES = [
    # name, generator, seed, numel per worker, P, W
    ("cfg3_switch_W8_grad_64MiB", "grad", 60, 16_777_216, 256, 8),
]


def make_input(gen, seed, n):
    if gen == "randbits":
        return O.c_ref_random_floats(seed, n)
    if gen == "pattern":
        return O.ref_pattern_floats(n)
    if gen == "grad":
        return O.splitmix_grad(seed, n)
    raise ValueError(gen)


def switch_input(gen, seed, rank, n):
    import numpy as np
    return make_input(gen, seed + rank, n) * np.float32(2.0 ** (rank % 4 - 1))


def oracle_switch_digests(gen, seed, numel, P, W):
    xs = [switch_input(gen, seed, r, numel) for r in range(W)]
    h = {k: hashlib.sha256() for k in ("inputs", "global_exps", "payload", "out")}
    for x in xs:
        h["inputs"].update(x.tobytes())
    g = O.switch_exps([O.exponents(x, P) for x in xs])
    agg = O.switch_payload([O.quantize(x, P, W, global_exps=g) for x in xs])
    out = O.dequantize(agg, g, numel, P, W)
    h["global_exps"].update(g.tobytes())
    h["payload"].update(agg.tobytes())
    h["out"].update(canonical_nan(out).tobytes())
    return {k: v.hexdigest() for k, v in h.items()}


def canonical_nan(out):
    import numpy as np
    b = out.view(np.uint32).copy()
    b[np.isnan(out)] = 0x7FC00000
    return b


def oracle_digests(gen, seed, numel, P, W, T):
    x = make_input(gen, seed, numel)
    h = {k: hashlib.sha256() for k in ("input", "exps", "payload", "out")}
    h["input"].update(x.tobytes())
    for t in range(T):
        off, n = O.slice_geometry(numel, T, t)
        if n == 0:
            continue
        xs = x[off:off + n]
        e = O.exponents(xs, P)
        q = O.quantize(xs, P, W)
        out = O.dequantize(O.loopback_aggregate(q, W), e, n, P, W)
        h["exps"].update(e.tobytes())
        h["payload"].update(q.tobytes())
        h["out"].update(canonical_nan(out).tobytes())
    return {k: v.hexdigest() for k, v in h.items()}


# Full-size cases for the (f) data formats and the VCL=1 rounding mode:
#   frames  DPDK frames of the whole slice (BuildPacket + PreprocessSingle for
#           every packet, dpdk_worker_thread_utils.inc:67-135), stride 1076,
#           frame params = switchml_amd.frame_params(job_id, pool_start,
#           pool_shift, max_outstanding_pkts)
#   rne     payload plane of the VCL=1 build (RNE body, scalar tail;
#           parity unpinned: VCL is not in the reference tree)
EXT_CASES = [
    # name, kind, generator, seed, numel, P, W, extra
    ("cfg2_frames_grad", "frames", "grad", 45, 16_777_216, 256, 1,
     {"batch_max": 64, "job_id": 5, "pool_index_start": 3, "pool_index_shift": 7, "max_outstanding_pkts": 64}),
    ("frames_P64_W2_ragged", "frames", "randbits", 9, 4_000_037, 64, 2,
     {"batch_max": 100, "job_id": 1, "pool_index_start": 0, "pool_index_shift": 0, "max_outstanding_pkts": 50}),
    ("cfg2_rne_grad_W3", "rne", "grad", 46, 16_777_216 + 77, 256, 3, {}),
]


def frame_params(extra):
    sys.path.insert(0, os.path.join(ROOT, "p4app-switchml_amd"))
    import switchml_amd as sw  # the ctypes struct only; no GPU library call
    return sw.frame_params(job_id=extra["job_id"], pool_index_start=extra["pool_index_start"],
                           pool_index_shift=extra["pool_index_shift"],
                           max_outstanding_pkts=extra["max_outstanding_pkts"])


def oracle_ext_digest(kind, gen, seed, numel, P, W, extra):
    x = make_input(gen, seed, numel)
    if kind == "frames":
        fr = O.build_frames(x, frame_params(extra), P, W, batch_max=extra["batch_max"])
        return hashlib.sha256(fr.tobytes()).hexdigest()
    if kind == "rne":
        return hashlib.sha256(O.quantize(x, P, W, rounding=O.RNE_VCL).tobytes()).hexdigest()
    raise ValueError(kind)


def main():
    ext = {}
    for name, kind, gen, seed, numel, P, W, extra in EXT_CASES:
        ext[name] = {"kind": kind, "gen": gen, "seed": seed, "numel": numel, "packet_numel": P,
                     "num_workers": W, "extra": extra,
                     "sha256": oracle_ext_digest(kind, gen, seed, numel, P, W, extra)}
        print(name, ext[name]["sha256"][:16], flush=True)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "digests_ext.json"), "w") as f:
        json.dump(ext, f, indent=1)
        f.write("\n")
    if "--ext-only" in sys.argv:
        return
    sw_res = {}
    for name, gen, seed, numel, P, W in SWITCH_CASES:
        sw_res[name] = {"gen": gen, "seed": seed, "numel": numel, "packet_numel": P, "num_workers": W,
                        "sha256": oracle_switch_digests(gen, seed, numel, P, W)}
        print(name, sw_res[name]["sha256"]["out"][:16], flush=True)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "digests_switch.json"), "w") as f:
        json.dump(sw_res, f, indent=1)
        f.write("\n")
    if "--switch-only" in sys.argv:
        return
    res = {}
    for name, gen, seed, numel, P, W, T in CASES:
        res[name] = {"gen": gen, "seed": seed, "numel": numel, "packet_numel": P, "num_workers": W,
                     "num_slices": T, "sha256": oracle_digests(gen, seed, numel, P, W, T)}
        print(name, res[name]["sha256"]["out"][:16], flush=True)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "digests.json"), "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
