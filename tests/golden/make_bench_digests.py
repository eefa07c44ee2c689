"""Generate tests/golden/digests_bench.json — SHA-256 of the planes bench.py's
timed K1 launches must leave (bind the timed kernel
instance to parity inside the bench).

bench.py fills its buckets with `bench_bucket` (a torch restatement of
O.splitmix_grad over the GLOBAL element index, so a rank's FIFO slice of a
job holds exactly that slice of the job) and, after the timed region, hashes
every bucket's exponent plane and big-endian payload plane and compares them
with these digests, made here by the C oracle:

  bucket_T1   the headline (weak_256MiB) at every N: 4 buckets (seeds
              4242..4245) of 67,108,864 elements (256 MiB), one slice,
              P = 256, W = 1 — every GPU holds its own copy of the same 4
  job_T{G}    the strong_1GiB reading at N = G (G = 1 included: the whole job
              on one GPU): configs[3]'s 1 GiB job (268,435,456 elements) of each
              seed split by the FIFO rule into G slices (fifo_scheduler.cc:
              93-109); slice g = rank g's bucket

Run: python tests/golden/make_bench_digests.py   (~2 min, ~12 GiB of RAM)
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SEED0 = 4242
BUCKETS = 4
P = 256
BUCKET_NUMEL = 67_108_864
JOB_NUMEL = 268_435_456
JOB_SLICES = (1, 2, 4, 8)


def planes_digest(x, P):
    e = O.exponents(x, P)
    q = O.quantize(x, P, 1)
    return {"exps": hashlib.sha256(e.tobytes()).hexdigest(), "payload": hashlib.sha256(q.tobytes()).hexdigest()}


def main():
    out = {"generator": "splitmix_grad(seed, global element index)", "seed0": SEED0, "buckets": BUCKETS,
           "packet_numel": P, "num_workers": 1, "bucket_numel": BUCKET_NUMEL, "job_numel": JOB_NUMEL,
           "bucket_T1": [], "job": {}}
    for b in range(BUCKETS):
        x = O.splitmix_grad(SEED0 + b, BUCKET_NUMEL)
        out["bucket_T1"].append(planes_digest(x, P))
        print("bucket", b, out["bucket_T1"][-1]["payload"][:16], flush=True)
        del x
    for G in JOB_SLICES:
        out["job"][f"T{G}"] = [[None] * G for _ in range(BUCKETS)]
    for b in range(BUCKETS):
        x = O.splitmix_grad(SEED0 + b, JOB_NUMEL)
        for G in JOB_SLICES:
            for g in range(G):
                off, n = O.slice_geometry(JOB_NUMEL, G, g)
                out["job"][f"T{G}"][b][g] = planes_digest(x[off:off + n], P)
            print("job", b, G, out["job"][f"T{G}"][b][0]["payload"][:16], flush=True)
        del x
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "digests_bench.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
