# round 5, job w: bench.py --extra's frames rx fields and the interleaved
# A/B tool on the same box (is bench's rx figure box variance or method?)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05w
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python3 -u tools/ab_rx_libs_cold.py p4app-switchml_amd/bin/ab/cur.so p4app-switchml_amd/bin/ab/ntclaim.so > $OUT/ab.json 2> $OUT/ab.err || exit $?
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/r05w/bench.json").read().strip().splitlines()[-1])
e = b.get("extra", {})
print({k: v for k, v in e.items() if "frames" in k})
print(json.load(open("gpurun_out/r05w/ab.json"))["bench_style_us"])
PY
