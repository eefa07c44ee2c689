# round 5, job aa: rocprofv3 kernel trace of bench.py --extra (the frames
# kernels incl. the one-pass INT32 rx k_rx_int32 + k_rx_int32_fixup)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05aa
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet --no-side > $OUT/bench.json 2> $OUT/bench.err || exit $?
find $OUT/prof -name "*kernel_stats.csv" | head -3
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05aa/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "rx" in r["Name"] or "frames" in r["Name"]:
        print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
