# round 3, job t: rocprofv3 kernel trace of packet mode (exchange bursts):
# per-launch kernel time vs the per-pass wall time (launch-bound evidence).
set -uo pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r03t
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
EXE=$ROOT/p4app-switchml_amd/bin/allreduce_benchmark
ARGS="--tensor-numel 16777216 --tensor-type float --num-workers 2 --num-worker-threads 4 --bandwidth 0 --device gpu --mode packet --num-jobs 5 --num-warmup-jobs 2 --verify true"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $EXE $ARGS > $OUT/kt.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -E "Duration|verified" $OUT/kt.log | tail -4
find $OUT/kt -name "*kernel_stats.csv" | head -2
