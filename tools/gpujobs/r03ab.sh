# round 3, job ab: per-burst latency, launch + sync vs the burst server.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03ab
mkdir -p $OUT
timeout -k 10 300 python -u tools/burst_latency.py $OUT/burst_latency.json > $OUT/lat.log 2>&1
rc=$?; echo "lat rc=$rc"; tail -16 $OUT/lat.log
