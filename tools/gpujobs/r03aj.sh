# round 3, job aj: rocprofv3 evidence on the final tree (kernel trace over the
# bench's timed window, PMC traffic passes, frames kernels) and the driver's
# N=1 bench command on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03aj
mkdir -p $OUT
bash profiles/run_profiles.sh r03 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
head -c 300 $OUT/bench.json
