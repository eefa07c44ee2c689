# round 3, job i: RCCL over the SwitchML net with the CollNet table declined
# (GPU test), then the driver's N=1 bench command (cycling buckets, digest
# self-check, rccl_collnet field).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_rccl_collnet.py \
  > $OUT/test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 $OUT/test.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
tail -c 3000 $OUT/bench.json
