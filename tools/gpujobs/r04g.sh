# round 4, job g: K4 / fused round trip on 2- vs 4-slice tiles — invariance
# tests, then the A/B on the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_launch_geometry.py \
  > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
AB_KIND=stream timeout -k 10 500 python -u tools/ab_slices_nt.py > $OUT/ab_stream.json 2> $OUT/ab_stream.err
rc=$?; echo "ab rc=$rc"
