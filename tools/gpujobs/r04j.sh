# round 4, job j: frames rx apply with non-temporal output stores past the
# threshold — rx tests, then the cold A/B (tools/ab_rx_nt.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_frames_rx.py \
  tests/test_frames.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/ab_rx_nt.py > $OUT/ab_rx_nt.json 2> $OUT/ab_rx_nt.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_rx_nt.json
