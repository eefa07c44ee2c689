# round 3, job r: the whole GPU suite on the tree with exchange bursts, smoke,
# and the driver's N=1 bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03r
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat $OUT/smoke.log | tail -2
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
head -c 600 $OUT/bench.json
