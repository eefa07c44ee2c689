# round 3, job k: the whole GPU suite after the round's changes, then the
# driver's N=1 bench command (64 MiB non-temporal threshold).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
head -c 1500 $OUT/bench.json
