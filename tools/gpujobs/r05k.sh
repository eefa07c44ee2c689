# round 5, job k: the whole GPU suite on the current tree, smoke, the
# driver's N=1 command and the N=2 rehearsal at the driver's defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${JOB:-r05k}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_rehearse_2.json 2> $OUT/bench_rehearse_2.err
rc=$?; echo "rehearse 2 rc=$rc"
