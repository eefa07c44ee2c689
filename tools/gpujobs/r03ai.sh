# round 3, job ai: the whole GPU suite on the final tree (push multicast, guarded bench),
# smoke, the driver's N=1 bench command, and a 2-rank rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03ai
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
head -c 400 $OUT/bench.json; echo
SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_2.json 2> $OUT/rehearse_2.err
rc=$?; echo "rehearse 2 rc=$rc"
