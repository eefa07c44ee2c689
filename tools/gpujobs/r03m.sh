# round 3, job m (session 2): the whole GPU suite on the restored tree, the
# driver's N=1 bench command, and the N>1 path rehearsed with 2 and 8 ranks
# on one GPU after the rccl_collnet worker-environment fix (diagnostic
# fields no longer decide the exit status; rccl_collnet runs 2 workers).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
for n in 2 8; do
  SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus $n --switch-numel 4194304 --steps 20 --warmup 5 \
    > $OUT/rehearse_$n.json 2> $OUT/rehearse_$n.err
  rc=$?; echo "rehearse $n rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
