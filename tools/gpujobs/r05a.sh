# round 5, job a: the new N=2 bench test alone (timing), then the multi-process
# tests touched this round (FileStore rendezvous, bounded p2p waits, setup
# failure agreement), then the whole GPU suite once.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_bench_multi_gpu.py > $OUT/bench_n2_test.log 2>&1
rc=$?; echo "bench n2 test rc=$rc"; tail -3 $OUT/bench_n2_test.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_switchsim_dist.py tests/test_switch_rccl_gpu.py > $OUT/mp_tests.log 2>&1
rc=$?; echo "mp tests rc=$rc"; tail -3 $OUT/mp_tests.log
