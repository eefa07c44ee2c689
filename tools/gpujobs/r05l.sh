# round 5, job l: the N=1 bench-line contract test.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05l
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_bench_multi_gpu.py -k n1 > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
