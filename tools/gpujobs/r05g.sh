# round 5, job g: what each hipIpc failure path returns (printed by the test).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_switchsim_dist.py -k ipc_failure > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "hipIpc failure" $OUT/tests.log; tail -2 $OUT/tests.log
