# round 5, job h: bounded device waits in the native in-node switch — its
# tests, the client / plugin suites that run over it, and the N=2 bench test.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xgmi_switch.py tests/test_client_gpu.py tests/test_collnet_plugin.py tests/test_bench_multi_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
