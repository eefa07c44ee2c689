# round 5, job i: backend.hip.vcl (the reference's VCL=1 rounding) through
# every Context dispatch and the in-node switch; the converted xgmi tests;
# the bounded-wait test.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_client_gpu.py tests/test_xgmi_switch.py tests/test_switchsim_dist.py -k "vcl or xgmi or wait_device" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
