# round 5, job s: device uint8 buckets through the CollNet plugin table, the
# plugin suites, and the INT32 frames / RDMA tests of this round's tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_collnet_plugin.py tests/test_rccl_collnet.py tests/test_xgmi_switch.py tests/test_frames_int32.py tests/test_frames.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
