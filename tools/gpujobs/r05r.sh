# round 5, job r: DPDK frames for INT32 job slices (sml_pack_frames_int32 /
# sml_unpack_frames_int32) against the oracle, and the FLOAT32 frames suites
# on the same build (their kernels are unchanged instruction for instruction).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_frames_int32.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
