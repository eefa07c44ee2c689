set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bj
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_frames.py tests/test_frames_rx.py tests/test_golden_digests.py tests/test_launch_geometry.py tests/test_large_gpu.py > $OUT/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/fr_kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_frames.py > $GRAFT_REPO_ROOT/$OUT/prof_frames.log 2>&1
