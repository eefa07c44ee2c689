set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frames_rx.py > $OUT/tests.log 2>&1
