set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02r
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frames_rx.py tests/test_launch_geometry.py tests/test_golden_digests.py > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_fast2.so bin/ab/rx_fast1.so > $OUT/ab_inorder.json 2> $OUT/ab_inorder.err && \
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_fast2.so bin/ab/rx_fast1.so > $OUT/ab_shuffle.json 2> $OUT/ab_shuffle.err
