set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_frames_rx.py tests/test_frames.py tests/test_golden_digests.py > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python tools/ab_rx.py tools/ab/k3_new.so tools/ab/rx_fold.so > $OUT/ab_rx_inorder.json 2> $OUT/ab_rx.err && \
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py tools/ab/k3_new.so tools/ab/rx_fold.so > $OUT/ab_rx_shuffled.json 2>> $OUT/ab_rx.err
