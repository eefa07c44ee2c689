set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 && \
AB_COUNTS=1 timeout -k 10 200 python tools/ab_rx.py tools/ab/rx_fold.so tools/ab/rx_cnt.so > $OUT/ab_rx_inorder.json 2> $OUT/ab_rx.err && \
AB_COUNTS=1 AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py tools/ab/rx_fold.so tools/ab/rx_cnt.so > $OUT/ab_rx_shuffled.json 2>> $OUT/ab_rx.err
