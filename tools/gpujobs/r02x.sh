set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02x
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frames_rx.py tests/test_launch_geometry.py > $OUT/tests.log 2>&1 && \
timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_new.so > $OUT/ab_inorder.json 2> $OUT/ab_inorder.err && \
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_new.so > $OUT/ab_shuffle.json 2> $OUT/ab_shuffle.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_frames.py > $GRAFT_REPO_ROOT/$OUT/kt.log 2>&1
