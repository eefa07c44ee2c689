set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 200 python tools/ab_k3b.py tools/ab/k3_old.so tools/ab/k3_new.so > $OUT/ab_k3_waitcnt.json 2> $OUT/ab.err && \
timeout -k 10 200 python tools/ab_rx.py tools/ab/k3_old.so tools/ab/k3_new.so > $OUT/ab_rx_inorder.json 2> $OUT/ab_rx.err && \
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py tools/ab/k3_old.so tools/ab/k3_new.so > $OUT/ab_rx_shuffled.json 2>> $OUT/ab_rx.err && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_launch_geometry.py tests/test_property_gpu.py tests/test_kat_gpu.py tests/test_golden_digests.py tests/test_frames.py tests/test_frames_rx.py > $OUT/tests.log 2>&1
