set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ba
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_launch_geometry.py tests/test_gpu_parity.py tests/test_kat_gpu.py > $OUT/tests_quick.log 2>&1 && \
timeout -k 10 300 python tools/sweep_cold.py > $OUT/sweep_p256.json 2> $OUT/sweep_p256.err && \
SWEEP_P=64 timeout -k 10 300 python tools/sweep_cold.py > $OUT/sweep_p64.json 2> $OUT/sweep_p64.err && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
