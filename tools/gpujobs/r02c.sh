set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 200 python tools/ab_k3b.py tools/ab/k3_base.so tools/ab/k3_const.so > $OUT/ab_k3b.json 2> $OUT/ab_k3b.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_client_gpu.py > $OUT/tests_client.log 2>&1
