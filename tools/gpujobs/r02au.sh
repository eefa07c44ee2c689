set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02au
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_large_gpu.py > $OUT/tests.log 2>&1
