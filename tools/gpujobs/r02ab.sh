set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_batch_gpu.py tests/test_client_gpu.py tests/test_collnet_plugin.py tests/test_client_property_gpu.py > $OUT/tests.log 2>&1
