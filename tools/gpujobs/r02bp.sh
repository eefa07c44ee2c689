set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bp
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_launch_geometry.py tests/test_gpu_parity.py tests/test_large_gpu.py tests/test_golden_digests.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab_nt_policy.py > $OUT/ab_nt_policy.json 2> $OUT/ab.err
