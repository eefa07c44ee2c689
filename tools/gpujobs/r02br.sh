set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02br
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline > $OUT/b1.json 2> $OUT/b1.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline > $OUT/b2.json 2> $OUT/b2.err || exit $?
timeout -k 10 300 python bench.py --no-side --no-cpu-baseline > $OUT/b3.json 2> $OUT/b3.err
