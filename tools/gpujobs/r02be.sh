set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02be
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_switch_gpu.py tests/test_xgmi_switch.py > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/ab_copy_segments.py > $OUT/ab_copy_segments.json 2> $OUT/ab.err || exit $?
SML_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 3 --switch-numel 4194305 --steps 20 --warmup 5 --no-side > $OUT/rehearse3.json 2> $OUT/rehearse3.err
