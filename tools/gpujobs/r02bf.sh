set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bf
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xgmi_switch.py > $OUT/tests.log 2>&1 || exit $?
SML_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 3 --switch-numel 70000000 --steps 20 --warmup 5 --no-side --no-plugin > $OUT/rehearse3_2chunks.json 2> $OUT/rehearse3.err
