set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bt
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_args.json 2> $OUT/bench.err
