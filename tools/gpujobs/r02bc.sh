set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bc
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_args.json 2> $OUT/bench_driver_args.err || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 1800 bash profiles/run_profiles.sh r02c > $OUT/prof.log 2>&1
