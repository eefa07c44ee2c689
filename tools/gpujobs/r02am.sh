set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02am
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 50 --warmup 50 > $OUT/bench1.json 2> $OUT/bench1.err || exit 1
SML_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
SML_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 --exchange-timeout 2 > $OUT/bench2_wd.json 2> $OUT/bench2_wd.err
echo "watchdog run rc=$?" > $OUT/wd_rc.txt
