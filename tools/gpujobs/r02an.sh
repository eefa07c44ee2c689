set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02an
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 --exchange-timeout 0.05 > $OUT/bench2_wd.json 2> $OUT/bench2_wd.err
echo "watchdog run rc=$?" > $OUT/wd_rc.txt
