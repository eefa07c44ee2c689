set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aa
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 500 python bench.py --gpus 8 --switch-numel 4194304 --steps 20 --warmup 20 > $OUT/bench8.json 2> $OUT/bench8.err
echo "rc=$?" >> $OUT/bench8.err
