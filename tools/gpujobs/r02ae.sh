set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ae
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 > $OUT/bench2.json 2> $OUT/bench2.err && \
timeout -k 10 300 python tools/ab_cold.py bin/ab/k1_base.so bin/ab/k1_ntstore.so > $OUT/ab_cold.json 2> $OUT/ab_cold.err
