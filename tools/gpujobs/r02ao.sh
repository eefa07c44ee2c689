set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02ao
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_batch.py > $OUT/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_batch.py > $OUT/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_batch.py > $OUT/write.log 2>&1 && \
cd $GRAFT_REPO_ROOT && SML_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 > $OUT/bench2.json 2> $OUT/bench2.err
