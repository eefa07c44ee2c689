set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ah
mkdir -p $OUT
timeout -k 10 200 python tools/ab_batch.py > $OUT/ab_batch.json 2> $OUT/ab_batch.err
