set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02z
mkdir -p $OUT
timeout -k 10 300 python tools/zero_copy_streams.py > $OUT/zcs.json 2> $OUT/zcs.err
