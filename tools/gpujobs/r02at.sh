set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02at
mkdir -p $OUT
timeout -k 10 300 python tools/ab_rx_stride.py > $OUT/stride.json 2> $OUT/stride.err
