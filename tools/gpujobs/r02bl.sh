set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bl
mkdir -p $OUT
timeout -k 10 200 python tools/ab_frames.py tools/ab/tx_base.so tools/ab/tx_bf.so > $OUT/ab_tx.json 2> $OUT/ab_tx.err
