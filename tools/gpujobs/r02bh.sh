set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bh
mkdir -p $OUT
timeout -k 10 200 python tools/ab_frames.py tools/ab/tx_base.so tools/ab/fr_w8.so > $OUT/ab_tx.json 2> $OUT/ab_tx.err || exit $?
timeout -k 10 200 python tools/ab_rx.py tools/ab/tx_base.so tools/ab/fr_w8.so > $OUT/ab_rx.json 2> $OUT/ab_rx.err || exit $?
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py tools/ab/tx_base.so tools/ab/fr_w8.so > $OUT/ab_rx_shuffled.json 2> $OUT/ab_rx_sh.err
