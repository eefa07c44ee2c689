set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bu
mkdir -p $OUT
timeout -k 10 200 python tools/ab_rx.py tools/ab/tx_base.so tools/ab/rx_ntout.so > $OUT/ab_rx.json 2> $OUT/ab_rx.err || exit $?
AB_SHUFFLE=64 timeout -k 10 200 python tools/ab_rx.py tools/ab/tx_base.so tools/ab/rx_ntout.so > $OUT/ab_rx_shuffled.json 2> $OUT/ab_rx_sh.err
