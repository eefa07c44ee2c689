set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02v
mkdir -p $OUT
timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_fu4.so bin/ab/rx_fu8.so > $OUT/ab.json 2> $OUT/ab.err && \
AB_NOCHECK=1 timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_diag1.so bin/ab/rx_fu8_diag1.so > $OUT/ab_diag.json 2> $OUT/ab_diag.err
