set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02u
mkdir -p $OUT
AB_NOCHECK=1 timeout -k 10 200 python tools/ab_rx.py bin/ab/rx_old.so bin/ab/rx_fast3.so bin/ab/rx_diag1.so bin/ab/rx_diag2.so > $OUT/ab.json 2> $OUT/ab.err
