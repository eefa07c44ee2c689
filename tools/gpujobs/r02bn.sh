set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bn
mkdir -p $OUT
AB_MIB=192,256,288,320,384,448 timeout -k 10 300 python tools/ab_store_size.py tools/ab/tx_base.so tools/ab/k1_ntstore.so > $OUT/ab_store_size.json 2> $OUT/ab.err
