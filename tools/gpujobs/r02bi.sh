set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bi
mkdir -p $OUT
timeout -k 10 300 python tools/ab_switch.py tools/ab/tx_base.so tools/ab/sw_w8.so > $OUT/ab_switch.json 2> $OUT/ab_switch.err
