set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aj
mkdir -p $OUT
timeout -k 10 120 ./bin/ptr_attr_cost > $OUT/cost.json 2> $OUT/cost.err
