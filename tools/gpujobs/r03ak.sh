# round 3, job ak: bench --extra on the final tree (secondary kernels,
# H<->D-inclusive variants, frames, switch aggregate, configs[4] plugin).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03ak
mkdir -p $OUT
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet \
  > $OUT/bench_extra.json 2> $OUT/bench_extra.err
rc=$?; echo "bench rc=$rc"
