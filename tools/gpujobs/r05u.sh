# round 5, job u: bench.py --extra on the final tree (every kernel's rate,
# H<->D-inclusive rates, frames FLOAT32 + INT32, K6, configs[4] through the plugin).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet > $OUT/bench_extra.json 2> $OUT/bench_extra.err
rc=$?; echo "bench extra rc=$rc"; tail -c 3000 $OUT/bench_extra.json
