# Full GPU suite, default bench, bench --extra (plugin configs[4], rx), RCCL plugin probe,
# per-LTU packet-mode client timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 400 python bench.py --extra --no-cpu-baseline --no-side --steps 50 --warmup 50 > $OUT/bench_extra.json 2> $OUT/bench_extra.err && \
timeout -k 10 240 python tools/rccl_plugin_probe.py 1 > $OUT/rccl_plugin_probe.json 2>&1 && \
for m in packet bulk fused; do timeout -k 10 200 p4app-switchml_amd/bin/allreduce_benchmark --tensor-numel 16777216 --tensor-type float --num-workers 2 --num-worker-threads 4 --bandwidth 0 --device gpu --mode $m --num-jobs 5 --num-warmup-jobs 2 --verify true > $OUT/allreduce_benchmark_64MiB_$m.log 2>&1 || exit 1; done
