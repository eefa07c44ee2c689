set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_client_gpu.py tests/test_collnet_plugin.py tests/test_capi_gpu.py tests/test_switchsim_dist.py > $OUT/tests.log 2>&1 && \
timeout -k 10 400 python bench.py --extra --no-cpu-baseline --no-side --steps 50 --warmup 50 > $OUT/bench_extra.json 2> $OUT/bench_extra.err && \
for se in 1 10; do timeout -k 10 200 p4app-switchml_amd/bin/allreduce_benchmark --tensor-numel 6553600 --tensor-type float --num-workers 8 --num-worker-threads 4 --bandwidth 0 --device gpu --mode fused --num-jobs 40 --num-warmup-jobs 5 --sync-every $se --inplace false --verify true > $OUT/allreduce_benchmark_25MiB_sync$se.log 2>&1 || exit 1; done
