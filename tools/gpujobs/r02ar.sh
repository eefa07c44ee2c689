set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ar
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_batch_gpu.py tests/test_client_gpu.py tests/test_collnet_plugin.py tests/test_client_property_gpu.py > $OUT/tests.log 2>&1 || exit 1
for T in 1 4; do for n in 256 6553600; do for se in 1 10 100; do timeout -k 10 100 p4app-switchml_amd/bin/allreduce_benchmark --tensor-numel $n --tensor-type float --num-workers 8 --num-worker-threads $T --bandwidth 0 --device gpu --mode fused --batch-jobs 16 --num-jobs 200 --num-warmup-jobs 20 --sync-every $se --inplace false --verify true > $OUT/n${n}_T${T}_sync$se.log 2>&1 || exit 1; done; done; done
timeout -k 10 200 python -c "
import sys, json, torch; sys.path[:0]=['.', 'p4app-switchml_amd']
import bench
print(json.dumps(bench.plugin_buckets(torch, torch.device('cuda:0'))))" > $OUT/plugin.json 2> $OUT/plugin.err
