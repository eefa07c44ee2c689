set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ai
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_batch_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_batch.py > $OUT/ab_batch.json 2> $OUT/ab_batch.err || exit 1
for rep in 1 2; do for bj in 16 0; do for T in 1 4; do timeout -k 10 100 p4app-switchml_amd/bin/allreduce_benchmark --tensor-numel 67108864 --tensor-type float --num-workers 1 --num-worker-threads $T --bandwidth 0 --device gpu --mode fused --batch-jobs $bj --num-jobs 30 --num-warmup-jobs 5 --verify true > $OUT/ab256_bj${bj}_T${T}_r$rep.log 2>&1 || exit 1; done; done; done
