set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aq
mkdir -p $OUT
for bj in 16 0; do for T in 1 4; do for n in 256 6553600; do timeout -k 10 100 p4app-switchml_amd/bin/allreduce_benchmark --tensor-numel $n --tensor-type float --num-workers 8 --num-worker-threads $T --bandwidth 0 --device gpu --mode fused --batch-jobs $bj --num-jobs 200 --num-warmup-jobs 20 --sync-every 100 --inplace false --verify true > $OUT/n${n}_bj${bj}_T${T}.log 2>&1 || exit 1; done; done; done
