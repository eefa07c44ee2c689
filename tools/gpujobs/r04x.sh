# round 4, job x: the reference's allreduce_benchmark program on the final
# client + kernels: 256 MiB device jobs in fused / bulk modes (T = 1 / 4,
# batched dispatch), 25 MiB W = 8 jobs, 64 MiB W = 2 packet / bulk / fused.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04x
mkdir -p $OUT
B=p4app-switchml_amd/bin/allreduce_benchmark
for m in fused bulk; do for T in 1 4; do
  timeout -k 10 100 $B --tensor-numel 67108864 --tensor-type float --num-workers 1 --num-worker-threads $T --bandwidth 0 \
    --device gpu --mode $m --num-jobs 30 --num-warmup-jobs 5 --verify true > $OUT/ab256_${m}_T${T}.log 2>&1 || exit 1
done; done
for T in 1 4; do for se in 1 10; do
  timeout -k 10 100 $B --tensor-numel 6553600 --tensor-type float --num-workers 8 --num-worker-threads $T --bandwidth 0 \
    --device gpu --mode fused --num-jobs 40 --num-warmup-jobs 5 --sync-every $se --inplace false --verify true \
    > $OUT/ab25_T${T}_sync$se.log 2>&1 || exit 1
done; done
for m in packet bulk fused; do
  timeout -k 10 200 $B --tensor-numel 16777216 --tensor-type float --num-workers 2 --num-worker-threads 4 --bandwidth 0 \
    --device gpu --mode $m --num-jobs 5 --num-warmup-jobs 2 --verify true > $OUT/allreduce_benchmark_64MiB_$m.log 2>&1 || exit 1
done
echo done
