# round 3, job u: the per-GPU slice sizes of the driver's N = 2 / 4 / 8
# configs[3] runs (512 / 256 / 128 MiB of the 1 GiB job) on one GPU, with the
# headline's own settings (4 buckets cycled, 20 timed steps): the expected
# per-GPU rate of each point of the strong-scaling curve.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03u
mkdir -p $OUT
for n in 134217728 67108864 33554432; do
  timeout -k 10 300 python -u bench.py --numel $n --steps 20 --warmup 5 --no-side --no-cpu-baseline --no-rccl-collnet \
    > $OUT/slice_$n.json 2> $OUT/slice_$n.err
  rc=$?; echo "numel $n rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
