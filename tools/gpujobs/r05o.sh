# round 5, job o: K1 per GPU at configs[3]'s N = 2 / 8 FIFO slice sizes
# (512 / 128 MiB buckets, 4 cycled), the one-GPU view of the strong-scaling
# headline's per-rank work; the driver's step count and a long one.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05o
mkdir -p $OUT
for SN in 134217728 33554432; do
  for K in 20 200; do
    timeout -k 10 300 python3 -u bench.py --numel $SN --steps $K --warmup 5 --no-cpu-baseline --no-side --no-rccl-collnet > $OUT/slice_${SN}_k$K.json 2> $OUT/slice_${SN}_k$K.err || exit $?
    python3 -c "import json; d=json.loads(open('$OUT/slice_${SN}_k$K.json').read().strip().splitlines()[-1]); print('$SN', 'K=$K', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['self_check'])"
  done
done
