# round 3, job q: the N>1 path rehearsed on one GPU at the driver's own
# switch size (2 ranks, 1 GiB per worker: 4 in-node-switch chunks per call),
# and 8 ranks at 64 MiB per worker.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03q
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 550 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
  > $OUT/rehearse_2_full.json 2> $OUT/rehearse_2_full.err
rc=$?; echo "rehearse 2 full rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 550 python -u bench.py --gpus 8 --switch-numel 16777216 --steps 20 --warmup 5 \
  > $OUT/rehearse_8_64MiB.json 2> $OUT/rehearse_8_64MiB.err
rc=$?; echo "rehearse 8 rc=$rc"
