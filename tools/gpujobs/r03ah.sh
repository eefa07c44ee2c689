# round 3, job ah: bench with guarded side fields (N=1 driver command) and
# the 2-rank rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03ah
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
head -c 300 $OUT/bench.json; echo
SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_2.json 2> $OUT/rehearse_2.err
rc=$?; echo "rehearse 2 rc=$rc"
